set -u
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  bash scripts/ablate_run.sh r01u "uni1 wpe1" "65536 4096" --env Unicycle --hazards 3 || exit 1
  bash scripts/ablate_run.sh r01u "uni1 wpe1" "65536" || exit 1
done

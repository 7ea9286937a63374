set -u
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  bash scripts/ablate_run.sh r01af "main2 notrig noatan" "65536 4096" --env Unicycle --hazards 3 || exit 1
done

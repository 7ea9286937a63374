set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
V="$*"
bash scripts/ablate_run.sh $TAG "$V" "65536" || exit 1
bash scripts/ablate_run.sh $TAG "$V" "65536" || exit 1
bash scripts/ablate_run.sh $TAG "$V" "65536" --env Unicycle --hazards 3 || exit 1

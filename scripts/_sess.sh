set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
bash scripts/gpu_session.sh $TAG "$@" || exit $?
if [ -d build/variants ]; then bash scripts/ablate_run.sh $TAG "$(ls build/variants | sed 's/librcbf_//; s/\.so//' | tr '\n' ' ')" "65536 1048576"; fi

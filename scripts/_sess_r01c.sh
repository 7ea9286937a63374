set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_session.sh r01c pytest bench || exit $?
bash scripts/ablate_run.sh r01c "full noqp memonly" "65536 1048576"

set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
bash scripts/gpu_session.sh $TAG "$@" || exit $?
RCBF_HIP_LIB=build/variants/librcbf_stamps.so timeout -k 10 200 python scripts/stamps.py 65536 > gpurun_out/$TAG/stamps65k.log 2>&1 || exit 1
RCBF_HIP_LIB=build/variants/librcbf_stamps.so timeout -k 10 200 python scripts/stamps.py 65536 unicycle > gpurun_out/$TAG/stamps_uni.log 2>&1

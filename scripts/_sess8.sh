set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit 1
bash scripts/ablate_run.sh $TAG "early0 early1 early0 early1" "65536" || exit 1
RCBF_HIP_LIB=build/variants/librcbf_stamps.so timeout -k 10 200 python scripts/stamps.py 65536 > $OUT/stamps65k.log 2>&1

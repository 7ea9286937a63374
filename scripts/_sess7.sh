set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python scripts/pdipm_diag.py > $OUT/pdipm_diag.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --solver pdipm > $OUT/pdipm_cars.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --solver pdipm --env Unicycle > $OUT/pdipm_uni.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest.log 2>&1 || exit 1

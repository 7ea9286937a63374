set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-r01i}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_cars_$r.json 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.e-]*\|"frac": [0-9.]*' $OUT/bench_cars_$r.json | tr '\n' ' '; echo
timeout -k 10 300 python bench.py --no-cpu-baseline --env Unicycle --hazards 3 > $OUT/bench_uni_$r.json 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.e-]*\|"frac": [0-9.]*' $OUT/bench_uni_$r.json | tr '\n' ' '; echo
done

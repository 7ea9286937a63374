set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01ak; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --no-graph --steps 2000 --no-cpu-baseline > $OUT/eager.json 2>&1 || { tail -20 $OUT/eager.json; exit 1; }
tail -1 $OUT/eager.json
timeout -k 10 200 python scripts/single_env_latency.py > $OUT/latency.json 2>&1 || { tail -20 $OUT/latency.json; exit 1; }
tail -1 $OUT/latency.json

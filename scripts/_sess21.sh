set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01al; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/default.json 2>&1 || { tail -20 $OUT/default.json; exit 1; }
tail -1 $OUT/default.json
timeout -k 10 200 python bench.py --no-graph --steps 2000 --no-cpu-baseline --env Unicycle > $OUT/eager_u.json 2>&1 || { tail -20 $OUT/eager_u.json; exit 1; }
tail -1 $OUT/eager_u.json

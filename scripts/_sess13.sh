set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01j; mkdir -p $OUT
for r in 1 2; do for gs in 50 100 200; do
timeout -k 10 300 python bench.py --no-cpu-baseline --graph-steps $gs > $OUT/b_${gs}_${r}.json 2>&1 || exit 1
echo "gs=$gs $(grep -o '"ms_per_step": [0-9.e-]*\|"kernel_ms": [0-9.]*' $OUT/b_${gs}_${r}.json | tr '\n' ' ')"
done; done
timeout -k 10 300 python bench.py --no-cpu-baseline --graph-steps 1000 --steps 1000 > $OUT/b_1000.json 2>&1 || exit 1
echo "gs=1000 steps=1000 $(grep -o '"ms_per_step": [0-9.e-]*\|"kernel_ms": [0-9.]*' $OUT/b_1000.json | tr '\n' ' ')"

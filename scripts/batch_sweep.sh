# Fused-step time vs batch (per-step floor = launch + kernel boundary).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:-sweep}; mkdir -p $OUT
for b in 1024 4096 16384 32768 65536 131072 262144 1048576; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --batch $b --steps 200 > $OUT/b$b.log 2>&1 || exit $?
  echo "$b $(grep -o '"ms_per_step": [0-9.e-]*' $OUT/b$b.log) $(grep -o '"frac": [0-9.]*' $OUT/b$b.log)" | tee -a $OUT/sweep.txt
done

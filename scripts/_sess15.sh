set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01n; mkdir -p $OUT
for r in 1 2; do for v in unset 0 1; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b_${v}_$r.json 2>&1 || exit 1
  echo "DEV_KERNARG=$v $(grep -o '"ms_per_step": [0-9.e-]*\|"kernel_ms": [0-9.]*' $OUT/b_${v}_$r.json | tr '\n' ' ')"
done; done
unset HIP_FORCE_DEV_KERNARG
timeout -k 10 200 python scripts/exp_streams.py --shards d1 > $OUT/floor.txt 2>&1; grep floor $OUT/floor.txt
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python scripts/exp_streams.py --shards d1 > $OUT/floor1.txt 2>&1; grep floor $OUT/floor1.txt

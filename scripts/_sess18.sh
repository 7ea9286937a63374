set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01ae; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gp.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lib in base main; do
  if [ $lib = base ]; then export RCBF_HIP_LIB=build/variants/librcbf_base.so; else unset RCBF_HIP_LIB; fi
  timeout -k 10 300 python scripts/gp_bench.py 10 3000 > $OUT/gp_${lib}_exact.json 2>&1 || exit 1
  timeout -k 10 300 python scripts/gp_bench.py 10 3000 100 > $OUT/gp_${lib}_r100.json 2>&1 || exit 1
  echo "$lib exact $(tail -1 $OUT/gp_${lib}_exact.json)"
  echo "$lib r100 $(tail -1 $OUT/gp_${lib}_r100.json)"
done

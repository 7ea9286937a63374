#!/usr/bin/env bash
# r04v study: the split-K GP instantiation staging 64 training rows at a time (4 workgroups per CU's LDS,
# occupancy 4) vs the product's 256.  Build: build_lib(out=build/variants/librcbf_gpch64.so,
# defines=['-DRCBF_GP_SK_CHUNK=64']).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r04v
mkdir -p "$OUT"
RCBF_HIP_LIB=build/variants/librcbf_gpch64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$OUT/pytest_ch64.log" 2>&1; tail -1 "$OUT/pytest_ch64.log"
for r in 1 2 3; do
  for v in prod ch64; do
    if [ $v = prod ]; then e=""; else e="RCBF_HIP_LIB=build/variants/librcbf_gpch64.so"; fi
    for B in 64 256 384; do echo "$v $(env $e timeout -k 10 120 python scripts/gp_one.py $B 20 2>/dev/null)" >> "$OUT/ab.txt" || exit 1; done
  done
done
sort -s -k1,1 "$OUT/ab.txt"

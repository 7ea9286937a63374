#!/usr/bin/env bash
# GP posterior variants on one box: the GP parity tests on each variant
# library, then 3 interleaved timing rounds (scripts/gp_one.py, B = 256 and
# 4096), then SQ counters and a kernel trace of the LAST variant.
# Usage: bash scripts/gp_ab.sh TAG variant [variant ...]   (build/variants/librcbf_<variant>.so; "prod" = the product)
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
lib() { [ "$1" = prod ] && echo "" || echo "RCBF_HIP_LIB=build/variants/librcbf_$1.so"; }
for v in "$@"; do
  [ "$v" = prod ] && continue
  env $(lib "$v") timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || { echo "pytest $v failed"; tail -5 "$OUT/pytest_$v.log"; exit 1; }
  echo "pytest $v: $(tail -1 "$OUT/pytest_$v.log")"
done
for r in 1 2 3; do
  for v in "$@"; do
    for B in 256 4096; do
      echo "$v $(env $(lib "$v") timeout -k 10 120 python scripts/gp_one.py $B 20 2>/dev/null)" >> "$OUT/ab.txt" || exit 1
    done
  done
done
cat "$OUT/ab.txt"
last=${!#}
for B in 4096 256; do
  env $(lib "$last") timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/pmc$B" -o run -- \
    python3 scripts/gp_one.py $B 3 > "$OUT/pmc$B.log" 2>&1 || exit 1
done
env $(lib "$last") timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr256" -o run -- \
  python3 scripts/gp_one.py 256 20 > "$OUT/tr256.log" 2>&1 || exit 1
rm -f "$OUT/tr256/run_kernel_trace.csv"
echo done

#!/usr/bin/env bash
# SQ counter passes of the product GP kernels (k_gp_*) at B = 256 and 4096;
# keeps only the k_gp_* rows of each counter CSV (the GP fit's torch/rocSOLVER
# dispatches would otherwise exceed what gpurun copies back).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:?tag}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name B counters...
  local name=$1 B=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/tmp_$name" -o run -- \
    python3 scripts/gp_one.py "$B" 3 > "$OUT/$name.log" 2>&1 || return 1
  { head -1 "$OUT/tmp_$name/run_counter_collection.csv"; grep 'k_gp_' "$OUT/tmp_$name/run_counter_collection.csv"; } \
    > "$OUT/$name.csv"
  rm -rf "$OUT/tmp_$name"
}
for B in 256 4096; do
  pass "sq1_B$B" $B SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES || exit 1
  pass "sq2_B$B" $B SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU || exit 1
done
echo ok

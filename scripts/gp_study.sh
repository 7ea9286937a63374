#!/usr/bin/env bash
# GP posterior kernel study on one box: per-kernel trace at B = 256 and 4096,
# then SQ counter passes of k_gp_qform at B = 4096 (each pass its own run,
# within the per-block counter limits) and one FETCH_SIZE pass.
# Usage: bash scripts/gp_study.sh TAG [lib.so ...]   (extra libs: A/B timing only)
set -u
TAG=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
log() { echo "[$(date +%H:%M:%S)] $*" | tee -a "$OUT/steps.log"; }
run() {
  local name=$1 lim=$2; shift 2
  log "start $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  log "end $name rc=$rc"
  case $rc in 0) ;; *) log "fatal rc=$rc, stopping"; exit $rc;; esac
}
for B in 256 4096; do
  run "trace_B$B" 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_B$B" -o run -- \
    python3 scripts/gp_one.py "$B" 20
  rm -f "$OUT/trace_B$B/run_kernel_trace.csv"
done
run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/pmc1" -o run -- python3 scripts/gp_one.py 4096 3
run pmc2 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD \
  SQ_INSTS_SALU --output-format csv -d "$OUT/pmc2" -o run -- python3 scripts/gp_one.py 4096 3
run pmc3 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc3" -o run -- python3 scripts/gp_one.py 4096 3
for lib in "$@"; do
  for r in 1 2 3; do
    for l in prod "$lib"; do
      if [ "$l" = prod ]; then e=""; else e="RCBF_HIP_LIB=$l"; fi
      for B in 256 4096; do
        env $e timeout -k 10 120 python scripts/gp_one.py "$B" 20 >> "$OUT/ab_$(basename "$l").txt" 2>&1 || exit 1
      done
    done
  done
done
log "study done"

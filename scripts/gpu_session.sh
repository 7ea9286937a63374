#!/usr/bin/env bash
# One GPU-box session: each GPU step under its own time limit; a fault,
# abort, segfault or time-out ends the session (no further GPU step).
# Usage: bash scripts/gpu_session.sh TAG step [step ...]
#   steps: smoke | pytest | bench | prof | pmc | benchx
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
  case $rc in 124|137|134|139|143) log "fatal rc=$rc, stopping"; exit $rc;; esac
  return 0
}
for step in "$@"; do
  case $step in
    smoke)  run smoke 400 python __graft_entry__.py smoke ;;
    pytest) run pytest 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider ;;
    bench)  run bench 600 python bench.py ;;
    benchu) run benchu 600 python bench.py --env Unicycle --hazards 3 --no-cpu-baseline ;;
    benchx) run benchx 600 python bench.py --extra --no-cpu-baseline ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
              python3 bench.py --no-cpu-baseline ;;
    pmcf)   run pmcf 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
              python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 ;;
    pmcw)   run pmcw 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
              python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 ;;
    pmcv)   run pmcv 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_valu" -o run -- \
              python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 ;;
    pmcfu)  run pmcfu 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_u" -o run -- \
              python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 --env Unicycle --hazards 3 ;;
    pmcwu)  run pmcwu 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_u" -o run -- \
              python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 --env Unicycle --hazards 3 ;;
    profu)  run profu 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profu" -o run -- \
              python3 bench.py --no-cpu-baseline --env Unicycle --hazards 3 ;;
    *) log "unknown step $step" ;;
  esac
done
log "session done"
# summarise the PMC passes on the box (the per-dispatch CSVs can be large)
K='k_safe_step<0, 0, 1>'
if [ -f "$OUT/pmc_fetch/run_counter_collection.csv" ] && [ -f "$OUT/pmc_write/run_counter_collection.csv" ]; then
  python scripts/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" \
    "$K" "$OUT/pmc_traffic_cars_B65536.json" B=65536 env=SimulatedCars > /dev/null
fi
if [ -f "$OUT/pmc_fetch_u/run_counter_collection.csv" ] && [ -f "$OUT/pmc_write_u/run_counter_collection.csv" ]; then
  python scripts/pmc_traffic.py "$OUT/pmc_fetch_u/run_counter_collection.csv" "$OUT/pmc_write_u/run_counter_collection.csv" \
    'k_safe_step<0, 1, 3>' "$OUT/pmc_traffic_unicycle3_B65536.json" B=65536 env=Unicycle hazards=3 > /dev/null
fi
[ -f "$OUT/prof/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/prof/run_kernel_trace.csv" "$K" "$OUT/cars_B65536_kernel_trace_summary.json"
[ -f "$OUT/profu/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/profu/run_kernel_trace.csv" 'k_safe_step<0, 1, 3>' "$OUT/unicycle3_B65536_kernel_trace_summary.json"
[ -f "$OUT/pmc_valu/run_counter_collection.csv" ] && python scripts/pmc_sq.py "$OUT/pmc_valu/run_counter_collection.csv" "$K" > "$OUT/pmc_sq_cars_B65536.txt"
# keep what comes back under gpurun's 64 MiB cap: drop per-dispatch traces larger than 4 MiB
find "$OUT" -type f -size +4M -print -delete

#!/usr/bin/env bash
# One GPU-box session: each GPU step under its own time limit; a fault,
# abort, segfault or time-out ends the session (no further GPU step).
# Usage: bash scripts/gpu_session.sh TAG step [step ...]
#   steps: smoke | pytest | bench | driver (the driver's 20-step form) | profdrv (it, traced) | benchx
#          b_<w> | prof_<w> | pmc_<w> | sq_<w>    with workload <w> = cars | uni3 | uni5 | carsT | uni5T
#          (bench.py without the CPU baseline;
#           rocprofv3 kernel-trace stats; FETCH_SIZE and WRITE_SIZE passes;
#           SQ instruction counts -- each counter pass its own run)
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
wl_args() {  # bench.py arguments of a workload
  case $1 in
    cars) echo "--env SimulatedCars" ;;
    uni3) echo "--env Unicycle --hazards 3" ;;
    uni5) echo "--env Unicycle --hazards 5" ;;
    carsT) echo "--env SimulatedCars --prior tensor" ;;
    carsR) echo "--env SimulatedCars --prior rows" ;;
    uni5T) echo "--env Unicycle --hazards 5 --prior tensor" ;;
  esac
}
wl_kernel() {  # the fused kernel's name in rocprofv3 output
  case $1 in
    cars|carsT|carsR) echo 'k_safe_step<0, 0, 1, false>' ;;
    uni3) echo 'k_safe_step<0, 1, 3, false>' ;;
    uni5|uni5T) echo 'k_safe_step<0, 1, 5, false>' ;;
  esac
}
wl_name() {
  case $1 in cars) echo cars ;; uni3) echo unicycle3 ;; uni5) echo unicycle5 ;;
    carsT) echo cars_tensorprior ;; carsR) echo cars_rowsprior ;; uni5T) echo unicycle5_tensorprior ;; esac
}
for step in "$@"; do
  wl=${step#*_}
  case $step in
    smoke)  run smoke 400 python __graft_entry__.py smoke ;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    bench)  run bench 600 python bench.py ;;
    driver) run driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    benchx) run benchx 600 python bench.py --extra --no-cpu-baseline ;;
    sweep)  # waves per SIMD: B = 32768 (half the SIMDs), 65536 (one wave each), 98304, 131072 (two)
      for w in cars uni3 uni5; do for b in 32768 65536 98304 131072; do
        run "sweep_${w}_$b" 300 python bench.py --no-cpu-baseline --batch "$b" $(wl_args "$w")
      done; done ;;
    b_*)    run "b_$wl" 300 python bench.py --no-cpu-baseline $(wl_args "$wl") ;;
    prof_*)
      run "prof_$wl" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline $(wl_args "$wl")
      [ -f "$OUT/prof_$wl/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/prof_$wl/run_kernel_trace.csv" \
        "$(wl_kernel "$wl")" "$OUT/$(wl_name "$wl")_B65536_kernel_trace_summary.json" ;;
    profdrv)  # the driver's own command under the tracer
      run profdrv 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profdrv" -o run -- \
        python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
      [ -f "$OUT/profdrv/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/profdrv/run_kernel_trace.csv" \
        "$(wl_kernel cars)" "$OUT/cars_B65536_driver_form_kernel_trace_summary.json" ;;
    pmc_*)
      run "pmcf_$wl" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcf_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      run "pmcw_$wl" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcw_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      if [ -f "$OUT/pmcf_$wl/run_counter_collection.csv" ] && [ -f "$OUT/pmcw_$wl/run_counter_collection.csv" ]; then
        python scripts/pmc_traffic.py "$OUT/pmcf_$wl/run_counter_collection.csv" "$OUT/pmcw_$wl/run_counter_collection.csv" \
          "$(wl_kernel "$wl")" "$OUT/pmc_traffic_$(wl_name "$wl")_B65536.json" B=65536 workload="$(wl_name "$wl")" > /dev/null
      fi ;;
    sq_*)
      run "sq_$wl" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        --output-format csv -d "$OUT/sq_$wl" -o run -- python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      [ -f "$OUT/sq_$wl/run_counter_collection.csv" ] && python scripts/pmc_sq.py "$OUT/sq_$wl/run_counter_collection.csv" \
        "$(wl_kernel "$wl")" > "$OUT/pmc_sq_$(wl_name "$wl")_B65536.txt" ;;
    *) log "unknown step $step" ;;
  esac
done
log "session done"
# keep what comes back under gpurun's 64 MiB cap: drop per-dispatch traces larger than 4 MiB
find "$OUT" -type f -size +4M -print -delete

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
    c1) echo "--config 1" ;;
    c2) echo "--config 2" ;;
    c3) echo "--config 3" ;;
    c4) echo "--config 4" ;;
    c4s) echo "--env SimulatedCars --batch 32768" ;;  # config 4's per-GPU shard at 8 GPUs
    c5) echo "--config 5" ;;
  esac
}
wl_kernel() {  # the timed kernel's name in rocprofv3 output (workgroup size from rcbf_common.hpp block_for_envs)
  case $1 in
    cars|carsT|carsR|c4) echo 'k_safe_step<0, 0, 1, false, 256, false>' ;;
    uni3) echo 'k_safe_step<0, 1, 3, false, 256, false>' ;;
    uni5|uni5T) echo 'k_safe_step<0, 1, 5, false, 256, false>' ;;
    c1|c2) echo 'k_safe_step<0, 0, 1, false, 64, false>' ;;
    c3) echo 'k_safe_step<0, 1, 3, false, 64, false>' ;;
    c4s) echo 'k_safe_step<0, 0, 1, false, 128, false>' ;;
    c5) echo 'k_safe_action_jac<0, 0, 1, true, 64>' ;;
  esac
}
wl_name() {  # <short>_B<batch>, the workload's name in profiles/ (bench.py workload_short)
  case $1 in cars) echo cars_B65536 ;; uni3) echo uni3_B65536 ;; uni5) echo uni5_B65536 ;;
    carsT) echo cars_tensorprior_B65536 ;; carsR) echo cars_rowsprior_B65536 ;; uni5T) echo uni5_tensorprior_B65536 ;;
    c1) echo cars_B1 ;; c2) echo cars_rowsprior_maxstd_B4096 ;; c3) echo uni3_B4096 ;; c4) echo cars_B262144 ;;
    c4s) echo cars_B32768 ;; c5) echo sacupd_cars_rowsprior_maxstd_B4096 ;; esac
}
for step in "$@"; do
  wl=${step#*_}
  case $step in
    smoke)  run smoke 400 python __graft_entry__.py smoke ;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ;;
    bench)  run bench 600 python bench.py ;;
    driver) run driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ;;
    drvgraph) run drvgraph 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --launch graph ;;
    recdrv)  # the driver's command with its roofline record (per-step GPU time, dispatch timestamps, span stamps, clock)
      run recdrv 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        --record "$OUT/roofline_record_driver_form_aql_cars_B65536_$TAG.json" ;;
    recdef) run recdef 300 python bench.py --no-cpu-baseline --record "$OUT/roofline_record_aql_cars_B65536_$TAG.json" ;;
    pmcbusy)  # GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES pass of the driver's command -> busy us per dispatch (needs recdrv first)
      run pmcbusy 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d "$OUT/pmcbusy" -o run -- \
        python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-span
      [ -f "$OUT/pmcbusy/run_counter_collection.csv" ] && python scripts/pmc_busy.py "$OUT/pmcbusy/run_counter_collection.csv" \
        "$(wl_kernel cars)" "$OUT/roofline_record_driver_form_aql_cars_B65536_$TAG.json" \
        "$OUT/pmc_busy_driver_form_aql_cars_B65536_$TAG.json" > /dev/null ;;
    benchx) run benchx 600 python bench.py --extra --no-cpu-baseline ;;
    aqltest) run aqltest 300 python -u -m pytest tests/test_gpu_aql.py -q -rf --timeout 200 --timeout-method thread ;;
    aqltl) run aqltl 300 python -u scripts/exp_aql_timeline.py ;;
    scal)  # per-shard batches for the 1 -> 8 projection (scripts/scaling_projection.py), both command forms
      for b in 65536 32768 16384 8192; do
        run "scal_d_$b" 200 python bench.py --no-cpu-baseline --no-span --batch "$b" --steps 20 --warmup 5
        run "scal_l_$b" 200 python bench.py --no-cpu-baseline --no-span --batch "$b"
      done
      python scripts/scaling_projection.py "$OUT/scaling_projection_$TAG.json" "$OUT"/scal_*.log > /dev/null ;;
    drvaql) run drvaql 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --launch aql ;;
    benchaql) run benchaql 300 python bench.py --no-cpu-baseline --launch aql ;;
    sweep)  # waves per SIMD: B = 32768 (half the SIMDs), 65536 (one wave each), 98304, 131072 (two)
      for w in cars uni3 uni5; do for b in 32768 65536 98304 131072; do
        run "sweep_${w}_$b" 300 python bench.py --no-cpu-baseline --batch "$b" $(wl_args "$w")
      done; done ;;
    b_*)    run "b_$wl" 300 python bench.py --no-cpu-baseline $(wl_args "$wl") ;;
    bc_*)   run "bc_$wl" 400 python bench.py $(wl_args "$wl") ;;  # with the CPU baselines
    prof_*)
      run "prof_$wl" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline $(wl_args "$wl")
      [ -f "$OUT/prof_$wl/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/prof_$wl/run_kernel_trace.csv" \
        "$(wl_kernel "$wl")" "$OUT/$(wl_name "$wl")_kernel_trace_summary.json"
      [ -f "$OUT/prof_$wl/run_kernel_stats.csv" ] && cp "$OUT/prof_$wl/run_kernel_stats.csv" "$OUT/kernel_stats_$(wl_name "$wl")_$TAG.csv" ;;
    profdrv)  # the driver's own command under the tracer (the AQL launch: rocprofv3 intercepts the library's queue)
      run profdrv 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profdrv" -o run -- \
        python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
      [ -f "$OUT/profdrv/run_kernel_trace.csv" ] && python scripts/trace_summary.py "$OUT/profdrv/run_kernel_trace.csv" \
        "$(wl_kernel cars)" "$OUT/cars_B65536_driver_form_aql_kernel_trace_summary.json"
      [ -f "$OUT/profdrv/run_kernel_stats.csv" ] && cp "$OUT/profdrv/run_kernel_stats.csv" "$OUT/kernel_stats_driver_form_aql_cars_B65536_$TAG.csv" ;;
    pmc_*)
      run "pmcf_$wl" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcf_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      run "pmcw_$wl" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcw_$wl" -o run -- \
        python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      if [ -f "$OUT/pmcf_$wl/run_counter_collection.csv" ] && [ -f "$OUT/pmcw_$wl/run_counter_collection.csv" ]; then
        python scripts/pmc_traffic.py "$OUT/pmcf_$wl/run_counter_collection.csv" "$OUT/pmcw_$wl/run_counter_collection.csv" \
          "$(wl_kernel "$wl")" "$OUT/pmc_traffic_$(wl_name "$wl").json" workload="$(wl_name "$wl")" > /dev/null
      fi ;;
    sq_*)
      run "sq_$wl" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        --output-format csv -d "$OUT/sq_$wl" -o run -- python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      [ -f "$OUT/sq_$wl/run_counter_collection.csv" ] && python scripts/pmc_sq.py "$OUT/sq_$wl/run_counter_collection.csv" \
        "$(wl_kernel "$wl")" > "$OUT/pmc_sq_$(wl_name "$wl").txt" ;;
    if_*)  # instruction-fetch waits: SQ wave-cycle shares and instruction-cache misses, one pass
      run "if_$wl" 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQC_ICACHE_MISSES \
        --output-format csv -d "$OUT/if_$wl" -o run -- python3 bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 5 $(wl_args "$wl")
      [ -f "$OUT/if_$wl/run_counter_collection.csv" ] && python scripts/pmc_sq.py "$OUT/if_$wl/run_counter_collection.csv" \
        "$(wl_kernel "$wl")" > "$OUT/pmc_ifetch_$(wl_name "$wl").txt" ;;
    pair)  # the unicycle lane-pair study build vs the product (scripts/uni_pair_study.py)
      run pair 300 python -u scripts/uni_pair_study.py
      RCBF_PAIR_VARIANT=core run pair_core 300 python -u scripts/uni_pair_study.py ;;
    pairsq)
      RCBF_PAIR_VARIANT=core run pairsq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU \
        --output-format csv -d "$OUT/pairsq" -o run -- python3 scripts/uni_pair_study.py --sq
      [ -f "$OUT/pairsq/run_counter_collection.csv" ] && for kk in "k_uni_pair_step<5, 256>" "k_safe_step<0, 1, 5, false, 256, false>" \
          "k_uni_pair_step<3, 64>" "k_uni_pair_step<3, 128>" "k_safe_step<0, 1, 3, false, 64, false>"; do
        echo "== $kk" >> "$OUT/pmc_sq_pair.txt"; python scripts/pmc_sq.py "$OUT/pairsq/run_counter_collection.csv" "$kk" >> "$OUT/pmc_sq_pair.txt"; done ;;
    tracer)  # control: torch kernels of the same bytes, untraced (events) and traced
      run tracer_plain 120 python scripts/tracer_control.py
      run tracer_traced 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tracer" -o run -- \
        python3 scripts/tracer_control.py
      [ -f "$OUT/tracer/run_kernel_stats.csv" ] && cp "$OUT/tracer/run_kernel_stats.csv" "$OUT/kernel_stats_tracer_control_$TAG.csv" ;;
    gpab)  # GP posterior timing, product vs build/variants/librcbf_gpold.so, 3 rounds (scripts/gp_bench.py, n_s 10, N 3000)
      for r in 1 2 3; do for n in prod gpold; do
        if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
        env $lib timeout -k 10 200 python scripts/gp_bench.py 10 3000 > "$OUT/gp_${n}_$r.log" 2>&1 || exit 1
        echo "$n $(tail -1 "$OUT/gp_${n}_$r.log")" >> "$OUT/gpab_sum.txt"
      done; done ;;
    gpt)    run gpt 600 python -u -m pytest tests/test_gpu_gp.py tests/test_gpu_parity.py -q -rf --timeout 300 --timeout-method thread ;;
    loop)   run loop 900 python -u -m pytest tests/test_gpu_training_loop.py -q -rf -s --timeout 600 --timeout-method thread ;;
    gpgb)   run gpgb 300 python -u scripts/gp_graph_bench.py ;;
    gpsk)   # split-K count sweep of the B = 256 GP posterior (study build build/variants/librcbf_gpsplit.so)
      for sk in ${GPSK_LIST:-0 6 11 16 22 32 47}; do
        if [ "$sk" = 0 ]; then e=""; else e="RCBF_GP_SPLIT=$sk"; fi
        env $e RCBF_HIP_LIB=build/variants/librcbf_gpsplit.so GP_BENCH_ONLY=love100:256 timeout -k 10 200 \
          python scripts/gp_graph_bench.py 20 5 > "$OUT/gpsk_$sk.log" 2>&1 || exit 1
        echo "sk=$sk $(tail -1 "$OUT/gpsk_$sk.log")" >> "$OUT/gpsk_sum.txt"
      done ;;
    single) run single 300 python -u scripts/single_env_latency.py ;;
    msab)   # model step / predict_next_state: product vs build/variants/librcbf_modelold.so, 3 rounds
      for r in 1 2 3; do for n in prod modelold; do
        if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
        env $lib timeout -k 10 200 python scripts/model_step_bench.py > "$OUT/ms_${n}_$r.log" 2>&1 || exit 1
        echo "$n $(tail -1 "$OUT/ms_${n}_$r.log")" >> "$OUT/msab_sum.txt"
      done; done ;;
    epw)    # lanes-per-wave study for small batches (build/variants/librcbf_epw{16,32}.so): parity, then A/B
      for n in epw16 epw32; do
        RCBF_HIP_LIB=build/variants/librcbf_$n.so run "epw_parity_$n" 300 python -u -m pytest tests/test_gpu_headline_parity.py \
          -q -rf -k "small_batch or config4_eight" --timeout 200 --timeout-method thread
        grep -q " passed" "$OUT/epw_parity_$n.log" || exit 1
      done
      bash scripts/ab_multi.sh "$TAG/epwab" "epw16 epw32" c2 c3 c5 || exit 1 ;;
    gppmc)  # HBM traffic of the rank-100 GEMV at B = 1 (eager calls; FETCH_SIZE and WRITE_SIZE in their own passes)
      GP_RANK=100 run gppmc_f 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/gppmc_f" -o run -- python3 scripts/gp_one.py 1 50
      GP_RANK=100 run gppmc_w 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/gppmc_w" -o run -- python3 scripts/gp_one.py 1 50
      if [ -f "$OUT/gppmc_f/run_counter_collection.csv" ] && [ -f "$OUT/gppmc_w/run_counter_collection.csv" ]; then
        python scripts/pmc_traffic.py "$OUT/gppmc_f/run_counter_collection.csv" "$OUT/gppmc_w/run_counter_collection.csv" \
          "k_gp_gemv<10, 1>" "$OUT/pmc_traffic_gp_gemv_rank100_B1.json" workload="GP N=3000 rank 100 B=1" \
          algorithmic_read_bytes=16724480 > /dev/null
      fi ;;
    soak)   run soak 600 python -u -m pytest tests/test_gpu_headline_parity.py -q -rf -k soak --timeout 500 --timeout-method thread ;;
    gpm)    run gpm 300 python -u -m pytest tests/test_gpu_model.py -q -rf --timeout 200 --timeout-method thread ;;
    rccl)   run rccl 300 python bench.py --rccl --steps 20 --warmup 5 --no-cpu-baseline ;;  # the N > 1 collectives on one rank
    gvstudy)  # GEMV study variants (build/variants/librcbf_gv*.so) vs the product, GP graph bench
      for n in prod ${GV_VARIANTS:-gv1 gv3 gvr128}; do
        if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
        env $lib timeout -k 10 200 python scripts/gp_graph_bench.py > "$OUT/gvstudy_$n.log" 2>&1 || exit 1
      done ;;
    profgp256) GP_BENCH_ONLY=love100:256 run profgp256 300 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$OUT/profgp256" -o run -- python3 scripts/gp_graph_bench.py 20 5
      [ -f "$OUT/profgp256/run_kernel_stats.csv" ] && cp "$OUT/profgp256/run_kernel_stats.csv" "$OUT/kernel_stats_gp_love100_B256_$TAG.csv" ;;
    profgp1) GP_BENCH_ONLY=love100:1 run profgp1 300 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$OUT/profgp1" -o run -- python3 scripts/gp_graph_bench.py 20 5
      [ -f "$OUT/profgp1/run_kernel_stats.csv" ] && cp "$OUT/profgp1/run_kernel_stats.csv" "$OUT/kernel_stats_gp_love100_B1_$TAG.csv" ;;
    profgp) run profgp 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profgp" -o run -- \
              python3 scripts/gp_graph_bench.py 20 5
      [ -f "$OUT/profgp/run_kernel_stats.csv" ] && cp "$OUT/profgp/run_kernel_stats.csv" "$OUT/kernel_stats_gp_graph_bench_$TAG.csv" ;;
    abjac) bash scripts/ab_multi.sh "$TAG/abjac" "jacgi" c5 || exit 1 ;;
    abbs)  bash scripts/ab_multi.sh "$TAG/abbs" "bs256" c2 c3 c4s c5 || exit 1 ;;
    absin) bash scripts/ab_multi.sh "$TAG/absin" "nosincos" u5 u3 || exit 1 ;;
    *) log "unknown step $step" ;;
  esac
done
log "session done"
# keep what comes back under gpurun's 64 MiB cap: drop per-dispatch traces larger than 4 MiB
find "$OUT" -type f -size +4M -print -delete

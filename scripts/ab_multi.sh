# A/B/n of library builds in one GPU session: the product librcbf_hip.so ("prod") against named
# builds under build/variants/ (librcbf_NAME.so), alternating, 3 rounds, bench.py without the CPU
# baseline; one line per run in gpurun_out/TAG/sum.txt.
# Usage: bash scripts/ab_multi.sh TAG "NAME ..." workload [workload ...]
#   (workload = cars | u3 | u5 | drv | carsT | u5T | c1 | c2 | c3 | c4 | c4s | c5)
cd "${GRAFT_REPO_ROOT:-.}"; O=gpurun_out/$1; NAMES=$2; shift 2; mkdir -p $O
for r in 1 2 3; do for w in "$@"; do
  case $w in cars) a="--env SimulatedCars";; u3) a="--env Unicycle --hazards 3";; u5) a="--env Unicycle --hazards 5";;
    drv) a="--gpus 1 --steps 20 --warmup 5";; carsT) a="--env SimulatedCars --prior tensor";;
    u5T) a="--env Unicycle --hazards 5 --prior tensor";; c1) a="--config 1";; c2) a="--config 2";;
    c3) a="--config 3";; c4) a="--config 4";; c4s) a="--batch 32768";; c5) a="--config 5";; esac
  for n in prod $NAMES; do
    if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
    env $lib timeout -k 10 100 python bench.py --no-cpu-baseline --no-span $a > $O/${n}_$w.log 2>&1 || exit 1
    echo "$n $w $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/${n}_$w.log | tr '\n' ' ')" >> $O/sum.txt
  done
done; done

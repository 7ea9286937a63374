# A/B of two library builds in one GPU session: the product librcbf_hip.so ("new") against
# sac-rcbf_amd/rcbf_amd/librcbf_hip_old.so ("old", e.g. one TU rebuilt from the previous source),
# alternating, 3 rounds, bench.py without the CPU baseline; one line per run in gpurun_out/TAG/sum.txt.
# Usage: bash scripts/ab_bench.sh TAG workload [workload ...]   (workload = cars | u3 | u5 | drv)
cd "${GRAFT_REPO_ROOT:-.}"; O=gpurun_out/$1; shift; mkdir -p $O
V=sac-rcbf_amd/rcbf_amd/librcbf_hip_old.so
for r in 1 2 3; do for w in "$@"; do
  case $w in cars) a="--env SimulatedCars";; u3) a="--env Unicycle --hazards 3";; u5) a="--env Unicycle --hazards 5";; drv) a="--gpus 1 --steps 20 --warmup 5";; esac
  timeout -k 10 100 python bench.py --no-cpu-baseline $a > $O/new_$w.log 2>&1 || exit 1
  echo "new $w $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/new_$w.log | tr '\n' ' ')" >> $O/sum.txt
  RCBF_HIP_LIB=$V timeout -k 10 100 python bench.py --no-cpu-baseline $a > $O/old_$w.log 2>&1 || exit 1
  echo "old $w $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/old_$w.log | tr '\n' ' ')" >> $O/sum.txt
done; done

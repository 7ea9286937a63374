# A/B of the product library vs build/variants/librcbf_late.so at large batches (4 M and 1 M envs, HBM-bound), 3 rounds
cd "${GRAFT_REPO_ROOT:-.}"; O=gpurun_out/r03p; mkdir -p $O
for r in 1 2 3; do for n in prod late; do
  if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
  for b in 4194304 1048576; do
    env $lib timeout -k 10 200 python bench.py --no-cpu-baseline --batch $b --steps 200 --warmup 10 > $O/${n}_$b.log 2>&1 || exit 1
    echo "$n B=$b $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/${n}_$b.log | tr '\n' ' ')" >> $O/sum.txt
  done
done; done

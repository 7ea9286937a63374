# A/B of GP posterior builds (scripts/gp_bench.py: cars n_s = 10, N = 3000, exact) over the product library and
# the named build/variants/librcbf_NAME.so, 2 rounds, then test_gpu_gp.py on each variant.
# Usage: bash scripts/ab_gp.sh TAG "NAME ..."
cd "${GRAFT_REPO_ROOT:-.}"; O=gpurun_out/$1; NAMES=$2; mkdir -p $O
for r in 1 2; do for n in prod $NAMES; do
  if [ "$n" = prod ]; then lib=""; else lib="RCBF_HIP_LIB=build/variants/librcbf_$n.so"; fi
  env $lib timeout -k 10 200 python scripts/gp_bench.py 10 3000 > $O/${n}_gp.log 2>&1 || exit 1
  echo "$n $(tail -1 $O/${n}_gp.log)" >> $O/sum.txt
done; done
for n in $NAMES; do
  RCBF_HIP_LIB=build/variants/librcbf_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gp.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > $O/pytest_$n.log 2>&1 || exit 1
done

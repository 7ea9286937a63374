set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_session.sh r03e pytest bench driver profdrv prof_cars prof_uni3 prof_uni5 pmc_cars pmc_uni3 pmc_uni5 pmc_carsT pmc_carsR pmc_uni5T b_carsT b_carsR b_uni5T benchx || exit 1
O=gpurun_out/r03e
for a in "65536" "65536 unicycle 3" "65536 unicycle 5"; do
  timeout -k 10 120 python scripts/stamps.py $a >> $O/stamps.txt 2>&1 || exit 1
done

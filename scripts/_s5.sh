set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/gpu_session.sh s5 pytest smoke bench driver benchx b_carsT b_uni5T pmc_carsT pmc_uni5T prof_cars || exit 1
timeout -k 10 120 python scripts/single_env_latency.py > gpurun_out/s5/lat.log 2>&1

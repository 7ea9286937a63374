set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s4; mkdir -p $O; export TMPDIR=/tmp
V=sac-rcbf_amd/rcbf_amd/librcbf_hip_early.so
b() { local n=$1; shift; timeout -k 10 150 "$@" > $O/$n.log 2>&1 || { echo "FAIL $n"; exit 1; }; }
b pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
b cars_a python bench.py --no-cpu-baseline
b cars_b env RCBF_HIP_LIB=$V python bench.py --no-cpu-baseline
b cars_a2 python bench.py --no-cpu-baseline
b cars_b2 env RCBF_HIP_LIB=$V python bench.py --no-cpu-baseline
b drv_a python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
b drv_b env RCBF_HIP_LIB=$V python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
b uni3 python bench.py --no-cpu-baseline --env Unicycle --hazards 3
b uni5 python bench.py --no-cpu-baseline --env Unicycle --hazards 5
b qp python scripts/qp_rows_prof.py
echo done

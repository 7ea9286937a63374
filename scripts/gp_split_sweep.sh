#!/usr/bin/env bash
# r04q study: GP tests, the split-K count at B = 256 (study build, RCBF_GP_SPLIT=sk), and the GEMV path
# (triangle vs dense) at B = 1 and 5.  Build the study library first:
#   python -c "import __graft_entry__ as g, os; g.build_lib(out=os.path.join(g.ROOT, 'build', 'variants',
#              'librcbf_gpsplit.so'), defines=['-DRCBF_STUDY_GP_SPLIT=1'])"
mkdir -p gpurun_out/r04q && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gp.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q/pytest_gp.log 2>&1; tail -1 gpurun_out/r04q/pytest_gp.log
for r in 1 2; do for sk in 2 3 4 5 6 8; do echo "sk=$sk $(RCBF_HIP_LIB=build/variants/librcbf_gpsplit.so RCBF_GP_SPLIT=$sk timeout -k 10 120 python scripts/gp_one.py 256 20 2>/dev/null)" >> gpurun_out/r04q/sk.txt || exit 1; done; echo "prod $(timeout -k 10 120 python scripts/gp_one.py 256 20 2>/dev/null)" >> gpurun_out/r04q/sk.txt; done
cat gpurun_out/r04q/sk.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q/tr256 -o run -- python3 scripts/gp_one.py 256 20 > gpurun_out/r04q/tr256.log 2>&1; rm -f gpurun_out/r04q/tr256/run_kernel_trace.csv
for r in 1 2 3; do for B in 1 5; do echo "B=$B tri $(timeout -k 10 120 python scripts/gp_one.py $B 50 2>/dev/null)  dense $(RCBF_GP_DENSE=1 timeout -k 10 120 python scripts/gp_one.py $B 50 2>/dev/null)" >> gpurun_out/r04q/gemv.txt || exit 1; done; done
cat gpurun_out/r04q/gemv.txt

set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/s3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python scripts/single_env_latency.py > $O/lat.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python scripts/qp_rows_prof.py > $O/qp.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/sq -o run -- python3 scripts/qp_rows_prof.py > $O/sq.log 2>&1 || exit 1
echo done

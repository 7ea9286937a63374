set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01h; mkdir -p $OUT
bash scripts/ablate_run.sh r01h "full st6 st12 st24 noslp full st6 st12 st24 noslp" "65536" || exit 1
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; exit $rc

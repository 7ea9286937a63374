set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01g; mkdir -p $OUT
:
timeout -k 10 300 python scripts/exp_streams.py > $OUT/streams.log 2>&1; rc=$?; cat $OUT/streams.log; exit $rc

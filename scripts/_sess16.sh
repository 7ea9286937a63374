set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "unicycle or cascade or Unicycle" > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  bash scripts/ablate_run.sh r01t "base uni1" "65536 4096" --env Unicycle --hazards 3 || exit 1
done
bash scripts/ablate_run.sh r01t "base uni1" "65536" || exit 1

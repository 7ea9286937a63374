#!/usr/bin/env bash
# GP posterior: the GP tests on the product, then 3 interleaved timing rounds of
#   base  = the level-0 kernel (build/variants/librcbf_gpl0.so: python __graft_entry__.py variant gpl0 -DRCBF_GP_DOT_MFMA=0), dense [R | alpha]
#   dense = the product kernel, dense [R | alpha] (RCBF_GP_DENSE=1)
#   tri   = the product kernel with the upper-triangular skip
# at B = 1, 256, 4096 (scripts/gp_one.py).  Usage: bash scripts/gp_ab2.sh TAG
set -u
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gp.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gp.log" 2>&1 || { tail -30 "$OUT/pytest_gp.log"; exit 1; }
echo "pytest: $(tail -1 "$OUT/pytest_gp.log")"
for r in 1 2 3; do
  for v in base dense tri; do
    case $v in
      base) e="RCBF_HIP_LIB=build/variants/librcbf_gpl0.so RCBF_GP_DENSE=1" ;;
      dense) e="RCBF_GP_DENSE=1" ;;
      tri) e="" ;;
    esac
    for B in 1 256 4096; do
      echo "$v $(env $e timeout -k 10 120 python scripts/gp_one.py $B 20 2>/dev/null)" >> "$OUT/ab.txt" || exit 1
    done
  done
done
cat "$OUT/ab.txt"

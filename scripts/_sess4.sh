set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
RCBF_HIP_LIB=build/variants/librcbf_stage.so timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider -k "fused or step or rollout or reset" > $OUT/pytest_stage.log 2>&1 || exit 1
bash scripts/ablate_run.sh $TAG "base early stage stage_early stage_nt sc1 base stage" "65536" || exit 1
bash scripts/ablate_run.sh $TAG "base stage" "65536" --env Unicycle --hazards 3 || exit 1

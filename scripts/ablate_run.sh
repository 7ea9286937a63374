#!/usr/bin/env bash
# Time each build/variants/librcbf_<name>.so with bench.py at several batches.
# Usage: bash scripts/ablate_run.sh TAG "name1 name2 ..." "B1 B2 ..." [extra bench args]
set -u
TAG=$1; NAMES=$2; BATCHES=$3; shift 3
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for n in $NAMES; do
  for b in $BATCHES; do
    RCBF_HIP_LIB=build/variants/librcbf_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --batch $b "$@" \
      > "$OUT/abl_${n}_${b}.log" 2>&1
    rc=$?
    echo "$n $b rc=$rc $(grep -o '"ms_per_step": [0-9.e-]*' "$OUT/abl_${n}_${b}.log")" | tee -a "$OUT/ablate.txt"
    case $rc in 124|137|134|139) exit $rc;; esac
  done
done

set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r01m; mkdir -p $OUT
export RCBF_HIP_LIB=build/variants/librcbf_stamps.so
for a in "" "--eager" "unicycle" "unicycle --eager"; do
  timeout -k 10 200 python scripts/stamps.py 65536 $a > "$OUT/stamps_${a// /_}.txt" 2>&1 || { cat "$OUT/stamps_${a// /_}.txt" | tail; exit 1; }
  sed '/amdgpu.ids/d' "$OUT/stamps_${a// /_}.txt"
done

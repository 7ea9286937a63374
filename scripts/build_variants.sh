#!/usr/bin/env bash
# Build performance-study variants of librcbf_hip.so into build/variants/
# (same sources, -DRCBF_ABLATE=<bits> / -DRCBF_BLOCK=<threads>).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
FLAGS="--offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Isac-rcbf_amd/csrc"
for spec in "$@"; do   # spec = name:defines   e.g. noqp:-DRCBF_ABLATE=1
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc $FLAGS ${defs//,/ } -o build/variants/librcbf_$name.so sac-rcbf_amd/csrc/rcbf_kernels.hip &
done
wait
ls -la build/variants

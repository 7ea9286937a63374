#!/usr/bin/env bash
# Build performance-study variants of librcbf_hip.so into build/variants/
# (same sources, extra -D defines).  spec = name:-DA=1,-DB=2
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  python __graft_entry__.py variant "$name" ${defs//,/ } > /dev/null &
done
wait
ls -la build/variants

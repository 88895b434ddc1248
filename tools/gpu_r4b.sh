#!/bin/bash
# Round-4 GPU pass b: write-pattern probe -- chunked vs interleaved schedules at 1-3 workgroups
# per CU, and the write granularity (aligned runs of G elements) each output array needs.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4b
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 ./tools/scatter_pattern > "$OUT/scatter_pattern.txt" 2>&1 || { echo "pattern probe failed"; tail -5 "$OUT/scatter_pattern.txt"; exit 1; }
cat "$OUT/scatter_pattern.txt"

#!/bin/bash
# Round-4 GPU pass a: the radix scatter's write pattern in isolation (tools/scatter_pattern) and
# config-3 build A/B over the existing radix knobs (3 passes at R = 47, 8-wave scatter, chunked).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4a
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 240 ./tools/scatter_pattern > "$OUT/scatter_pattern.txt" 2>&1 || { echo "pattern probe failed"; tail -5 "$OUT/scatter_pattern.txt"; exit 1; }
cat "$OUT/scatter_pattern.txt"
timeout -k 10 900 bash tools/ab.sh "KMHG_X=0" "KMHG_MAXR=47" "KMHG_SC8=1" "KMHG_RADIX=chunked" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

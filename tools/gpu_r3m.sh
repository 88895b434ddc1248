#!/bin/bash
# Round-3 GPU pass m: A/B of the fused query (probe + look-back + emit) against the three-kernel
# query now that the diagonal path makes the probe cheap.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3m
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 bash tools/ab.sh "KMHG_QUERY=classic" "KMHG_QUERY=fused" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

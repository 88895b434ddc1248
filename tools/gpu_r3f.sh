#!/bin/bash
# Round-3 GPU pass f: A/B of scatter workgroups per CU at config 3 (beyond the Infinity Cache)
# and config 2.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3f
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 900 bash tools/ab.sh "KMHG_SCATTER_WPC=3" "KMHG_SCATTER_WPC=2" "KMHG_SCATTER_WPC=1" \
  -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_SCATTER_WPC=3" "KMHG_SCATTER_WPC=2" \
  -- --no-cpu --no-reads || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"

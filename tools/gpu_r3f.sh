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
# FETCH_SIZE calibration for random 16-B / 4-B reads (tools/calib/fetch_calib.hip)
mkdir -p "$REPO/gpurun_out/calib"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$REPO/gpurun_out/calib/fetch" \
  -o run -- "$REPO/tools/calib/fetch_calib" > "$REPO/gpurun_out/calib/fetch.log" 2>&1 \
  || { echo "calib failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/calib/kt" \
  -o run -- "$REPO/tools/calib/fetch_calib" > "$REPO/gpurun_out/calib/kt.log" 2>&1 \
  || { echo "calib kt failed"; exit 1; }
echo "calib done"

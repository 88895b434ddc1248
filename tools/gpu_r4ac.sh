#!/bin/bash
# Round 4: read k-mer walk from global memory at full occupancy (KMHG_RK_GLOBAL variant: no LDS
# staging) against the LDS-staged walk -- reads leg A/B at config 2.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4ac
mkdir -p "$OUT"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=rkg" -- --no-cpu \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"

#!/bin/bash
# Round-4 GPU pass n: owner-computes per-rank step rehearsed on one GPU (tools/part_step.py), and
# the host-boundary query's D2H copy threads A/B.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4n
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python -u tools/part_step.py 10 10 > "$OUT/part_step.log" 2>&1 || { echo "part_step failed"; tail -20 "$OUT/part_step.log"; exit 1; }
cat "$OUT/part_step.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_D2H_THREADS=4" "KMHG_D2H_THREADS=8" "KMHG_D2H_THREADS=16" -- --no-cpu --no-reads \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_d2h.log"

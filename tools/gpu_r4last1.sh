#!/bin/bash
# Round-4 closing evidence final library (adaptive anchors), part 1: whole
# GPU suite + smoke + default bench, then configs 3-5.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/gpu_check.sh rd4last || exit 1
OUT=$REPO/gpurun_out/cfg_rd4last
mkdir -p "$OUT"
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  echo "config $c ok"
done
timeout -k 10 300 python -u tools/part_step.py 10 10 > "$OUT/part_step.log" 2>&1 || { echo "part_step failed"; tail -20 "$OUT/part_step.log"; exit 1; }
cat "$OUT/part_step.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_COUNT_BID=1" "KMHG_COUNT_BID=0" -- --no-cpu --no-reads \
  || { echo "ab count bid failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_count_bid.log"

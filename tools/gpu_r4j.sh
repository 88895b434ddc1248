#!/bin/bash
# Round-4 mid-round evidence (j): full GPU suite + smoke + default bench, configs 3-5 bench lines.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/gpu_check.sh rd4j || exit 1
OUT=$REPO/gpurun_out/cfg_rd4j
mkdir -p "$OUT"
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  echo "config $c ok"
done

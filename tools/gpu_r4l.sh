#!/bin/bash
# Round-4 evidence (l): configs 4 and 5 bench lines, then the rocprofv3 passes of tools/gpu_r4k.sh.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/cfg_rd4j
mkdir -p "$OUT"
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  echo "config $c ok"
done
bash tools/gpu_r4k.sh

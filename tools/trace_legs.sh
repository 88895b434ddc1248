#!/bin/bash
# Kernel trace (per dispatch) of the default bench legs, for attributing time inside the counts /
# reads / depth legs:  bash tools/trace_legs.sh <tag>   (through gpurun)
set -euo pipefail
TAG=${1:-legs}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$REPO/bench.py" --no-cpu --steps 3 --warmup 1 > "$OUT/bench.log" 2>&1
echo "trace $TAG done"

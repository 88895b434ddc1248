#!/bin/bash
# Round evidence after tools/gpu_check.sh (through gpurun): the other BASELINE configs' bench lines
# and the rocprofv3 kernel-trace / PMC passes of the default bench (tools/profile.sh).
#   bash tools/evidence.sh <tag>
set -uo pipefail
TAG=${1:-rNN}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/cfg_$TAG
mkdir -p "$OUT"
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  echo "config $c ok"
done
bash tools/profile.sh "$TAG" || exit 1

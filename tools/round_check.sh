#!/bin/bash
# Round-end evidence through gpurun: gpu tests + smoke + default bench (tools/gpu_check.sh), the
# other BASELINE configs, and the rocprofv3 kernel-trace / PMC passes (tools/profile.sh).
#   bash tools/round_check.sh <tag>
set -uo pipefail
TAG=${1:-rNN}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/gpu_check.sh "$TAG" || exit 1
OUT=$REPO/gpurun_out/cfg_$TAG
mkdir -p "$OUT"
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  cat "$OUT/config$c.json"
done
bash tools/profile.sh "$TAG" || exit 1

#!/bin/bash
# Round-4 GPU pass d: write-combined radix pass geometries at config 3 (A/B in one run), with
# a parity check of each geometry first.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4d
mkdir -p "$OUT"
cd "$REPO"
for gm in 1 2; do
  KMHG_SCATTER_WC_GEOM=$gm timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 240 --timeout-method thread -p no:cacheprovider -k "multi_pass and keyswc and lane" \
    > "$OUT/pytest_g$gm.log" 2>&1 || { echo "tests failed geom $gm"; tail -30 "$OUT/pytest_g$gm.log"; exit 1; }
  tail -1 "$OUT/pytest_g$gm.log"
done
timeout -k 10 900 bash tools/ab.sh "KMHG_SCATTER_WC=0" "KMHG_SCATTER_WC=1 KMHG_SCATTER_WC_GEOM=0" "KMHG_SCATTER_WC=1 KMHG_SCATTER_WC_GEOM=1" "KMHG_SCATTER_WC=1 KMHG_SCATTER_WC_GEOM=2" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

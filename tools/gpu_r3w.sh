#!/bin/bash
# Round-3 GPU pass w: the sorted bucket build (KMHG_BUCKET=sort) with atomic-rank sort passes --
# its tests, then A/B against the CAS build with key streams at config 2 and at config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3w
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "bucket or config4 or multi_pass or determinism or repeat" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_BUILD_BID=0" "KMHG_BUILD_BID=0 KMHG_BUCKET=sort" "KMHG_BUILD_BID=1" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_BUCKET=group" "KMHG_BUCKET=sort" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

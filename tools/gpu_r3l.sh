#!/bin/bash
# Round-3 GPU pass l: key streams whose first pass reads V_hist0's ids and cuts the keys from the
# code words (KMHG_BUILD_IDS0) -- parity subset, A/B at config 3 and at config 2 (key streams).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3l
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "multi_pass or bucket or 10mbp or config3 or config4" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_BUILD_IDS0=1" "KMHG_BUILD_IDS0=0" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUILD_BID=0 KMHG_BUILD_IDS0=1" "KMHG_BUILD_BID=0 KMHG_BUILD_IDS0=0" "KMHG_BUILD_BID=1" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

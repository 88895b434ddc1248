#!/bin/bash
# Round-3 GPU pass k: bucket kernel code-word loads hidden behind the table clear -- parity
# subset, config 2 A/B against key streams.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3k
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "multi_pass and bid or bucket or 10mbp" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUILD_BID=1" "KMHG_BUILD_BID=0" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

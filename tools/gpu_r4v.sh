#!/bin/bash
# Round-4 GPU pass v: count.kmers batches built with bucket-id streams (their code words kept) --
# counts tests, then A/B of the counts leg at config 2 against key streams (KMHG_COUNT_BID=0).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4v
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_counts.py tests/test_r_glue.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_COUNT_BID=1" "KMHG_COUNT_BID=0" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

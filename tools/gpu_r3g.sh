#!/bin/bash
# Round-3 GPU pass g: bucket-kernel tests + A/B of the claim-aware insert.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3g
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "bucket" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUCKET_FP=0" "KMHG_BUCKET_FP=3" -- --no-cpu --no-reads \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab.log"

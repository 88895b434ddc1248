#!/bin/bash
# Round-3 GPU pass za: single-workgroup build statistics (k_v2_stats1) -- build tests, A/B against
# the multi-workgroup form (KMHG_STATS1=0) at config 2.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3za
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sh.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "multi_pass or 10mbp or golden or config2 or config4 or bucket or counts or disorder or determinism" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_STATS1=1" "KMHG_STATS1=0" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

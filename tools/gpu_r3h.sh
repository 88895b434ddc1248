#!/bin/bash
# Round-3 GPU pass h: bucket-id radix streams -- parity (build tests, full-size digests), then
# an A/B of KMHG_BUILD_BID=0/1 at config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3h
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_gpu_parts.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "multi_pass or bucket or golden or edge or testfa or random or k32 or all_n or tandem or repeat_rich or determinism or 10mbp or khash or config or parts" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUILD_BID=1" "KMHG_BUILD_BID=0" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_BUILD_BID=1" "KMHG_BUILD_BID=0" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

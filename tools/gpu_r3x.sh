#!/bin/bash
# Round-3 GPU pass x: the first histogram pass with 8 consecutive windows per thread (Win8: 8 LDS
# reads per 8 windows) -- partition tests, A/B against the strided loop (KMHG_LIB_VARIANT=h0s) at
# config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3x
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_parts.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "multi_pass or 10mbp or golden or edge or window or random or config2 or config3 or part or disorder" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=h0s" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=h0s" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

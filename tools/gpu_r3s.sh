#!/bin/bash
# Round-3 GPU pass s: radix ranks from the returning LDS count atomics (lane-ordered), the
# bucket kernels' stream-order check -- the whole GPU suite, then A/B against the ballot-rank
# variant library (KMHG_LIB_VARIANT=ballot) at config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3s
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=ballot" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=ballot" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

#!/bin/bash
# Round-4 GPU pass w: the diagonal probe's anchor stride (64 = default) against 128 and 32
# (variant builds), query legs at configs 2, 3 and 5.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4w
mkdir -p "$OUT"
cd "$REPO"
KMHG_LIB_VARIANT=dg128 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "query or diagonal" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_dg128.log" 2>&1 || { echo "dg128 tests failed"; tail -30 "$OUT/pytest_dg128.log"; exit 1; }
tail -1 "$OUT/pytest_dg128.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg128" "KMHG_LIB_VARIANT=dg32" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg128" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg128" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"

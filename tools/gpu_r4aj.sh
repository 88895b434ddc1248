#!/bin/bash
# Round 4: persistent multi-hit emit grid of 1 / 2 workgroups per CU (variants em1 / em2) against
# the occupancy-sized grid -- query parity on the variants, then the query legs at configs 2 and 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4aj
mkdir -p "$OUT"
for v in em1 em2; do
  KMHG_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "query" > "$OUT/pytest_$v.log" 2>&1 \
    || { echo "pytest $v failed"; tail -30 "$OUT/pytest_$v.log"; exit 1; }
  tail -1 "$OUT/pytest_$v.log"
done
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=em1" "KMHG_LIB_VARIANT=em2" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=em1" "KMHG_LIB_VARIANT=em2" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"

#!/bin/bash
# Round 4: diagonal anchor stride 512 / 1024 (variant builds) against 256 -- query parity on the
# variants, then the query legs at configs 2, 3 and 5.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4ae
mkdir -p "$OUT"
for v in dg512 dg1024; do
  KMHG_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "query or diag" > "$OUT/pytest_$v.log" 2>&1 \
    || { echo "pytest $v failed"; tail -30 "$OUT/pytest_$v.log"; exit 1; }
  tail -1 "$OUT/pytest_$v.log"
done
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg512" "KMHG_LIB_VARIANT=dg1024" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg512" "KMHG_LIB_VARIANT=dg1024" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg512" "KMHG_LIB_VARIANT=dg1024" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config5.log"

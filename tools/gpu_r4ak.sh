#!/bin/bash
# Round 4: the query's tile-total scan in one workgroup up to 64 K / 256 K tiles (variants s64k /
# s256k) instead of reduce-then-scan (3 launches) beyond 16 K -- query parity, then the query
# legs at configs 3 (49 K tiles) and 5 (244 K tiles).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4ak
mkdir -p "$OUT"
for v in s64k s256k; do
  KMHG_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "query or config3" > "$OUT/pytest_$v.log" 2>&1 \
    || { echo "pytest $v failed"; tail -30 "$OUT/pytest_$v.log"; exit 1; }
  tail -1 "$OUT/pytest_$v.log"
done
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=s64k" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=s256k" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config5.log"

#!/bin/bash
# Round 4: bucket-aligned count walk over one bucket per tile (KMHG_WALK_B=1 variant library:
# 6 waves per SIMD instead of 3) -- counts parity, then A/B of the counts / reads legs at
# configs 2 and 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4aa
mkdir -p "$OUT"
KMHG_LIB_VARIANT=walkb1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_counts.py tests/test_gpu_sh.py > "$OUT/pytest_walkb1.log" 2>&1 \
  || { echo "pytest failed"; tail -30 "$OUT/pytest_walkb1.log"; exit 1; }
tail -1 "$OUT/pytest_walkb1.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=walkb1" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=walkb1" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"

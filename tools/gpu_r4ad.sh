#!/bin/bash
# Round 4: read k-mer walk reading RK_CH positions' bases and terms together (4 = the library,
# 8 = variant rk8) against the previous per-base walk (prerk) -- read-counting parity, then the
# reads leg A/B at config 2.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4ad
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sh.py tests/test_counts.py > "$OUT/pytest.log" 2>&1 \
  || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
KMHG_LIB_VARIANT=rk8 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sh.py > "$OUT/pytest_rk8.log" 2>&1 \
  || { echo "pytest rk8 failed"; tail -30 "$OUT/pytest_rk8.log"; exit 1; }
tail -1 "$OUT/pytest_rk8.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=rk8" "KMHG_LIB_VARIANT=prerk" -- --no-cpu \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"

#!/bin/bash
# Round-4 GPU pass x: anchor stride 128 (new default) -- query tests, then A/B against 256 and 64.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4x
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multidevice.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
KMHG_LIB_VARIANT=dg256 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "query or diagonal" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_dg256.log" 2>&1 || { echo "dg256 tests failed"; tail -30 "$OUT/pytest_dg256.log"; exit 1; }
tail -1 "$OUT/pytest_dg256.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg256" "KMHG_LIB_VARIANT=dg64" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg256" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=dg256" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

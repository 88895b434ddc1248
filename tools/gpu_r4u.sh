#!/bin/bash
# Round-4 GPU pass u: persistent query probe (next tile's chars prefetched, XCD-contiguous tiles)
# -- query tests, then A/B against the one-workgroup-per-tile probe (variant probe1).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4u
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multidevice.py tests/test_gpu_dist.py tests/test_gpu_device_api.py -m gpu -x -q \
  -k "query or diagonal or fullsize or config or device or shard or rank or golden or edge or random or khash" \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=probe1" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=probe1" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=probe1" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"

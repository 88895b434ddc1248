#!/bin/bash
# Round-4 GPU pass r: two-kernel query emit -- query / fullsize / multi-device tests, then A/B
# against the previous library at configs 2, 3 and 5 (query legs).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4r
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multidevice.py tests/test_gpu_dist.py tests/test_gpu_device_api.py tests/test_gpu_boundary.py tests/test_counts.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preq" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preq" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preq" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"

#!/bin/bash
# Round-3 GPU pass y: the diagonal query probe over 8 consecutive windows per lane
# (diag_resolve8) -- every query test, A/B against the strided probe (KMHG_LIB_VARIANT=pst) at
# config 2 (self + unrelated query) and config 5 (one GPU).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3y
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multidevice.py tests/test_gpu_device_api.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "query or diag or golden or 10mbp or config2 or config3 or config5 or range or shard or multi or device" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=pst" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=pst" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"

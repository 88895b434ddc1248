#!/bin/bash
# Round 4: adaptive diagonal anchors (odd anchors probed only at a tile head without a
# predicting even anchor) -- query parity (incl. the full-size config 3 / 5 digests), then A/B
# against the previous library (preanc; round 2: odd anchors skipped in tiles where no even anchor predicts) at configs 2, 3 and 5.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4ag2
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_device_api.py tests/test_gpu_multidevice.py tests/test_gpu_dist.py \
  tests/test_gpu_fullsize.py -k "query or diag or device or shard or config3 or config5 or config2" \
  > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preanc" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config2.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preanc" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config3.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=preanc" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config5.log"

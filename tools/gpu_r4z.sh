#!/bin/bash
# Round 4: k_read_pairs staged in two halves (6 or 8 workgroups per CU) -- parity (positions / pairs
# readouts incl. the config-4 digest), then A/B against the previous library at config 4.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4z
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_device_api.py tests/test_gpu_fullsize.py -k "pair or pos or config4 or device" \
  > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=pairs8" "KMHG_LIB_VARIANT=prepairs" -- --config 4 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_config4.log"
grep -o '^### .*\|"value": [0-9.]*, "unit": "G\|"kernels_ms": {[^}]*}' "$OUT/ab_config4.log"

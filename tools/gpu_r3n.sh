#!/bin/bash
# Round-3 GPU pass n: fused query A/B; 32-per-thread look-back scan of the radix histograms
# (KMHG_SCAN) -- parity subset, A/B at config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3n
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "multi_pass and bid or 10mbp or golden or query_paths" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_QUERY=classic" "KMHG_QUERY=fused" -- --no-cpu --no-reads \
  || { echo "abq failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/abq.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_SCAN=32" "KMHG_SCAN=8" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
KMHG_SCAN=L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "10mbp" > "$OUT/pytest_L.log" 2>&1 || { echo "tests L failed"; tail -40 "$OUT/pytest_L.log"; exit 1; }
timeout -k 10 700 bash tools/ab.sh "KMHG_SCAN=32" "KMHG_SCAN=L" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

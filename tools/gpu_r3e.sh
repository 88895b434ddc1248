#!/bin/bash
# Round-3 GPU pass e: readout + bucket tests, A/B of build-time tags (word stores), config 4 line.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3e
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "bucket or diagonal or tandem or golden" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUILD_TAGS=1" "KMHG_BUILD_TAGS=0" -- --no-cpu --no-reads \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab.log"
timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > "$OUT/config4.json" \
  2> "$OUT/config4.err" || { echo "config 4 failed"; tail -20 "$OUT/config4.err"; exit 1; }
cat "$OUT/config4.json"

#!/bin/bash
# Round-3 GPU pass c: the whole -m gpu suite, smoke, the default bench, then A/B of the new knobs.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3c
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 700 bash tools/ab.sh "KMHG_BUCKET_TB=256" "KMHG_BUCKET_TB=512" "KMHG_BUCKET_FP=1" \
  "KMHG_BUCKET_TB=512 KMHG_BUCKET_FP=1" "KMHG_BUILD_TAGS=0" "KMHG_H2D=direct" \
  -- --no-cpu --no-reads || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab.log"

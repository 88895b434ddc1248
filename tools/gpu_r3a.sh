#!/bin/bash
# Round-3 first GPU pass: new tests first (fullsize / multidevice / boundary), then the suite,
# smoke and the default bench.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3a
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_multidevice.py \
  tests/test_gpu_boundary.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${KSEL:-not config5}" \
  > "$OUT/pytest_new.log" 2>&1 || { echo "new gpu tests failed"; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -3 "$OUT/pytest_new.log"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  --deselect tests/test_gpu_fullsize.py --deselect tests/test_gpu_multidevice.py \
  --deselect tests/test_gpu_boundary.py > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "gpu tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"

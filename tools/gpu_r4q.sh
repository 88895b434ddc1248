#!/bin/bash
# Round-4 GPU pass q: the whole GPU suite with its slowest tests listed (suite-time budget).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4q
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --durations=40 \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -60 "$OUT/pytest.log"; exit 1; }
tail -50 "$OUT/pytest.log"

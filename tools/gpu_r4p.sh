#!/bin/bash
# Round-4 GPU pass p: part builds read their own windows compacted by V_hist0 -- parts / dist /
# parity tests, then the per-rank step rehearsal with and without the compaction.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4p
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parts.py tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/part_step.py 10 10 > "$OUT/part_step.log" 2>&1 || { echo "part_step failed"; tail -20 "$OUT/part_step.log"; exit 1; }
cat "$OUT/part_step.log"
KMHG_PART_COMPACT=0 timeout -k 10 300 python -u tools/part_step.py 10 10 > "$OUT/part_step_nocompact.log" 2>&1 || { echo "part_step nc failed"; tail -20 "$OUT/part_step_nocompact.log"; exit 1; }
cat "$OUT/part_step_nocompact.log"

#!/bin/bash
# Round-4 GPU pass g: V_bounds_lo folded into the last radix pass (parity + A/B at configs 2/3),
# then the 500 Mbp build with tile-by-tile vs write-combined radix passes (A/B in one run).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4g
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh.py tests/test_counts.py tests/test_gpu_parts.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "multi_pass or bucket_kernels or golden or disorder or 10mbp or sh or count or part" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_FUSE_BOUNDS=1" "KMHG_FUSE_BOUNDS=0" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 1000 bash tools/gpu_r4f.sh || { echo "r4f failed"; exit 1; }

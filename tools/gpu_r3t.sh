#!/bin/bash
# Round-3 GPU pass t: the bucket kernels' stream-order check by shuffles (no neighbour loads
# for one-batch buckets) -- build/parity subset incl. the disorder fallback, A/B against a
# variant without any check (KMHG_LIB_VARIANT=nochk) at config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3t
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "disorder or bucket or multi_pass or 10mbp or golden or config3 or config4 or sh" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=nochk" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_LIB_VARIANT=" "KMHG_LIB_VARIANT=nochk" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

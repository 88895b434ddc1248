#!/bin/bash
# Round-4 GPU pass i: bucket-aligned counts walk (row offsets from the bucket statistics) --
# counts / sh / parity tests, then the counts and reads legs at config 2 and config 3 (A/B
# against the look-back walk), then the 500 Mbp build against the previous commit's library
# (same box: is the slower r4h scatter the box or the code?).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4i
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_counts.py tests/test_gpu_sh.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_COUNT_WALK=b" "KMHG_COUNT_WALK=lb" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_COUNT_WALK=b" "KMHG_COUNT_WALK=lb" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
if [ -f kmer_hasher_amd/libkmhgpu_prev.so ]; then
  timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=prev KMHG_SCATTER_WC=0" -- --config 5 --steps 3 --warmup 1 --no-cpu \
    || { echo "ab5 failed"; exit 1; }
  cp gpurun_out/ab.log "$OUT/ab5.log"
fi

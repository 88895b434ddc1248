#!/bin/bash
# Round-3 GPU pass o: compact 12-B LDS group table (KMHG_BUCKET_C12, 8 workgroups per CU) --
# parity subset incl. the 16-B table and count-only builds, A/B at config 2 and config 3, and
# the LDS atomic probe (tools/lds_atomics).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3o
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sh.py -m gpu -x -v \
  --timeout 300 --timeout-method thread \
  -k "bucket or (multi_pass and bid and lo) or 10mbp or golden or sh or reads" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 bash tools/ab.sh "KMHG_BUCKET_C12=1" "KMHG_BUCKET_C12=0" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_BUCKET_C12=1" "KMHG_BUCKET_C12=0" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 120 ./tools/lds_atomics > "$OUT/lds_atomics.txt" 2>&1 || { echo "lds probe failed"; exit 1; }
cat "$OUT/lds_atomics.txt"

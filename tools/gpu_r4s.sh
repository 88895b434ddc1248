#!/bin/bash
# Round-4 GPU pass s: 2048-window group buckets (variant library bw2048: 3,072-slot LDS tables,
# 4 workgroups per CU, radix halved) -- parity subset on the variant, then A/B at configs 3, 5, 2.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4s
mkdir -p "$OUT"
cd "$REPO"
KMHG_LIB_VARIANT=bw2048 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "multi_pass or bucket_kernels or golden or random_strings or tandem or disorder" \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_variant.log" 2>&1 || { echo "variant tests failed"; tail -40 "$OUT/pytest_variant.log"; exit 1; }
tail -1 "$OUT/pytest_variant.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "multi_pass or bucket_kernels or disorder or build_kind" \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_default.log" 2>&1 || { echo "default tests failed"; tail -40 "$OUT/pytest_default.log"; exit 1; }
tail -1 "$OUT/pytest_default.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=bw2048" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=bw2048" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"
timeout -k 10 400 bash tools/ab.sh "KMHG_X=0" "KMHG_LIB_VARIANT=bw2048" -- --no-cpu --no-reads \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"

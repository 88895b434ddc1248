#!/bin/bash
# Round-3 GPU pass z: persistent prefetching histogram for the later radix passes (k_v2_histp) --
# partition / read-counting / full-size tests, A/B against one workgroup per tile (KMHG_HISTP=0)
# at config 2 and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3z
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sh.py tests/test_counts.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "multi_pass or 10mbp or golden or config2 or config3 or config4 or bucket or sh or count or disorder" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 bash tools/ab.sh "KMHG_HISTP=1" "KMHG_HISTP=0" -- --no-cpu \
  || { echo "ab2 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab2.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_HISTP=1" "KMHG_HISTP=0" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"

#!/bin/bash
# Round-3 GPU pass p: pass-A variants in isolation (tools/lds_atomics: per-wave failure queue),
# phase stamps of the compact-table bucket kernel, 8-wave scatter A/B with bucket-id streams.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3p
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "(multi_pass and bid) or 10mbp" > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 ./tools/lds_atomics > "$OUT/lds_atomics.txt" 2>&1 || { echo "lds probe failed"; exit 1; }
grep "pass A" "$OUT/lds_atomics.txt"
timeout -k 10 200 python tools/stamps.py 10000000 31 > "$OUT/stamps.txt" 2>&1 || { echo "stamps failed"; tail "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
timeout -k 10 500 bash tools/ab.sh "KMHG_SC8=0" "KMHG_SC8=1" -- --no-cpu --no-reads \
  || { echo "ab failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab_sc8.log"

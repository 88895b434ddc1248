#!/bin/bash
# Round-4 GPU pass h: bucket starts from the histograms for every pass count (one level per
# radix pass, fused), count.kmers rows in slot order with order keys; the whole GPU suite, then
# A/B at config 3 (2 passes vs 3 narrower passes, fused vs unfused levels) and the 500 Mbp build.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4h
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_MAXR=47" "KMHG_FUSE_BOUNDS=0" -- --config 3 --steps 5 --warmup 2 --no-cpu --no-reads \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_X=0" "KMHG_FUSE_BOUNDS=0" -- --config 5 --steps 3 --warmup 1 --no-cpu \
  || { echo "ab5 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab5.log"
python3 - "$OUT/ab5.log" <<'PY'
import json, sys
cur = None
for line in open(sys.argv[1]):
    if line.startswith("###"):
        cur = line.strip(); continue
    if line.startswith("{"):
        d = json.loads(line); b = d.get("index_build") or {}
        print(cur, "query", d["value"], "build_ms", b.get("ms_per_build"), "ksum", b.get("kernel_ms_sum"), b.get("kernels_ms_per_build"))
PY

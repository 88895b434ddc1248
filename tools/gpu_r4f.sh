#!/bin/bash
# Round-4 GPU pass f: the 500 Mbp build (config 5's index) with the tile-by-tile and the
# write-combined radix passes (radix 79, three passes), A/B in one run.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4f
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 1000 bash tools/ab.sh "KMHG_SCATTER_WC=0" "KMHG_SCATTER_WC=1 KMHG_SCATTER_WC_GEOM=0" "KMHG_SCATTER_WC=1 KMHG_SCATTER_WC_GEOM=1" -- --config 5 --steps 3 --warmup 1 --no-cpu \
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

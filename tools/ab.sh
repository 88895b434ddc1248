#!/bin/bash
# A/B timing of bench.py under environment variants (run through gpurun).
#   bash tools/ab.sh "<env assignments A>" "<env assignments B>" ... -- [bench args]
# Each variant runs twice, interleaved; the JSON lines land in gpurun_out/ab.log.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ $# -gt 0 ] && shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--no-cpu)
: > "$OUT/ab.log"
for rep in 1 2; do
  for v in "${VARS[@]}"; do
    echo "### [$v] rep $rep" >> "$OUT/ab.log"
    env $v timeout -k 10 240 python3 "$REPO/bench.py" "${ARGS[@]}" >> "$OUT/ab.log" 2>&1 || { echo "FAILED [$v]"; exit 1; }
  done
done
python3 - "$OUT/ab.log" <<'PY'
import json, sys
cur = None
for line in open(sys.argv[1]):
    if line.startswith("###"):
        cur = line.strip(); continue
    if line.startswith("{"):
        d = json.loads(line)
        km = d.get("kernels_ms", {})
        rd = d.get("reads", {})
        print(cur, "value", d["value"], "ms", d["ms_per_step"], "q", d.get("query", {}).get("value"), "qu", d.get("query", {}).get("unrelated", {}).get("value"),
              "reads", rd.get("value"), "walk", rd.get("kernels_ms_per_step", {}).get("k_count_walk"),
              "rk", rd.get("kernels_ms_per_step", {}).get("k_read_kmers_emit"),
              "counts", d.get("counts", {}).get("value"),
              "counts_k", d.get("counts", {}).get("kernels_ms_per_step"),
              "order_ms", d.get("counts", {}).get("first_readout_row_order", {}).get("ms"),
              "depth", d.get("depth", {}).get("value"),
              "dprobe", d.get("depth", {}).get("kernels_ms_per_step", {}).get("k_depth_probe"),
              "hb_build_ms", d.get("host_boundary", {}).get("build", {}).get("ms"),
              "hb_query_ms", d.get("host_boundary", {}).get("query", {}).get("ms"),
              "q_first_new", d.get("query", {}).get("first_query_new_index_ms"),
              " ".join(f"{k}={v:.4f}" for k, v in sorted(km.items())))
PY

#!/bin/bash
# Round-4 GPU pass m: count.kmers row order as a permutation (rows never move): counts / sh /
# R-glue tests, then the default bench (counts leg + its one-time readout ordering) and config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4m
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_counts.py tests/test_gpu_sh.py tests/test_r_glue.py tests/test_gpu_boundary.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --no-cpu > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "bench failed"; tail -20 "$OUT/bench2.err"; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu --no-reads > "$OUT/bench3.json" 2> "$OUT/bench3.err" || { echo "bench3 failed"; tail -20 "$OUT/bench3.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
for f in ("bench2", "bench3"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    c = d.get("counts", {})
    print(f, d["value"], "counts", c.get("value"), c.get("kernels_ms_per_step"), c.get("first_readout_row_order"))
PY

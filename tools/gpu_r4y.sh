#!/bin/bash
# Round 4: zero-copy query rows (DeviceQuery.rows_view) -- device API tests, config 5 bench.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=$REPO/gpurun_out/r4y
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_device_api.py tests/test_gpu_dist.py > "$OUT/pytest.log" 2>&1 \
  || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu > "$OUT/config5.json" \
  2> "$OUT/config5.err" || { echo "config 5 failed"; tail -20 "$OUT/config5.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/config5.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['kernels_ms'],d['config']['phases_ms'])"

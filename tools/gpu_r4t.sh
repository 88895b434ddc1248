#!/bin/bash
# Round-4 GPU pass t: LDS-staged part compaction and the two-source count-row store -- parts /
# counts / sh tests, the part-step rehearsal, and the counts leg at config 3.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4t
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parts.py tests/test_counts.py tests/test_gpu_sh.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/part_step.py 10 10 > "$OUT/part_step.log" 2>&1 || { echo "part_step failed"; tail -20 "$OUT/part_step.log"; exit 1; }
cat "$OUT/part_step.log"
timeout -k 10 300 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu --no-reads > "$OUT/bench3.json" 2> "$OUT/bench3.err" || { echo "bench3 failed"; tail -20 "$OUT/bench3.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench3.json')); c=d['counts']
print('config3', d['value'], 'query', d['query']['value'], d['query']['kernels_ms'], 'counts', c['value'], c['kernels_ms_per_step'])"

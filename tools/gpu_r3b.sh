#!/bin/bash
# Round-3 GPU pass b: part / dist tests, then the config 3 / 4 / 5 bench lines (CPU baselines).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r3b
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parts.py tests/test_gpu_dist.py \
  tests/test_gpu_fullsize.py -k "parts or part_index or dist or owner or ranks or config5" \
  -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config$c.json" \
    2> "$OUT/config$c.err" || { echo "config $c failed"; tail -20 "$OUT/config$c.err"; exit 1; }
  cat "$OUT/config$c.json"
done
# N > 1 bench code rehearsed on one GPU: two ranks on cuda:0 over gloo (config 2 + sharded build)
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  --backend gloo --rehearse --no-cpu --no-reads > "$OUT/rehearse2.json" 2> "$OUT/rehearse2.err" \
  || { echo "rehearsal failed"; tail -30 "$OUT/rehearse2.err"; exit 1; }
cat "$OUT/rehearse2.json"

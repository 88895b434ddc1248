#!/bin/bash
# Round-6 evidence on the GPU box (through gpurun): part 1 = GPU suite, smoke, the default bench
# line as the driver runs it, the other configs' lines, and the N > 1 rehearsals (RCCL at world
# size 1, gloo with two ranks on one GPU); part 2 = tools/profile_all.sh A (PMC of config 2, its
# side legs, config 3 and the general lookup), part 2B = tools/profile_all.sh B (config 4, config 5
# and the out-of-cache record).
#   bash tools/evidence_r6.sh <tag> 1|2A|2B
set -uo pipefail
TAG=${1:-r6h}; PART=${2:-1}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
OUT=gpurun_out/ev_$TAG
mkdir -p "$OUT"
if [ "$PART" = 1 ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" \
    2> "$OUT/bench_default.err" || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 1; }
  for c in 3 4 5; do
    timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/bench_config$c.json" \
      2> "$OUT/bench_config$c.err" || { echo "config $c failed"; tail -20 "$OUT/bench_config$c.err"; exit 1; }
  done
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --backend nccl --dist --steps 10 \
    --no-cpu --no-reads > "$OUT/rehearse_nccl_n1.json" 2> "$OUT/rehearse_nccl_n1.err" \
    || { echo "nccl rehearsal failed"; tail -20 "$OUT/rehearse_nccl_n1.err"; exit 1; }
  # bench.py starts the two ranks itself (no launcher): the driver's `bench.py --gpus N` form
  timeout -k 10 400 python bench.py --gpus 2 --backend gloo --rehearse \
    --steps 5 --no-cpu --no-reads > "$OUT/rehearse_gloo_n2.json" 2> "$OUT/rehearse_gloo_n2.err" \
    || { echo "gloo rehearsal failed"; tail -20 "$OUT/rehearse_gloo_n2.err"; exit 1; }
  echo "evidence part 1 done"
else
  bash tools/profile_all.sh "$TAG" ${PART#2} || exit 1
  echo "evidence part 2 done"
fi

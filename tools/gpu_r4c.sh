#!/bin/bash
# Round-4 GPU pass c: pruned library + write-combined radix passes (k_v2_scatter_wc) + runtime
# lane-order self-check: parity (partition / bucket / ballot / fallback / full-size / R glue /
# multi-device / parts), config-3 A/B of the write-combined passes, a config-2 check and the
# N = 2 owner-computes headline rehearsed with gloo on the one GPU.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4c
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_r_glue.py \
  tests/test_gpu_multidevice.py tests/test_gpu_parts.py tests/test_gpu_dist.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${R4C_K:-bucket_kernels or multi_pass or disorder or build_kind or lane_order or golden or config3 or config2 or config4 or glue or multidevice or kmhg_devices or part or dist}" \
  > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 700 bash tools/ab.sh "KMHG_SCATTER_WC=0" "KMHG_SCATTER_WC=1" -- --config 3 --steps 5 --warmup 2 --no-cpu \
  || { echo "ab3 failed"; exit 1; }
cp gpurun_out/ab.log "$OUT/ab3.log"
timeout -k 10 300 python3 bench.py --no-cpu > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "bench2 failed"; tail -5 "$OUT/bench2.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench2.json').read().strip().splitlines()[-1]);print('config2',d['value'],d['ms_per_step'],d['build_path'],d.get('kernels_ms'))"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --backend gloo --rehearse --steps 5 --warmup 2 --no-cpu --no-reads > "$OUT/rehearse_n2.json" 2> "$OUT/rehearse_n2.err" \
  || { echo "rehearsal failed"; tail -20 "$OUT/rehearse_n2.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/rehearse_n2.json').read().strip().splitlines()[-1]);print('n2',d['value'],d['config']['parallelism'],d['sharded_build'].get('assemble_ms'),d['replicas']['value'])"

#!/bin/bash
# SQ-level counters of bench.py kernels (occupancy / stall attribution), two --pmc passes.
#   bash tools/pmc_sq.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-sq}; shift || true
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 5 --warmup 1 --profile)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU \
  --output-format csv -d "$OUT/p1" -o run -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/p2" -o run -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/p2.log" 2>&1
echo "pmc $TAG done"
# L2 request sizes / hit rate (random slot probes: 32/64/128-B fills?)
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d "$OUT/p3" -o run -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/p3.log" 2>&1
echo "pmc $TAG tcc done"

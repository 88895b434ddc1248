#!/bin/bash
# L2 / fabric read counters of the query probe (diagonal vs table-only), run through gpurun.
#   bash tools/pmc_query.sh <tag>
set -euo pipefail
TAG=${1:-q}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/pmcq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=(--steps 5 --warmup 1 --profile)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f_diag" -o run \
  -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/f_diag.log" 2>&1
KMHG_QUERY_DIAG=0 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f_table" -o run \
  -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/f_table.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o run \
  -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/tcc.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d "$OUT/tcp" -o run \
  -- python3 "$REPO/bench.py" "${ARGS[@]}" > "$OUT/tcp.log" 2>&1
echo "pmc_query $TAG done"

#!/bin/bash
# Where the 500 Mbp build's device allocations come from: build-only timing with the pool's
# best-fit reuse on / off (test build: KMHG_POOL_BESTFIT=0), every hipMalloc traced
# (KMHG_POOL_TRACE=1, stderr).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for bf in 1 0; do
    echo "### bestfit=$bf rep $rep"
    KMHG_LIB_VARIANT=test KMHG_POOL_BESTFIT=$bf KMHG_POOL_TRACE=1 timeout -k 10 120 \
      python tools/build_only.py 500 31 10 2> gpurun_out/pool_trace_bf${bf}_r${rep}.err
    grep -c "hipMalloc" gpurun_out/pool_trace_bf${bf}_r${rep}.err || true
  done
done

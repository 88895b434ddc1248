#!/bin/bash
# Probe-kernel counters under two table layouts (CAS build vs sorted build).
#   bash tools/pmc_probe.sh   (through gpurun)
set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/pmc_probe
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in group sort; do
  KMHG_BUCKET=$v timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD \
    --output-format csv -d "$OUT/$v" -o run -- python3 "$REPO/bench.py" --steps 3 --warmup 1 --profile > "$OUT/$v.log" 2>&1
done
echo done

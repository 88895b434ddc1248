#!/bin/bash
# Round-4 GPU pass e: SQ counters of the config-3 build (key streams vs bucket-id streams), then
# config 5 through the compiled reference on this box's host (tools/ref_config5.py, CPU only).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/r4e
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for bid in ${R4E_BIDS:-0 1}; do
  KMHG_BUILD_BID=$bid timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU \
    --output-format csv -d "$OUT/b${bid}p1" -o run -- python3 "$REPO/bench.py" --config ${R4E_CFG:-3} --steps 3 --warmup 1 --profile > "$OUT/b${bid}p1.log" 2>&1 || { echo "pmc1 failed"; tail -5 "$OUT/b${bid}p1.log"; exit 1; }
  KMHG_BUILD_BID=$bid timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/b${bid}p2" -o run -- python3 "$REPO/bench.py" --config ${R4E_CFG:-3} --steps 3 --warmup 1 --profile > "$OUT/b${bid}p2.log" 2>&1 || { echo "pmc2 failed"; tail -5 "$OUT/b${bid}p2.log"; exit 1; }
done
echo "pmc done"
[ -n "${R4E_SKIP_REF:-}" ] && exit 0
cd "$REPO"
timeout -k 10 900 python3 -u tools/ref_config5.py "$OUT/ref_config5.json" > "$OUT/ref_config5.log" 2>&1 || { echo "ref config5 failed"; tail -5 "$OUT/ref_config5.log"; exit 1; }
cat "$OUT/ref_config5.json"

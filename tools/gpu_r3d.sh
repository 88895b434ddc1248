#!/bin/bash
# Round-3 GPU pass d: rocprofv3 kernel-trace + PMC (FETCH / WRITE in separate passes) at
# config 3 (100 Mbp), config 4 (the pair readout) and config 5 (500 Mbp), and the unrelated-query
# probe's bytes per miss.  Summaries: tools/pmc_summary.py on this side.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
for c in 3 4 5; do
  bash tools/profile.sh rd3c$c --config $c --steps 3 --warmup 1 --profile || { echo "profile $c failed"; exit 1; }
done
OUT=$REPO/gpurun_out/prof_rd3u
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run \
  -- python3 "$REPO/tools/query_unrelated.py" > "$OUT/ktrace.log" 2>&1 || { echo "u ktrace failed"; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 "$REPO/tools/query_unrelated.py" > "$OUT/pmc_fetch.log" 2>&1 || { echo "u fetch failed"; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 "$REPO/tools/query_unrelated.py" > "$OUT/pmc_write.log" 2>&1 || { echo "u write failed"; exit 1; }
echo "pass d done"

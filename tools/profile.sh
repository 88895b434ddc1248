#!/bin/bash
# Kernel-trace + PMC profile of bench.py on the GPU box (run through gpurun).
#   bash tools/profile.sh <tag> [bench args...]
#   PROG=tools/query_unrelated.py bash tools/profile.sh <tag> [args...]   (another driver script)
# Writes gpurun_out/prof_<tag>/...; tools/pmc_summary.py turns the CSVs into profiles/.
# Counters follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE in separate --pmc passes
# (TCC slots), no tracing domains beside --pmc.
set -euo pipefail
TAG=${1:-r01}; shift || true
REPO=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 10 --warmup 2 --profile)
PROG=${PROG:-bench.py}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run \
  -- python3 "$REPO/$PROG" "${ARGS[@]}" > "$OUT/ktrace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 "$REPO/$PROG" "${ARGS[@]}" > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 "$REPO/$PROG" "${ARGS[@]}" > "$OUT/pmc_write.log" 2>&1
echo "profile $TAG done"

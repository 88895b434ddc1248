#!/bin/bash
# Regenerate every PMC / kernel-trace profile the bench lines read (profiles/pmc_*.json), with the
# shipping library, on the GPU box (through gpurun).  Part A: config 2, its side legs, config 3,
# the general lookup; part B: config 4, config 5 and the out-of-cache record.
#   bash tools/profile_all.sh <tag-prefix> A|B
# then on the CPU side: python tools/pmc_summary.py <tag> <pmc name> for each (tools/profile_all.sh
# prints the commands).
set -uo pipefail
P=${1:-r5}; PART=${2:-A}
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
run() { local tag=$1; shift; bash tools/profile.sh "$tag" "$@" || { echo "profile $tag failed"; exit 1; }; echo "profile $tag ok"; }
if [ "$PART" = A ]; then
  run ${P}p2 --steps 10 --warmup 2 --profile
  run ${P}plegs --steps 3 --warmup 1 --no-cpu --no-large
  run ${P}p3 --config 3 --steps 3 --warmup 1 --profile --no-cpu
  PROG=tools/query_unrelated.py run ${P}punrel --steps 10
else
  run ${P}p4 --config 4 --steps 3 --warmup 1 --profile --no-cpu
  run ${P}p5 --config 5 --steps 3 --warmup 1 --no-cpu
  run ${P}plarge --only-large --steps 3 --warmup 1
  PROG=tools/query_unrelated.py run ${P}plargeunrel --L 500000000 --steps 10
fi

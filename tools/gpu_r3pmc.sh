#!/bin/bash
# Round-3 PMC + kernel-trace profiles of configs 3 and 5 with the final round-3 kernels
# (tools/profile.sh; tools/pmc_summary.py turns them into profiles/pmc_config{3,5}.json).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/profile.sh rd3f3 --config 3 --steps 3 --warmup 1 --profile --no-cpu || { echo "profile 3 failed"; exit 1; }
bash tools/profile.sh rd3f5 --config 5 --steps 2 --warmup 1 --profile --no-cpu || { echo "profile 5 failed"; exit 1; }
echo "pmc done"

#!/bin/bash
# Round-4 closing evidence, part 2: rocprofv3 kernel traces + FETCH / WRITE PMC of config 2, the
# side legs and config 3 (tools/profile.sh; tools/pmc_summary.py turns them into profiles/).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/profile.sh rd4end2 --steps 10 --warmup 2 --profile || { echo "profile 2 failed"; exit 1; }
bash tools/profile.sh rd4endlegs --steps 3 --warmup 1 --no-cpu || { echo "profile legs failed"; exit 1; }
bash tools/profile.sh rd4end3 --config 3 --steps 3 --warmup 1 --profile --no-cpu || { echo "profile 3 failed"; exit 1; }
echo "profiles done"

#!/bin/bash
# Round-4 profiles (k): rocprofv3 kernel trace + FETCH/WRITE PMC passes of the default bench,
# of the side legs (counts / reads / depth at config 2) and of config 3's build.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/profile.sh rd4k2 --steps 10 --warmup 2 --profile || { echo "profile 2 failed"; exit 1; }
bash tools/profile.sh rd4klegs --steps 3 --warmup 1 --no-cpu || { echo "profile legs failed"; exit 1; }
bash tools/profile.sh rd4k3 --config 3 --steps 3 --warmup 1 --profile --no-cpu || { echo "profile 3 failed"; exit 1; }
echo "profiles done"

#!/bin/bash
# Round-4 closing evidence (final library, adaptive anchors), part 2: rocprofv3 kernel traces + FETCH / WRITE PMC of config 2, the
# side legs and config 3 (tools/profile.sh; tools/pmc_summary.py turns them into profiles/).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-/root/repo}
cd "$REPO"
bash tools/profile.sh rd4last2 --steps 10 --warmup 2 --profile || { echo "profile 2 failed"; exit 1; }
bash tools/profile.sh rd4lastlegs --steps 3 --warmup 1 --no-cpu || { echo "profile legs failed"; exit 1; }
bash tools/profile.sh rd4last3 --config 3 --steps 3 --warmup 1 --profile --no-cpu || { echo "profile 3 failed"; exit 1; }
echo "profiles done"
# bench lines again after the query roofline's pricing change (bench.py only; same library)
OUT=$REPO/gpurun_out/cfg_rd4last
mkdir -p "$OUT"
for c in 2 3 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 > "$OUT/config${c}_b.json" \
    2> "$OUT/config${c}_b.err" || { echo "config $c failed"; tail -20 "$OUT/config${c}_b.err"; exit 1; }
  echo "config $c ok"
done

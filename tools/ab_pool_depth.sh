#!/bin/bash
# A/B of the device pool's depth (blocks per size class before an allocation waits for queued
# work): asynchronous back-to-back builds as bench.py times them, build only, test build
# (KMHG_POOL_DEPTH=1 / 2), interleaved on one box.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for d in 1 2; do
    for cfg in "10 31 50" "100 21 20" "500 31 10"; do
      KMHG_LIB_VARIANT=test KMHG_POOL_DEPTH=$d timeout -k 10 120 python tools/build_only.py $cfg 2>/dev/null | sed "s/^/$rep depth=$d /"
    done
  done
done

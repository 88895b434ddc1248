#!/bin/bash
# A/B of the radix plan (test build: KMHG_MAXR caps the radix) at config 3 (100 Mbp, k = 21:
# 2 passes of radix 313 by default, 3 of radix 47 under a cap) -- build only, interleaved.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for m in "" 47 64; do
    KMHG_LIB_VARIANT=test KMHG_MAXR=$m timeout -k 10 120 python tools/build_only.py 100 21 20 2>/dev/null | sed "s/^/$rep maxr=${m:-default} /"
  done
done

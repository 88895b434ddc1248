#!/bin/bash
# A/B of the query probe's phase-2 unroll (tag-group loads in flight per lane), interleaved runs
# on one box: general lookup at 500 Mbp (beyond the cache) and 10 Mbp (config 2).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for v in "" p2u4 p2u8; do
    for L in 500000000 10000000; do
      KMHG_LIB_VARIANT=$v timeout -k 10 120 python tools/query_unrelated.py --L $L --steps 20 | sed "s/^/$rep ${v:-base} /"
    done
  done
done

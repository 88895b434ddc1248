"""General-lookup query for rocprofv3 PMC passes (GPU box): an index of config 2's sequence
(10 Mbp, k=31; or --L) queried K times with an unrelated i.i.d. sequence of the same length, so
every window misses and goes through the slot tags.  Prints one JSON line: the probe's average
time and the misses per query, so a PMC pass's FETCH_SIZE per launch gives the bytes per miss.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/x -- python3 tools/query_unrelated.py --steps 10
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from kmer_hasher_amd import synth  # noqa: E402
from kmer_hasher_amd import device as D  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=10_000_000)
ap.add_argument("--k", type=int, default=31)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--seed-index", type=int, default=None, help="default: 1 (4 at --L 500000000)")
ap.add_argument("--seed-query", type=int, default=None, help="default: 101 (6 at --L 500000000)")
a = ap.parse_args()
big = a.L == 500_000_000               # bench.py large.unrelated: A seed 4, query seed 6
sa = a.seed_index if a.seed_index is not None else (4 if big else 1)
sq = a.seed_query if a.seed_query is not None else (6 if big else 101)
seq = torch.from_numpy(synth.iid(a.L, sa)).cuda()
other = torch.from_numpy(synth.iid(a.L, sq)).cuda()
idx = D.DeviceIndex.build(seq, a.k)
idx.info()
q = idx.query(other, a.k)
H = q.n_rows
q.free()
D.timing_enable(True)
D.timing_reset()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    idx.query(other, a.k).free()
torch.cuda.synchronize()
t = (time.perf_counter() - t0) / a.steps
per = {n: v[1] / v[0] for n, v in D.timing_report().items() if v[0]}
print(json.dumps({"L": a.L, "k": a.k, "windows": a.L - a.k + 1, "rows": H,
                  "ms_per_query": round(t * 1e3, 4),
                  "kernels_ms": {n: round(v, 5) for n, v in per.items()}}))
idx.free()

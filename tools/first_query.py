"""Where the first seq.kmer.pos call of an index goes (config 2 self dot plot, GPU box): the
first query of a fresh index in a fresh process (device pool cold for the query's buffers), the
first query of a second index (pool warm: only the per-index diagonal-path preparation is left),
and a steady-state query, each with the kernels it ran (HIP events, kmhg_timing_*)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from kmer_hasher_amd import synth  # noqa: E402
from kmer_hasher_amd import device as D  # noqa: E402

k = 31
seq = torch.from_numpy(synth.iid(10_000_000, 1)).cuda()
stream = torch.cuda.current_stream()
out = {}


def timed_query(idx, label):
    D.timing_enable(True)
    D.timing_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = idx.query(seq, k, stream)
    q.free()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    kt = D.timing_report()
    D.timing_enable(False)
    out[label] = {"ms": round(t * 1e3, 3),
                  "kernels_ms": {n: round(v[1], 4) for n, v in kt.items() if v[0]}}


a = D.DeviceIndex.build(seq, k, stream)
a.info()
timed_query(a, "first_query_cold_pool")
timed_query(a, "second_query")
b = D.DeviceIndex.build(seq, k, stream)
b.info()
timed_query(b, "first_query_warm_pool")
for _ in range(5):
    b.query(seq, k, stream).free()
timed_query(b, "steady")
print(json.dumps(out))

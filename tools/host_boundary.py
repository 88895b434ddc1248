"""PCIe-inclusive R-API rates (host sequence in, host rows out) on cuda:0, for A/B of the
D2H staging knobs (KMHG_D2H=direct, KMHG_D2H_THREADS=n).  Also times a bare first touch of a
fresh host array of the rows' size, the floor any host result pays.
    python tools/host_boundary.py [calls]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import torch
    assert torch.cuda.is_available()
    from kmer_hasher_amd import api, synth
    seq = synth.iid(10_000_000, 1).tobytes()
    k = 31
    ptr = api.make_kmer_hash(seq, k)
    rows = api.seq_kmer_pos(ptr, seq, k)
    t0 = time.perf_counter()
    for _ in range(calls):
        rows = api.seq_kmer_pos(ptr, seq, k)
    t_q = (time.perf_counter() - t0) / calls
    t0 = time.perf_counter()
    for _ in range(calls):
        a = np.empty(rows.size, np.int32)
        a[::1024] = 0                                 # one store per 4-KiB page
    t_touch = (time.perf_counter() - t0) / calls
    ptr.free()
    print(json.dumps({"env": {e: os.environ.get(e) for e in ("KMHG_D2H", "KMHG_D2H_THREADS")},
                      "query_ms": round(t_q * 1e3, 3), "rows": int(rows.shape[0]),
                      "first_touch_ms": round(t_touch * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()

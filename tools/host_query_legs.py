"""Where the R-API query's host time goes (config 2: 10 Mbp self query, 10 M rows), one call at
a time: the sequence argument, kmhg_query_run (H2D + device query), the host matrix's
allocation, kmhg_query_fill (D2H into it), kmhg_query_free, and the release of the previous
call's matrix -- the legs of api.seq_kmer_pos (the .Call path of src/kmer_hash.c:1151-1172).
    python tools/host_query_legs.py [calls]"""
import ctypes as C
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
    from kmer_hasher_amd import _lib, api, synth
    seq = synth.iid(10_000_000, 1).tobytes()
    k = 31
    ptr = api.make_kmer_hash(seq, k)
    L = _lib.lib()
    legs = {n: 0.0 for n in ("as_bytes", "query_run", "alloc", "fill", "query_free", "release",
                             "whole_api_call")}
    prev = api.seq_kmer_pos(ptr, seq, k)
    for _ in range(calls):
        t0 = time.perf_counter()
        b = api._as_seq_bytes(seq, "x")
        t1 = time.perf_counter()
        q, h = C.c_void_p(), C.c_int64()
        _lib.check(L.kmhg_query_run(ptr.handle, b, len(b), k, C.byref(q), C.byref(h)))
        t2 = time.perf_counter()
        rows = np.empty(2 * h.value, np.int32)
        t3 = time.perf_counter()
        _lib.check(L.kmhg_query_fill(q, rows.ctypes.data))
        t4 = time.perf_counter()
        L.kmhg_query_free(q)
        t5 = time.perf_counter()
        del prev
        t6 = time.perf_counter()
        prev = rows
        for n, dt in (("as_bytes", t1 - t0), ("query_run", t2 - t1), ("alloc", t3 - t2),
                      ("fill", t4 - t3), ("query_free", t5 - t4), ("release", t6 - t5)):
            legs[n] += dt
    del prev
    t0 = time.perf_counter()
    for _ in range(calls):
        r = api.seq_kmer_pos(ptr, seq, k)
        del r
    legs["whole_api_call"] = time.perf_counter() - t0
    rows_kept = None
    t0 = time.perf_counter()
    for _ in range(calls):
        rows_kept = api.seq_kmer_pos(ptr, seq, k)      # the previous result freed on rebind
    legs["whole_api_call_rebind"] = time.perf_counter() - t0
    ptr.free()
    print(json.dumps({"calls": calls, "rows": int(rows_kept.shape[0]),
                      "legs_ms": {n: round(v / calls * 1e3, 3) for n, v in legs.items()}}),
          flush=True)


if __name__ == "__main__":
    main()

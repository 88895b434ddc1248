"""kmhg_query_fill into a fresh host matrix with the rows crossing PCIe as diagonal runs
(expanded by host threads) against the plain staged copy (KMHG_HOST_RUNS=0, test build), A/B in
one process: config 2's self dot plot (10 Mbp, 10 M rows) and config 5's related query
(500 Mbp, 376 M rows).  numpy's own huge-page hint is turned off (R's allocMatrix gives plain
malloc memory); the library asks for huge pages itself.
    python tools/host_runs_probe.py [reps]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    import torch
    assert torch.cuda.is_available()
    try:
        from numpy._core.multiarray import _set_madvise_hugepage
    except ImportError:
        from numpy.core.multiarray import _set_madvise_hugepage
    _set_madvise_hugepage(False)
    from kmer_hasher_amd import _lib, synth
    from kmer_hasher_amd.device import DeviceIndex
    out = {}
    with _lib.using_test_build() as L:
        for name, n, derived in (("config2_self", 10_000_000, False),
                                 ("config5_related", 500_000_000, True)):
            a = synth.iid(n, 4)
            ta = torch.from_numpy(a).cuda()
            tb = torch.from_numpy(synth.derived(a, 5)).cuda() if derived else ta
            del a
            idx = DeviceIndex.build(ta, 31)
            q = idx.query(tb, 31)
            H = q.n_rows
            res = {"rows": H}
            for mode in ("runs", "plain", "runs", "plain"):
                os.environ["KMHG_HOST_RUNS"] = "1" if mode == "runs" else "0"
                ts = []
                for _ in range(reps):
                    m = np.empty(2 * H, np.int32)
                    t0 = time.perf_counter()
                    _lib.check(L.kmhg_query_fill(q._h, C.c_void_p(m.ctypes.data)))
                    ts.append(time.perf_counter() - t0)
                    del m
                res.setdefault(mode + "_ms", []).append(round(min(ts) * 1e3, 3))
            out[name] = res
            print(json.dumps({name: res}), flush=True)
            q.free()
            idx.free()
            del ta, tb
            torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

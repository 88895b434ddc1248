"""What freeing an 80 MB result matrix costs the host, by how its pages were written: one thread
(numpy fill), the library's staged copy (KMHG_HOST_RUNS=0: 8 copy threads) or its run expansion
(16 threads), with and without huge pages.  The R API's matrix is freed by R's collector; this
asks whether the way the library fills it changes that cost.
    python tools/release_probe.py [reps]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import torch
    assert torch.cuda.is_available()
    try:
        from numpy._core.multiarray import _set_madvise_hugepage
    except ImportError:
        from numpy.core.multiarray import _set_madvise_hugepage
    from kmer_hasher_amd import _lib, synth
    from kmer_hasher_amd.device import DeviceIndex
    out = {}
    with _lib.using_test_build() as L:
        seq = torch.from_numpy(synth.iid(10_000_000, 1)).cuda()
        idx = DeviceIndex.build(seq, 31)
        q = idx.query(seq, 31)
        H = q.n_rows
        for hint in (False, True):
            _set_madvise_hugepage(hint)
            for how in ("numpy_fill", "staged_copy", "run_expand"):
                rel, fill = [], []
                for _ in range(reps):
                    a = np.empty(2 * H, np.int32)
                    t0 = time.perf_counter()
                    if how == "numpy_fill":
                        a.fill(1)
                    else:
                        os.environ["KMHG_HOST_RUNS"] = "0" if how == "staged_copy" else "1"
                        _lib.check(L.kmhg_query_fill(q._h, C.c_void_p(a.ctypes.data)))
                    t1 = time.perf_counter()
                    del a
                    t2 = time.perf_counter()
                    fill.append(t1 - t0)
                    rel.append(t2 - t1)
                out[f"{how}{'_numpy_hint' if hint else ''}"] = {
                    "fill_ms": round(min(fill) * 1e3, 3), "release_ms": round(min(rel) * 1e3, 3),
                    "release_med_ms": round(sorted(rel)[len(rel) // 2] * 1e3, 3)}
        q.free()
        idx.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

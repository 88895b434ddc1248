"""kmer.pos(opt) into fresh host matrices (kmhg_positions_fill, the R API's readout) against the
same readout into HBM (kmhg_positions_fill_device), config 4's repeat-rich 40 Mbp index (k = 31,
686 M pair rows).  numpy's own huge-page hint is off (R's allocMatrix gives plain malloc
memory).  Runs on the test build, which reads the A/B knobs from the environment;
`--no-host-pairs`: KMHG_HOST_PAIRS=0 (pair rows copied).
    python tools/host_readout_probe.py [opt] [reps] [--no-host-pairs]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    opt = int(args[0]) if args else 14
    reps = int(args[1]) if len(args) > 1 else 3
    plain = "--no-host-pairs" in sys.argv
    if plain:
        os.environ["KMHG_HOST_PAIRS"] = "0"
    import torch
    assert torch.cuda.is_available()
    try:
        from numpy._core.multiarray import _set_madvise_hugepage
    except ImportError:
        from numpy.core.multiarray import _set_madvise_hugepage
    _set_madvise_hugepage(False)
    from kmer_hasher_amd import _lib, synth
    from kmer_hasher_amd.device import DeviceIndex
    with _lib.using_test_build():               # (reads KMHG_HOST_PAIRS / KMHG_HOST_NT)
        L = _lib.lib()
        seq = torch.from_numpy(synth.config4(40_000_000, 3)).cuda()
        idx = DeviceIndex.build(seq, 31)
        idx.info()
        nk, npos, npair, ncnt = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check(L.kmhg_positions_size(idx.handle, opt, C.byref(nk), C.byref(npos),
                                         C.byref(npair), C.byref(ncnt)))
        res = {"opt": opt, "pos_rows": npos.value, "pair_rows": npair.value,
               "host_pairs": not plain}
        idx.positions(opt)                      # the readout's one-time ordering + pools
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = idx.positions(opt)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del out
        res["device_ms"] = round(min(ts) * 1e3, 3)
        ts = []
        for _ in range(reps):
            pos = np.empty(2 * npos.value, np.int32) if opt & 2 else None
            pairs = np.empty(3 * npair.value, np.int32) if opt & 4 else None
            cnt = np.empty(ncnt.value, np.int32) if opt & 8 else None

            def ptr(a):
                return C.c_void_p(a.ctypes.data) if a is not None and a.size else None

            t0 = time.perf_counter()
            _lib.check(L.kmhg_positions_fill(idx.handle, opt, None, ptr(pos), ptr(pairs),
                                             ptr(cnt)))
            ts.append(time.perf_counter() - t0)
            if pairs is not None:
                res["pairs_sum"] = int(pairs[::97].astype(np.int64).sum())
            del pos, pairs, cnt
        res["host_ms"] = round(min(ts) * 1e3, 3)
        idx.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

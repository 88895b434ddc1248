"""Host-side cost of one synchronous seq.kmer.pos query on the GPU box (config 2 self dot plot):
the period of back-to-back calls through the Python wrapper and through bare ctypes, the
device time of the query's kernels, and the cost of a stream synchronize on an idle stream --
to see how much of a query's period the host turnaround takes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import torch  # noqa: E402
from kmer_hasher_amd import _lib, synth  # noqa: E402
from kmer_hasher_amd import device as D  # noqa: E402

k = 31
seq = torch.from_numpy(synth.iid(10_000_000, 1)).cuda()
stream = torch.cuda.current_stream()
idx = D.DeviceIndex.build(seq, k, stream)
idx.info()
for _ in range(5):
    idx.query(seq, k, stream).free()
torch.cuda.synchronize()
N = 200


def period(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e6


L = _lib.lib()
sp = C.c_void_p(stream.cuda_stream)
sptr = C.c_void_p(seq.data_ptr())
n = seq.numel()
q = C.c_void_p()
h = C.c_int64()


def raw():
    L.kmhg_query_run_device(idx._h, sptr, n, k, sp, C.byref(q), C.byref(h))
    L.kmhg_query_free(q)


def wrapped():
    idx.query(seq, k, stream).free()


D.timing_enable(True)
D.timing_reset()
for _ in range(20):
    idx.query(seq, k, stream).free()
qt = D.timing_report()
D.timing_enable(False)
dev_us = sum(v[1] / v[0] for v in qt.values() if v[0]) * 1e3
res = {
    "wrapped_us": round(period(wrapped), 1),
    "raw_ctypes_us": round(period(raw), 1),
    "kernels_us": round(dev_us, 1),
    "idle_stream_sync_us": round(period(lambda: stream.synchronize()), 1),
}
print(res)

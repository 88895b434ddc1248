"""Host-side cost of one build step on the GPU box: the asynchronous enqueue (ctypes + engine +
launches), the wait, and the free -- to see whether the host or the device paces the steps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import torch  # noqa: E402
from kmer_hasher_amd import _lib, synth  # noqa: E402
from kmer_hasher_amd import device as D  # noqa: E402

seq = torch.from_numpy(synth.iid(10_000_000, 1)).cuda()
L = _lib.lib()
stream = torch.cuda.current_stream()
sp = C.c_void_p(stream.cuda_stream)
for _ in range(5):
    D.DeviceIndex.build(seq, 31).free()
torch.cuda.synchronize()
N = 50
acc = {"enqueue": 0.0, "wait": 0.0, "free": 0.0}
for _ in range(N):
    t0 = time.perf_counter()
    idx = D.DeviceIndex.build(seq, 31, stream)
    t1 = time.perf_counter()
    idx.wait()
    t2 = time.perf_counter()
    idx.free()
    t3 = time.perf_counter()
    acc["enqueue"] += t1 - t0
    acc["wait"] += t2 - t1
    acc["free"] += t3 - t2
out = C.c_void_p()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    L.kmhg_build_device(C.c_void_p(seq.data_ptr()), seq.numel(), 31, 0, sp, C.byref(out))
    L.kmhg_free(out)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
acc["raw_enqueue_loop"] = t1 - t0
acc["raw_total_loop"] = t2 - t0
print({k: round(v / N * 1e6, 1) for k, v in acc.items()}, "us per step")

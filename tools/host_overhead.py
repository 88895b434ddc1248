"""Host-side cost of one build step (ctypes + engine enqueue + sync + free), on the GPU box."""
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
acc = {"py_build": 0.0, "raw_build": 0.0, "info": 0.0, "free": 0.0, "loop": 0.0}
t_loop = time.perf_counter()
for _ in range(N):
    t0 = time.perf_counter()
    idx = D.DeviceIndex.build(seq, 31, stream)
    t1 = time.perf_counter()
    idx.info()
    t2 = time.perf_counter()
    idx.free()
    t3 = time.perf_counter()
    acc["py_build"] += t1 - t0
    acc["info"] += t2 - t1
    acc["free"] += t3 - t2
acc["loop"] = time.perf_counter() - t_loop
out = C.c_void_p()
t0 = time.perf_counter()
for _ in range(N):
    L.kmhg_build_device(C.c_void_p(seq.data_ptr()), seq.numel(), 31, 0, sp, C.byref(out))
    L.kmhg_free(out)
acc["raw_build"] = time.perf_counter() - t0
print({k: round(v / N * 1e6, 1) for k, v in acc.items()}, "us per step")

"""Phase breakdown of k_v2_bucket from the diagnostic stamp build (libkmhgpu_stamps.so).

    python tools/stamps.py [L] [k]     (on the GPU box)
Loads kmer_hasher_amd/libkmhgpu_stamps.so instead of the product library, builds one index and
prints the mean/median cycles of each phase per bucket wave (s_memtime ticks)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kmer_hasher_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "kmer_hasher_amd", "libkmhgpu_stamps.so")
import torch  # noqa: E402
from kmer_hasher_amd import device as D, synth  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 31
seq = torch.from_numpy(synth.iid(L, 1)).cuda()
for _ in range(2):
    D.DeviceIndex.build(seq, k).free()
f = "/tmp/kmhg_stamps.bin"
os.environ["KMHG_STAMP_FILE"] = f
D.DeviceIndex.build(seq, k).free()
a = np.fromfile(f, np.uint64).reshape(-1, 8).astype(np.int64)
a = a[a[:, 0] > 0]
mode = os.environ.get("KMHG_BUCKET", "group")
wg = mode == "group"
names = {"group": ["clear", "passA(+load)", "scan", "passB", "table"],
         "sort": ["load", "sort pass 0", "sort pass 1", "runs", "place", "empties+stats"],
         "wave": ["init+start", "loads", "passA", "scan", "passB", "table"]}[mode]
last = len(names)
t0 = a[:, 0].min()
print(f"buckets {len(a)}  kernel span {a[:, last].max() - t0} ticks")
for i, n in enumerate(names):
    d = a[:, i + 1] - a[:, i]
    print(f"{n:12s} mean {d.mean():9.0f}  median {np.median(d):9.0f}  p99 {np.percentile(d, 99):9.0f}")
life = a[:, last] - a[:, 0]
print(f"{'lifetime':12s} mean {life.mean():9.0f}  median {np.median(life):9.0f}")
if wg:   # stamp 6: after wave 0's loads landed (drained right after stamp 1)
    d = a[:, 6] - a[:, 1]
    print(f"{'load wait':12s} mean {d.mean():9.0f}  median {np.median(d):9.0f}  (inside passA)")
st = np.sort(a[:, 0] - t0)
print("start ticks quantiles", [int(x) for x in np.percentile(st, [0, 10, 50, 90, 100])])

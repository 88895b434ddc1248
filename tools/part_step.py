"""Rehearsal of the owner-computes build's per-rank step on ONE GPU (tools, not product):
part 0 of n of an (n x L)-base sequence, timed like bench.py's sharded_build steps, for
n = 1, 2, 4, 8, with per-kernel times.  The per-rank step of an n-GPU run is this part build
(every rank walks all n x L windows), so L * n / step estimates the n-GPU value.

    python tools/part_step.py [L_mbp] [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth
    L = int(float(sys.argv[1]) * 1e6) if len(sys.argv) > 1 else 10_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    k = 31
    dev = torch.device("cuda", 0)
    out = {}
    for n in (1, 2, 4, 8):
        seq = torch.from_numpy(synth.iid(L * n, 1000 + n)).to(dev)
        for _ in range(2):
            D.DeviceIndex.build_part(seq, k, 0, n).wait().free()
        D.timing_enable(True)
        D.timing_reset()
        D.DeviceIndex.build_part(seq, k, 0, n).wait().free()
        per = {kk: round(v[1], 4) for kk, v in D.timing_report().items() if v[0]}
        D.timing_enable(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            D.DeviceIndex.build_part(seq, k, 0, n).free()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        out[n] = {"ms_per_step": round(ms, 4), "est_value_mbps": round(L * n / 1e6 / ms * 1e3, 1),
                  "kernels_ms": per}
        print(n, json.dumps(out[n]), flush=True)
        del seq
    base = out[1]["est_value_mbps"]
    print(json.dumps({"L": L, "eff": {n: round(o["est_value_mbps"] / (base * n), 3)
                                      for n, o in out.items()}}), flush=True)


if __name__ == "__main__":
    main()

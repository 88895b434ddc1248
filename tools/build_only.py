"""Build-only timing (A/B of build variants whose tables are not meant to be queried).

    python tools/build_only.py <Mbp> <k> [steps]

Builds a synthetic iid sequence (splitmix64 seed 2 for 100 Mbp, 1 otherwise) `steps` times like
bench.py's headline (asynchronous builds, freed, bracketed by synchronize) and prints one JSON
line: ms per build, Gbp/s, and the per-kernel HIP-event times of one build.  No query, readout or
other use of the tables is made, so a timing-only variant (e.g. -DKMHG_EXP_SLOT8) is safe here.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth
    mbp, k = int(sys.argv[1]), int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    L = mbp * 1_000_000
    seed = {10: 1, 100: 2, 500: 4}.get(mbp, 1)
    torch.cuda.set_device(0)
    seq = torch.from_numpy(synth.iid(L, seed)).cuda()
    stream = torch.cuda.current_stream()
    for _ in range(3):
        D.DeviceIndex.build(seq, k, stream).wait().free()
    D.timing_enable(True)
    D.timing_select(None)
    D.timing_reset()
    D.DeviceIndex.build(seq, k, stream).wait().free()
    per = {n: round(v[1], 5) for n, v in D.timing_report().items() if v[0]}
    D.timing_enable(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        D.DeviceIndex.build(seq, k, stream).free()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({"mbp": mbp, "k": k, "steps": steps, "ms_per_build": round(ms, 4),
                      "gbps": round(L / 1e9 / (ms * 1e-3), 3), "kernels_ms": per,
                      "lib": os.environ.get("KMHG_LIB_VARIANT", "product")}), flush=True)


if __name__ == "__main__":
    main()

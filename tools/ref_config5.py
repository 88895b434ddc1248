"""Config 5 through the reference itself, on the GPU box's host (test infrastructure).

    python tools/ref_config5.py OUT.json

BASELINE.json configs[4]: A = 500 Mbp iid (synth.iid seed 4), B = synth.derived(A, 5),
seq.kmer.pos(B vs make.kmer.hash(A, 31)).  The reference's index needs ~65 GB of host memory
(SURVEY.md §6), more than the build container holds, so tests/golden/fullsize.json pins config 5
to the clean-room oracle.  The GPU box's host has the room: this runs the compiled reference core
(oracle/_ref/libkmh_ref.so = src/kmer_pos.c + src/kmer_util.c + klib, gcc -O2) on one pinned core,
digests its query rows exactly as make_fullsize_golden.py digests the oracle's (sha256 of the
int32 (i, j) rows in order), and times build, query and teardown -- the whole-size CPU baseline
of config 5 (bench.py's own cpu_baseline leg stays a bounded sample).  No GPU is used.
"""
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kmer_hasher_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    out_path = sys.argv[1]
    L, k = 500_000_000, 31
    stop = threading.Event()

    def beat():                           # a line a minute: a long C call is not a hang
        while not stop.wait(45):
            log("... running")
    threading.Thread(target=beat, daemon=True).start()
    assert O.ref_available(), "oracle/_ref/libkmh_ref.so missing (built by oracle/Makefile)"
    A = synth.iid(L, 4)
    B = synth.derived(A, 5)
    a, b = A.tobytes(), B.tobytes()
    del A, B
    prev = os.sched_getaffinity(0)
    os.sched_setaffinity(0, {min(prev)})  # one core, as taskset -c would
    log("reference build of A")
    t0 = time.perf_counter()
    ref = O.RefIndex(a, k)
    t_build = time.perf_counter() - t0
    N, P, mx = ref.totals()
    log("built", ref.kmer_count, N, f"{t_build:.1f}s")
    t0 = time.perf_counter()
    rows = ref.query(b, k)
    t_query = time.perf_counter() - t0
    H = rows.size // 2
    log("queried", H, f"{t_query:.1f}s")
    d = hashlib.sha256(memoryview(rows)).hexdigest()
    del rows
    t0 = time.perf_counter()
    ref.close()
    t_free = time.perf_counter() - t0
    os.sched_setaffinity(0, prev)
    stop.set()
    rec = {"name": "config5", "L": L, "k": k, "U": int(ref.kmer_count), "N": int(N), "P": int(P),
           "max_n": int(mx),
           "source": "reference itself: oracle/_ref/libkmh_ref.so (src/kmer_pos.c + "
                     "src/kmer_util.c + klib, gcc -O2) run on the GPU box's host "
                     "(tools/ref_config5.py)",
           "query": {str(k): {"H": int(H), "sha": d}},
           "cpu": {"cores": 1, "build_s": round(t_build, 2), "query_s": round(t_query, 2),
                   "teardown_s": round(t_free, 2),
                   "build_mbps": round(L / 1e6 / t_build, 3),
                   "query_mbps": round(L / 1e6 / t_query, 3)}}
    try:
        import platform
        rec["cpu"]["host"] = {"nproc": os.cpu_count(), "machine": platform.machine()}
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                rec["cpu"]["host"]["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)
    log("wrote", out_path)


if __name__ == "__main__":
    main()

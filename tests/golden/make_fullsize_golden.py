"""Full-size golden digests for BASELINE.json configs[1..4].

    python tests/golden/make_fullsize_golden.py [2] [3] [4] [5]

Configs 2, 3 and 4 come from the REFERENCE ITSELF: oracle/_ref/libkmh_ref.so is the
reference's src/kmer_pos.c + src/kmer_util.c + klib compiled by oracle/Makefile (needs
/root/reference, so this runs in the build container).  Its outputs are digested in the
reference's own khash row order (kmer_positions' bucket walk, src/kmer_hash.c:1096-1124,
streamed by ref_harness.c's ref_rows_chunk so config 4's 8 GB pair table is never held):

  config 2  10 Mbp iid (seed 1), k=31: build + kmer.pos $pos/$count/$kmer + self seq.kmer.pos
  config 3  100 Mbp iid (seed 2), k=21: build + kmer.pos $pos/$count + self seq.kmer.pos
            (31.5 s build, 16.7 s query, 10.35 GB RSS on one core)
  config 4  40 Mbp synth.config4 (seed 3), k=31: kmer.pos $pos/$pair.pos/$count
            (P = 685,613,382 rows, inside §8(d)'s [0.5e9, 1.5e9])

Config 5 (A = 500 Mbp iid seed 4, B = synth.derived(A, 5), seq.kmer.pos(B vs index(A)), k=31)
needs ~65 GB of host memory in the reference, more than this container has, so
its digest comes from the clean-room restatement oracle/kmer_oracle.c (itself checked against
the compiled reference and every golden record by tests/test_oracle_golden.py), driven here
without Python-side copies (~40 GB peak).

Writes tests/golden/fullsize.json (merging with the configs already there).
"""
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
from kmh_canon import sha  # noqa: E402
from kmer_hasher_amd import synth  # noqa: E402

OUT = os.path.join(HERE, "fullsize.json")
REF_SRC = ("oracle/_ref/libkmh_ref.so = reference src/kmer_pos.c + src/kmer_util.c (+klib) "
           "compiled by oracle/Makefile; digests in its khash row order")


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def ref_record(name, seq: np.ndarray, k, qks, opts, with_kmer=False):
    b = seq.tobytes()
    t0 = time.time()
    ref = O.RefIndex(b, k)
    t_build = time.time() - t0
    N, P, mx = ref.totals()
    cnt = ref.positions(8 | (1 if with_kmer else 0))
    rec = {"name": name, "L": int(seq.size), "k": k, "U": int(len(cnt["count"])), "N": N,
           "P": P, "max_n": mx, "kmer_count": ref.kmer_count, "source": REF_SRC,
           "raw_sha": {"count": sha(cnt["count"])}, "query": {},
           "ref_build_s": round(t_build, 2)}
    if with_kmer:
        rec["raw_sha"]["kmer"] = sha(cnt["kmer"])
    del cnt
    for opt, field in ((2, "pos"), (4, "pair.pos")):
        if opt in opts:
            t0 = time.time()
            d, n = ref.rows_sha256(opt)
            assert n == (N if opt == 2 else P)
            rec["raw_sha"][field] = d
            log(name, field, n, f"{time.time() - t0:.1f}s")
    for kq in qks:
        t0 = time.time()
        q = ref.query(b, kq)
        rec["query"][str(kq)] = {"H": int(q.size // 2), "sha": sha(q),
                                 "ref_query_s": round(time.time() - t0, 2)}
        del q
    t0 = time.time()
    ref.close()
    rec["ref_teardown_s"] = round(time.time() - t0, 2)
    log(name, {x: rec[x] for x in ("U", "N", "P", "max_n")}, rec["query"])
    return rec


def oracle_config5(L=500_000_000, k=31):
    """seq.kmer.pos(B vs index(A)) through kmer_oracle.c's canonical CSR (no copies)."""
    A = synth.iid(L, 4)
    B = synth.derived(A, 5)
    a, bq = A.tobytes(), B.tobytes()
    del A, B
    lib = O._orc()
    cap = L + 1
    keys = np.empty(cap, np.uint64)
    counts = np.empty(cap, np.int32)
    offs = np.empty(cap + 1, np.int64)
    pos = np.empty(cap, np.int32)
    n, p, mx = C.c_long(0), C.c_int64(0), C.c_int32(0)
    t0 = time.time()
    U = lib.orc_index_build(a, L, k, keys, counts, offs, pos, C.byref(n), C.byref(p), C.byref(mx))
    assert U > 0
    log("config5 index", U, n.value, p.value, mx.value, f"{time.time() - t0:.1f}s")
    del a
    t0 = time.time()
    H = lib.orc_query(keys, counts, offs, pos, U, bq, len(bq), k, None)
    rows = np.empty(2 * H + 1, np.int32)
    H2 = lib.orc_query(keys, counts, offs, pos, U, bq, len(bq), k, rows.ctypes.data)
    assert H2 == H
    d = hashlib.sha256(memoryview(rows[:2 * H])).hexdigest()
    log("config5 query", H, f"{time.time() - t0:.1f}s")
    return {"name": "config5", "L": L, "k": k, "U": int(U), "N": int(n.value), "P": int(p.value),
            "max_n": int(mx.value),
            "source": "clean-room oracle/kmer_oracle.c (orc_index_build + orc_query); the "
                      "reference needs ~65 GB here (SURVEY.md §6)",
            "query": {str(k): {"H": int(H), "sha": d}}}


def main():
    want = [int(x) for x in sys.argv[1:]] or [2, 3, 4, 5]
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    if any(c in want for c in (2, 3, 4)):
        assert O.ref_available(), "build oracle/_ref first: make -C oracle"
    if 2 in want:
        out["config2"] = ref_record("config2", synth.iid(10_000_000, 1), 31, [31], (2,),
                                    with_kmer=True)
    if 3 in want:
        out["config3"] = ref_record("config3", synth.iid(100_000_000, 2), 21, [21], (2,))
    if 4 in want:
        out["config4"] = ref_record("config4", synth.config4(40_000_000, 3), 31, [], (2, 4))
    if 5 in want:
        out["config5"] = oracle_config5()
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    log("wrote", OUT)


if __name__ == "__main__":
    main()

"""Generate the golden vectors in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (needs /root/reference and oracle/_ref/libkmh_ref.so, which
``make -C oracle`` compiles from the reference's own src/kmer_pos.c + src/kmer_util.c):

    python tests/golden/make_golden.py

Writes
  golden.json          per (input, k): U, N, P, max n, self-query H and sha256 digests of the
                       reference outputs, both raw (khash bucket order) and canonical
                       (k-mers ranked by first position; tests/kmh_canon.py)
  edge_cases.json      full reference outputs for the short edge-case strings
  testfa_k15.npz,
  testfa_k31.npz       canonical counts / pos rows / k-mer strings for test.fa
test.fa is the reference's own fixture (59,940 bp, one record), copied verbatim as data.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
from kmh_canon import canon_from_raw, sha  # noqa: E402
from kmer_hasher_amd import synth  # noqa: E402


def read_fasta(path):
    return "".join(l.strip() for l in open(path) if not l.startswith(">"))


EDGE = [
    ("ACGTA", 3, [3]), ("ACGTNACG", 3, [3]), ("ACGTNACGT", 3, [3, 2]), ("acgtNNacgt", 2, [2]),
    ("AAAAAA", 2, [2, 1]), ("AAAAAA", 5, [5]), ("ACGTACGT", 1, [1, 2]), ("ACGTACGTAC", 4, [4, 3, 5]),
    ("NACGTN", 3, [3]), ("NNNNACGTACGTNNNN", 4, [4]), ("ACGNTACGTNNAC", 3, [3, 2]),
    ("RYKMSWBDHV-.RYKMSWBDHV-.", 5, [5, 3]), ("acgtRYKMnACGTacgtSWBD", 4, [4]),
    ("G" * 40, 32, [31, 20]), ("G" * 33, 32, [31]), ("GGGGGGGGGGGGGGGGGGGGGGGGGGGGGGGGA", 32, [31]),
    ("ACGT" * 12, 32, [31, 16]), ("TTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTTT", 31, [31, 7]),
    ("ACGTNACGTNACGTNACGT", 4, [4, 3]), ("AC", 1, [1]), ("ACN", 1, [1]), ("NAC", 1, [1]),
    ("ACGTACGTTGCAN" * 5, 6, [6, 9, 2]),
]


def record(name, seq, k, qks, want_arrays=False):
    ref = O.RefIndex(seq, k)
    raw = ref.positions(15)
    can, order = canon_from_raw(raw)
    cnt = raw["count"]
    rec = {
        "name": name, "k": k, "U": int(len(cnt)), "N": int(cnt.sum()),
        "P": int((cnt.astype(np.int64) * (cnt - 1) // 2).sum()),
        "max_n": int(cnt.max()) if len(cnt) else 0,
        "kmer_count": ref.kmer_count,
        "raw_sha": {"kmer": sha(raw["kmer"]), "pos": sha(raw["pos"]),
                    "pair.pos": sha(raw["pair.pos"]), "count": sha(raw["count"])},
        "canon_sha": {"kmer": sha(can["kmer"]), "pos": sha(can["pos"]),
                      "pair.pos": sha(can["pair.pos"]), "count": sha(can["count"])},
        "khash_order_sha": sha(order.astype(np.int64)),
        "query": {},
    }
    for kq in qks:
        q = ref.query(seq, kq)
        rec["query"][str(kq)] = {"H": int(q.size // 2), "sha": sha(q)}
    if want_arrays:
        rec["arrays"] = {
            "raw": {"kmer": raw["kmer"], "pos": raw["pos"].tolist(),
                    "pair.pos": raw["pair.pos"].tolist(), "count": raw["count"].tolist()},
            "canon": {"kmer": can["kmer"], "pos": can["pos"].tolist(),
                      "pair.pos": can["pair.pos"].tolist(), "count": can["count"].tolist()},
            "query": {str(kq): ref.query(seq, kq).tolist() for kq in qks},
        }
    ref.close()
    return rec, can


def main():
    assert O.ref_available(), "build oracle/_ref first: make -C oracle"
    out = {"source": "oracle/_ref/libkmh_ref.so = reference src/kmer_pos.c + src/kmer_util.c "
                     "(+klib) compiled by oracle/Makefile", "records": []}
    seq = read_fasta(os.path.join(HERE, "test.fa"))
    for k in (10, 15, 16, 17, 21, 31, 32):
        qks = [k] if k <= 31 else [31]
        if k == 16:
            qks = [16, 21]           # test.R:41,49-55 queries a k=16 index with k=21
        rec, can = record("test.fa", seq, k, qks)
        out["records"].append(rec)
        if k in (15, 31):
            np.savez_compressed(os.path.join(HERE, f"testfa_k{k}.npz"),
                                count=can["count"], pos=can["pos"],
                                kmer=np.array(can["kmer"], dtype=f"S{k}"))
        print("test.fa", k, rec["U"], rec["N"], rec["P"], rec["max_n"], rec["query"])
    # seeded synthetic inputs with N-runs, lower case and ambiguity codes
    synth_specs = [
        ("iid200k_s1", lambda: synth.iid(200_000, 1), [21, 31], [21, 31, 15]),
        ("iid200k_nruns_lc_s2",
         lambda: synth.add_lowercase(synth.add_n_runs(synth.iid(200_000, 2), 0.01, 7), 0.1, 11),
         [15, 31, 32], [15, 31, 12]),
        ("amb100k_s3", lambda: synth.add_ambiguity(synth.iid(100_000, 3), 0.02, 13), [11, 25],
         [11, 25]),
        ("rep300k_s3", lambda: synth.repeat_rich(300_000, 3, n_gap_every=50_000), [31, 17],
         [31, 17]),
    ]
    for name, gen, ks, qks in synth_specs:
        s = gen().tobytes().decode("latin-1")
        for k in ks:
            rec, _ = record(name, s, k, qks)
            out["records"].append(rec)
            print(name, k, rec["U"], rec["N"], rec["P"], rec["max_n"], rec["query"])
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    edge = []
    for s, k, qks in EDGE:
        rec, _ = record(s, s, k, qks, want_arrays=True)
        edge.append(rec)
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(edge, f, indent=1)
    print("edge cases:", len(edge))


if __name__ == "__main__":
    main()

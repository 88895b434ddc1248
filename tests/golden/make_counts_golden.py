"""Generate tests/golden/counts_golden.json (count.kmers) from the REFERENCE ITSELF.

Run in the build container (needs oracle/_ref/libkmh_ref.so, which ``make -C oracle`` compiles
from the reference's own src/kmer_pos.c + src/kmer_util.c + klib; count_kmers / seq_to_counts /
kmer_count_insert live in src/kmer_hash.c, which needs R, and are restated over that compiled
core in oracle/ref_harness.c):

    python tests/golden/make_counts_golden.py

Each case is a sequence of count.kmers calls (k, source, source_n, character vector) into one
pointer, then kmer.pos(opt.flag = 15) in the reference's khash order and seq.kmer.pos of a query.
Recorded: U, kmer_count and sha256 digests of every output (raw = the reference's bytes); small
cases also keep the full arrays.  Inputs are regenerated from the seeds by tests/synth_inputs.py.
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
from kmh_canon import sha  # noqa: E402
from synth_inputs import counts_cases  # noqa: E402


def run_case(name, k, source_n, calls, query, qk, want_arrays):
    ref = None
    for source, seqs in calls:
        ref = O.RefIndex.counts(seqs, k, source, source_n, into=ref)
    raw = ref.positions(15)
    q = ref.query(query, qk) if len(query) > qk else np.empty(0, np.int32)
    rec = {"name": name, "k": k, "source_n": source_n, "U": len(raw["count"]),
           "kmer_count": ref.kmer_count,
           "raw_sha": {"kmer": sha(raw["kmer"]), "pos": sha(raw["pos"]),
                       "pair.pos": sha(raw["pair.pos"]), "count": sha(raw["count"])},
           "query": {"k": qk, "H": int(q.size // 2), "sha": sha(q)}}
    if want_arrays:
        rec["arrays"] = {"kmer": raw["kmer"], "pos": raw["pos"].tolist(),
                         "pair.pos": raw["pair.pos"].tolist(), "count": raw["count"].tolist(),
                         "query": q.tolist()}
    ref.close()
    return rec


def main():
    assert O.ref_available(), "build oracle/_ref first: make -C oracle"
    out = {"source": "oracle/_ref/libkmh_ref.so: reference src/kmer_pos.c + src/kmer_util.c "
                     "(+klib) compiled by oracle/Makefile; count_kmers restated in ref_harness.c",
           "cases": []}
    for c in counts_cases(os.path.join(HERE, "test.fa")):
        rec = run_case(**c)
        out["cases"].append(rec)
        print(rec["name"], rec["k"], rec["source_n"], rec["U"], rec["kmer_count"],
              rec["query"]["H"])
    with open(os.path.join(HERE, "counts_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

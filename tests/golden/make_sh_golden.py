"""Generate tests/golden/sh_golden.json (count.kmers.fq.sh.rp / seq.kmer.depth.sh /
kmer.spec.sh.n) from the REFERENCE ITSELF.

Run in the build container (needs oracle/_ref/libkmh_ref_sh.so, which ``make -C oracle``
compiles from the reference's own src/suffix_hash.c + src/kmer_reader.c + src/kmer_util.c +
src/thread_queue.c with klib's kseq/khash, zlib and pthreads; the .Call wrappers of
src/kmer_hash.c need R and are restated in oracle/ref_sh_harness.c):

    python tests/golden/make_sh_golden.py

It also checks, once, that the phred -> log-likelihood table the oracle and the GPU engine
regenerate from its formula equals the 256 doubles of the reference's src/Q_to_log_likelihood.h
(read here as text; only the digest of the values is recorded).  Each case is a sequence of
count.kmers.fq.sh.rp calls into one pointer; recorded: U and sha256 digests of the
(key-sorted) keys and counts, the depth of each query string, and spectra.  Inputs: the
reference's own FASTQ files (copied to tests/golden/ as data fixtures) and the seeded inputs of
tests/sh_inputs.py.
"""
import json
import os
import re
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O  # noqa: E402
from kmh_canon import sha  # noqa: E402
import sh_inputs as I  # noqa: E402

REF_HEADER = "/root/reference/src/Q_to_log_likelihood.h"


def check_qll():
    txt = open(REF_HEADER).read()
    body = txt[txt.index("{") + 1:txt.index("}")]
    vals = np.array([float(x) for x in re.findall(r"-?[0-9.]+(?:e-?[0-9]+)?", body)], np.float64)
    mine = O.qll_table()
    assert len(vals) == 256 and np.array_equal(vals, mine), "q_to_ll regeneration differs"
    return sha(mine)


CASES = [
    # name, k, source_n, calls [(file, prefix_bits, min_q, max_reads, source)], depth strings
    ("repeat40_k21", 21, 1, [("repeat_40.fq", 10, 0, -1, 0)], "sim"),
    ("test10_k15_q20", 15, 2, [("test_10.fastq", 10, 20, -1, 0), ("test_10.fastq", 8, 0, 5, 1)],
     "sim"),
    ("testgz_k21", 21, 1, [("test.fastq.gz", 12, 0, -1, 0)], None),
    ("testgz_k31_q25_s3", 31, 3, [("test.fastq.gz", 20, 25, 2000, 2),
                                  ("test.fastq.gz", 20, 10, 500, 0)], None),
    ("tricky_k5", 5, 4, [("tricky.fq", 6, 10, -1, 3), ("tricky.fq", 6, 0, -1, 1)], None),
    ("tricky_k9_q30", 9, 1, [("tricky.fq", 10, 30, -1, 0)], None),
    ("random_k7_q12", 7, 2, [("random.fq", 8, 12, -1, 1)], None),
    ("sim_k15", 15, 2, [("sim.fq", 10, 15, -1, 0), ("sim.fq", 10, 30, 1500, 1)], "sim"),
    ("sim_k21", 21, 1, [("sim.fq", 10, 20, -1, 0)], "sim"),
    ("sim_k31", 31, 2, [("sim.fq", 24, 0, -1, 1), ("sim.fq", 24, 35, -1, 0)], "sim"),
]
SPECTRA = [(50, [1, 2, 3], [0, 0, 1]), (10, [1], [1]), (300, [1, 2], [1, 0])]


def main():
    out = {"source": "oracle/_ref/libkmh_ref_sh.so: reference src/suffix_hash.c + kmer_reader.c + "
                     "kmer_util.c + thread_queue.c (+klib kseq/khash, zlib) compiled by "
                     "oracle/Makefile; .Call wrappers restated in ref_sh_harness.c",
           "qll_sha": check_qll(), "cases": []}
    with tempfile.TemporaryDirectory() as tmp:
        files, genome = I.materialise(tmp)
        for name, k, S, calls, dstr in CASES:
            ref = O.RefSH()
            for f, pb, mq, mr, src in calls:
                ref.add_fastq(files[f], k, pb, mq, mr if mr >= 0 else 2**62, S, src)
            keys, M = ref.arrays()
            rec = {"name": name, "k": k, "source_n": S,
                   "calls": [list(c) for c in calls], "U": int(len(keys)),
                   "keys_sha": sha(keys), "counts_sha": sha(M.astype(np.int32)),
                   "depth": [], "spectra": []}
            if len(keys) <= 400:
                rec["keys"] = [int(x) for x in keys]
                rec["counts"] = M.astype(int).tolist()
            if dstr:
                for j, s in enumerate(I.depth_strings(genome, k)):
                    if len(s) < k:
                        continue
                    d = ref.depth(s, k)
                    rec["depth"].append({"string": j, "L": len(s), "sha": sha(d.astype(np.int32))})
            for mc, comb, inner in SPECTRA:
                comb = [c for c in comb if c < (1 << S)] or [1]
                inner = inner[:len(comb)]
                smin = [1 + (j % 3) for j in range(S)]
                sp = ref.spectrum(mc, comb, inner, smin)
                rec["spectra"].append({"max_count": mc, "comb": comb, "comb_inner": inner,
                                       "source_min": smin, "sha": sha(sp)})
            ref.close()
            out["cases"].append(rec)
            print(name, rec["U"], len(rec["depth"]), file=sys.stderr)
    with open(os.path.join(HERE, "sh_golden.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()

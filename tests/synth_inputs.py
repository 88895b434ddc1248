"""Regenerates the synthetic inputs named in tests/golden/golden.json (same seeds as
tests/golden/make_golden.py)."""
from kmer_hasher_amd import synth

SYNTH = {
    "iid200k_s1": lambda: synth.iid(200_000, 1),
    "iid200k_nruns_lc_s2":
        lambda: synth.add_lowercase(synth.add_n_runs(synth.iid(200_000, 2), 0.01, 7), 0.1, 11),
    "amb100k_s3": lambda: synth.add_ambiguity(synth.iid(100_000, 3), 0.02, 13),
    "rep300k_s3": lambda: synth.repeat_rich(300_000, 3, n_gap_every=50_000),
}


def sequence(name, testfa):
    if name == "test.fa":
        return testfa
    return SYNTH[name]().tobytes().decode("latin-1")


def _s(a) -> str:
    return a.tobytes().decode("latin-1")


def counts_cases(testfa_path: str) -> list[dict]:
    """count.kmers scenarios of tests/golden/counts_golden.json: each is a list of
    (source, character vector) calls into one pointer of (k, source_n), then kmer.pos(15) and
    seq.kmer.pos(query, qk).  test.R:340-343 is the model (two calls, sources 0 and 1 of 2)."""
    fa = "".join(l.strip() for l in open(testfa_path) if not l.startswith(">"))
    iid = _s(synth.iid(100_000, 21))
    noisy = _s(synth.add_lowercase(synth.add_n_runs(synth.iid(60_000, 22), 0.01, 5), 0.1, 6))
    rep = _s(synth.repeat_rich(60_000, 23, n_gap_every=20_000))
    rep2 = _s(synth.repeat_rich(100_000, 24, n_gap_every=30_000))
    return [
        dict(name="testfa_k21_s2", k=21, source_n=2,
             calls=[(0, [fa[:7000], fa[7000:19000], fa[19000:41000], fa[41000:]]),
                    (1, [fa[30000:], fa[:12000]])],
             query=fa[:5000], qk=21, want_arrays=False),
        dict(name="testfa_k15_s1", k=15, source_n=1, calls=[(0, [fa])],
             query=fa[:3000], qk=15, want_arrays=False),
        dict(name="edge_multi_k3_s3", k=3, source_n=3,
             calls=[(0, ["ACGTACGTTTNACGTACGA", "GGGACGTACG", "ACG", "ACGTNACG", "", "NNNN"]),
                    (2, ["ACGTTTTACGTAAN", "acgtNNacgt"]), (1, ["TTTACG", "NACGT"])],
             query="ACGTACGTNACGT", qk=3, want_arrays=True),
        dict(name="edge_tail_k4_s2", k=4, source_n=2,
             calls=[(0, ["ACGTNACGT", "ACGTACGTNGGCC", "GGCCNTTAA", "ACGT", "ACGTA"]),
                    (1, ["NNACGTNN", "CCCCNAAAAN", "TTTTT"])],
             query="ACGTACGTGGCC", qk=4, want_arrays=True),
        dict(name="edge_k32_allG_s2", k=32, source_n=2,
             calls=[(0, ["G" * 40, "G" * 33, "ACGT" * 12]), (1, ["G" * 35])],
             query="G" * 40, qk=31, want_arrays=True),
        dict(name="edge_negsource_k5_s2", k=5, source_n=2,
             calls=[(0, ["ACGTACGTACGGT", "TTTTTTT"]), (-1, ["CCCCCCCCC", "ACGTACGTAC"])],
             query="ACGTACGTACGGT", qk=5, want_arrays=True),
        dict(name="synth_k31_s3", k=31, source_n=3,
             calls=[(0, [iid[:40_000], iid[40_000:70_000], iid[70_000:]]), (1, [noisy]),
                    (2, [rep, iid[10_000:50_000]])],
             query=iid[:20_000], qk=31, want_arrays=False),
        dict(name="rep_k17_s4", k=17, source_n=4,
             calls=[(3, [rep2]), (0, [rep2[50_000:]]), (3, [rep2[:30_000]])],
             query=rep2[:10_000], qk=17, want_arrays=False),
    ]

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

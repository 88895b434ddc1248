"""kmer.pairs (kmer_pair_pos, reference src/kmer_hash.c:1174-1203) on the GPU against the oracle.

The reference implementation crashes (test.R:330), so no reference output exists to pin this
row: parity is against the oracle's restatement of the intended loop (OracleIndex.pairs_with),
the checker being pinned on the rest of the index by test_oracle_golden.py."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _mutate(s: bytes, rate: float, seed: int) -> bytes:
    rng = np.random.default_rng(seed)
    a = np.frombuffer(s, np.uint8).copy()
    hit = rng.random(len(a)) < rate
    a[hit] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, hit.sum())]
    return a.tobytes()


def test_pairs_match_oracle(gpu):
    from kmer_hasher_amd import kmer_pairs, make_kmer_hash, set_row_order, synth
    a = synth.add_n_runs(synth.repeat_rich(80_000, 9, n_gap_every=30_000), 0.002, 4).tobytes()
    b = _mutate(a[20_000:] + a[:20_000], 0.01, 2)
    for k in (11, 21, 31, 32):
        pa, pb = make_kmer_hash(a.decode("latin-1"), k), make_kmer_hash(b.decode("latin-1"), k)
        oa, ob = O.OracleIndex(a, k), O.OracleIndex(b, k)
        got = kmer_pairs(pa, pb)
        want = oa.pairs_with(ob)
        assert got.shape[1] == 2 and len(want) > 0
        assert np.array_equal(got.reshape(-1), want), k
        # b against a, and a against itself
        assert np.array_equal(kmer_pairs(pb, pa).reshape(-1), ob.pairs_with(oa)), k
        assert np.array_equal(kmer_pairs(pa, pa).reshape(-1), oa.pairs_with(oa)), k
        # a's k-mers in the reference's khash order, as the reference's bucket walk visits them
        set_row_order(pa, "khash")
        assert np.array_equal(kmer_pairs(pa, pb).reshape(-1), oa.pairs_with(ob, oa.khash_order()))
        pa.free()
        pb.free()


def test_pairs_edge_cases(gpu):
    from kmer_hasher_amd import KmerHashError, kmer_pairs, make_kmer_hash
    p1 = make_kmer_hash("AAAAAAAAAA", 3)
    p2 = make_kmer_hash("CCCCCCCCCC", 3)
    assert kmer_pairs(p1, p2).shape == (0, 2)             # nothing shared
    p3 = make_kmer_hash("AAAAAAAAAAAAAAAA", 3)            # one k-mer, many positions
    got = kmer_pairs(p1, p3)
    want = O.OracleIndex("AAAAAAAAAA", 3).pairs_with(O.OracleIndex("AAAAAAAAAAAAAAAA", 3))
    assert np.array_equal(got.reshape(-1), want)
    p4 = make_kmer_hash("AAAAAAAAAA", 4)
    with pytest.raises(KmerHashError, match="the two indices must have the same k"):
        kmer_pairs(p1, p4)
    g = make_kmer_hash("G" * 40, 32)                      # the k = 32 side-slot key
    assert np.array_equal(kmer_pairs(g, g).reshape(-1),
                          O.OracleIndex("G" * 40, 32).pairs_with(O.OracleIndex("G" * 40, 32)))

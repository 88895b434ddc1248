"""The oracle (CPU restatement) against the reference's golden vectors -- pins the checker."""
import numpy as np
import pytest

from kmh_canon import sha
from oracle import oracle as O
from synth_inputs import sequence


def _records(golden):
    return golden[0]["records"]


def test_golden_present(golden):
    g, e = golden
    assert len(g["records"]) >= 10 and len(e) >= 20


@pytest.mark.parametrize("i", range(15))
def test_oracle_matches_reference_digests(golden, testfa, i):
    recs = _records(golden)
    if i >= len(recs):
        pytest.skip()
    r = recs[i]
    s = sequence(r["name"], testfa)
    oi = O.OracleIndex(s, r["k"])
    assert (oi.U, oi.N, oi.P, oi.max_n) == (r["U"], r["N"], r["P"], r["max_n"])
    assert sha(oi.counts) == r["canon_sha"]["count"]
    assert sha(oi.pos_rows()) == r["canon_sha"]["pos"]
    km = oi.kmer_strings()
    assert sha(km) == r["canon_sha"]["kmer"]
    # the khash bucket order replay reproduces the reference's raw row order exactly
    order = oi.khash_order()
    assert sha(oi.counts[order]) == r["raw_sha"]["count"]
    assert sha([km[j] for j in order]) == r["raw_sha"]["kmer"]
    if r["P"] <= 20_000_000:
        assert sha(oi.pair_rows()) == r["canon_sha"]["pair.pos"]
    for kq, qv in r["query"].items():
        q = oi.query(s, int(kq))
        assert q.size // 2 == qv["H"]
        assert sha(q) == qv["sha"]


def test_oracle_edge_cases(golden):
    _, edge = golden
    for r in edge:
        s, k = r["name"], r["k"]
        oi = O.OracleIndex(s, k)
        a = r["arrays"]["canon"]
        assert oi.counts.tolist() == a["count"], (s, k)
        assert oi.pos_rows().tolist() == a["pos"], (s, k)
        assert oi.pair_rows().tolist() == a["pair.pos"], (s, k)
        assert oi.kmer_strings() == a["kmer"], (s, k)
        order = oi.khash_order()
        assert oi.counts[order].tolist() == r["arrays"]["raw"]["count"], (s, k)
        for kq, rows in r["arrays"]["query"].items():
            assert oi.query(s, int(kq)).tolist() == rows, (s, k, kq)


def test_window_rule_examples():
    # SURVEY.md §8.0 verified examples
    keys, s1, e1 = O.windows("ACGTNACG", 3)
    assert len(keys) == 2                      # the final N-free run of length exactly k drops
    keys, s1, e1 = O.windows("ACGTA", 3)
    assert list(s1) == [1, 2, 3] and list(e1) == [3, 4, 5]


@pytest.mark.skipif(not O.ref_available(), reason="reference core not compiled here")
@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_compiled_reference_random(seed):
    rng = np.random.default_rng(seed)
    L = int(rng.integers(40, 4000))
    alphabet = np.frombuffer(b"ACGTACGTACGTacgtNnRY-", np.uint8)
    p = np.full(alphabet.size, 1.0)
    p[12:16] = 0.3
    p[16:18] = 0.2 if seed % 2 else 0.02
    p /= p.sum()
    s = alphabet[rng.choice(alphabet.size, L, p=p)].tobytes().decode()
    for k in (1, 2, 5, 13, 31, 32):
        if L <= k:
            continue
        ref = O.RefIndex(s, k)
        raw = ref.positions(15)
        oi = O.OracleIndex(s, k)
        order = oi.khash_order()
        assert raw["count"].tolist() == oi.counts[order].tolist()
        km = oi.kmer_strings()
        assert raw["kmer"] == [km[j] for j in order]
        assert raw["pair.pos"].tolist() == oi.pair_rows(order).tolist()
        for kq in (k, max(1, k - 3), min(31, k + 2)):
            if kq <= 31 and L > kq:
                assert ref.query(s, kq).tolist() == oi.query(s, kq).tolist()
        ref.close()

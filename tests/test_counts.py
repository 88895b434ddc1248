"""count.kmers (SURVEY.md §8 f next-4): per-source k-mer counts.

CPU: the oracle's restatement (OracleCounts) against the reference's golden vectors
(tests/golden/counts_golden.json, made by make_counts_golden.py from the compiled reference core)
and against the compiled reference on random multi-sequence inputs; argument validation.
GPU (-m gpu): the HIP path through the C-ABI against the same golden vectors -- byte-identical in
the reference's khash order -- and against the oracle in first-insertion order.
"""
import json
import os

import numpy as np
import pytest

from kmh_canon import sha
from oracle import oracle as O
from synth_inputs import counts_cases

HERE = os.path.dirname(os.path.abspath(__file__))
FA = os.path.join(HERE, "golden", "test.fa")


@pytest.fixture(scope="module")
def cgold():
    with open(os.path.join(HERE, "golden", "counts_golden.json")) as f:
        g = json.load(f)
    cases = {c["name"]: c for c in counts_cases(FA)}
    return [(cases[r["name"]], r) for r in g["cases"]]


def _oracle(case) -> O.OracleCounts:
    oc = O.OracleCounts(case["k"], case["source_n"])
    for source, seqs in case["calls"]:
        oc.add(seqs, source)
    return oc


def _raw_from_oracle(oc: O.OracleCounts):
    """kmer.pos(15) of the counts in the reference's khash order (what the reference returns)."""
    ix = oc.index()
    order = ix.khash_order()
    U, S = ix.U, oc.S
    km = ix.kmer_strings()
    M = ix.positions.reshape(U, S) if U else np.empty((0, S), np.int32)
    pos = np.stack([np.repeat(np.arange(1, U + 1, dtype=np.int32), S),
                    M[order].reshape(-1)], 1).reshape(-1)
    return {"kmer": [km[j] for j in order], "pos": pos.astype(np.int32),
            "pair.pos": ix.pair_rows(order), "count": ix.counts[order]}, ix


def test_counts_golden_present(cgold):
    assert len(cgold) >= 8


def test_oracle_counts_match_reference_digests(cgold):
    for case, r in cgold:
        oc = _oracle(case)
        raw, ix = _raw_from_oracle(oc)
        assert (oc.U, oc.kmer_count) == (r["U"], r["kmer_count"]), case["name"]
        for f in ("kmer", "pos", "pair.pos", "count"):
            assert sha(raw[f]) == r["raw_sha"][f], (case["name"], f)
        q = ix.query(case["query"], case["qk"]) if len(case["query"]) > case["qk"] else \
            np.empty(0, np.int32)
        assert q.size // 2 == r["query"]["H"] and sha(q) == r["query"]["sha"], case["name"]
        if "arrays" in r:
            assert raw["pos"].tolist() == r["arrays"]["pos"], case["name"]
            assert raw["kmer"] == r["arrays"]["kmer"], case["name"]


@pytest.mark.skipif(not O.ref_available(), reason="reference core not compiled here")
@pytest.mark.parametrize("seed", range(4))
def test_oracle_counts_vs_compiled_reference_random(seed):
    rng = np.random.default_rng(100 + seed)
    alphabet = np.frombuffer(b"ACGTACGTACGTacgtNnRY", np.uint8)
    p = np.full(alphabet.size, 1.0)
    p[16:18] = 0.1 if seed % 2 else 0.01
    p /= p.sum()

    def rnd(n):
        return alphabet[rng.choice(alphabet.size, n, p=p)].tobytes().decode()

    for k in (1, 4, 11, 31, 32):
        S = int(rng.integers(1, 5))
        ref, oc = None, O.OracleCounts(k, S)
        for _ in range(3):
            seqs = [rnd(int(rng.integers(0, 600))) for _ in range(int(rng.integers(1, 6)))]
            src = int(rng.integers(0, S))
            ref = O.RefIndex.counts(seqs, k, src, S, into=ref)
            oc.add(seqs, src)
        raw = ref.positions(15)
        mine, _ = _raw_from_oracle(oc)
        for f in ("count", "pos", "pair.pos"):
            assert raw[f].tolist() == mine[f].tolist(), (k, f)
        assert raw["kmer"] == mine["kmer"]
        assert ref.kmer_count == oc.kmer_count
        ref.close()


def test_count_kmers_argument_errors():
    from kmer_hasher_amd import KmerHashError, count_kmers
    cases = [
        (([], (5, 0, 1)), "seq_r should be a character vector of length at least one"),
        ((["ACGT"], (5, 0)), "k_r must be an integer vector of length 3"),
        ((["ACGT"], (0, 0, 1)), "k must be a positive integer less than 1+MAX_K"),
        ((["ACGT"], (33, 0, 1)), "k must be a positive integer less than 1+MAX_K"),
        ((["ACGT"], (5, 1, 1)), "source_n must be larger than 1 and larger than source"),
        ((["ACGT"], (5, 0, 0)), "source_n must be larger than 1 and larger than source"),
    ]
    for args, msg in cases:
        with pytest.raises(KmerHashError, match=msg.replace("+", r"\+")):
            count_kmers(*args)
    with pytest.raises(KmerHashError, match="failed to extract kmer_hash"):
        count_kmers(["ACGTACGT"], (3, 0, 1), "not a pointer")


# ------------------------------------------------------------------------------------ GPU
def _gpu_counts(case):
    from kmer_hasher_amd import count_kmers
    ptr = None
    for source, seqs in case["calls"]:
        if source < 0:
            with pytest.warns(UserWarning):
                ptr = count_kmers(seqs, (case["k"], source, case["source_n"]), ptr)
        else:
            ptr = count_kmers(seqs, (case["k"], source, case["source_n"]), ptr)
    return ptr


@pytest.mark.gpu
def test_gpu_counts_golden_khash_order(gpu, cgold):
    from kmer_hasher_amd import kmer_pos, seq_kmer_pos, set_row_order
    for case, r in cgold:
        ptr = _gpu_counts(case)
        set_row_order(ptr, "khash")
        res = kmer_pos(ptr, 15)
        assert len(res["count"]) == r["U"], case["name"]
        assert sha(res["count"]) == r["raw_sha"]["count"], case["name"]
        assert sha(res["pos"].reshape(-1)) == r["raw_sha"]["pos"], case["name"]
        assert sha(res["pair.pos"].reshape(-1)) == r["raw_sha"]["pair.pos"], case["name"]
        assert sha(res["kmer"]) == r["raw_sha"]["kmer"], case["name"]
        if len(case["query"]) > case["qk"]:
            q = seq_kmer_pos(ptr, case["query"], case["qk"])
            assert q.shape[0] == r["query"]["H"], case["name"]
            assert sha(q.reshape(-1)) == r["query"]["sha"], case["name"]
        inf = ptr.info()
        assert (inf.sources, inf.kmer_count) == (case["source_n"], r["kmer_count"])
        ptr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("table", ["adopt", "adopt-lb", "rebuild", "probe"])
def test_gpu_counts_first_order_vs_oracle(gpu, cgold, test_lib, monkeypatch, table):
    """Every way of making the counts table: the first batch's own table adopted (the default
    for a new pointer; its rows from bucket-aligned tiles offset by the bucket statistics, or by
    the look-back walk, adopt-lb: KMHG_COUNT_WALK=lb), the partitioned build over the key list
    (KMHG_COUNT_TABLE=rebuild; the default for later batches) and global linear probing (its
    overflow fallback, KMHG_COUNT_TABLE=probe)."""
    from kmer_hasher_amd import kmer_pos
    monkeypatch.setenv("KMHG_COUNT_TABLE", table.split("-")[0])
    monkeypatch.setenv("KMHG_COUNT_WALK", "lb" if table.endswith("-lb") else "b")
    for case, _ in cgold:
        oc = _oracle(case)
        ix = oc.index()
        ptr = _gpu_counts(case)
        res = kmer_pos(ptr, 15)
        assert np.array_equal(res["count"], ix.counts), case["name"]
        assert np.array_equal(res["pos"].reshape(-1), ix.pos_rows()), case["name"]
        assert np.array_equal(res["pair.pos"].reshape(-1), ix.pair_rows()), case["name"]
        assert res["kmer"] == ix.kmer_strings(), case["name"]
        ptr.free()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["place", "sort"])
@pytest.mark.parametrize("table", ["adopt", "rebuild"])
def test_gpu_counts_readout_between_batches(gpu, cgold, test_lib, monkeypatch, table, order):
    """A batch's new rows are written in slot order with their insertion-order keys and sorted
    into first-insertion order only when a readout asks for rows (ensure_row_order).  A readout
    after every call -- rows sorted, then more appended unsorted and sorted again, the earlier
    rows' counts changed by later sources -- equals the oracle each time; golden cases plus
    200 kbp batches that share half their sequence (known and new keys in one batch).  The
    order comes from the order-key placement (F, 4 B per character counted) or from the radix
    sort of the U order keys (O(U) scratch; the default beyond 8 characters per row)."""
    from kmer_hasher_amd import count_kmers, kmer_pos, synth
    monkeypatch.setenv("KMHG_COUNT_TABLE", table)
    monkeypatch.setenv("KMHG_ROW_ORDER_SORT", "1" if order == "sort" else "0")
    base = synth.add_n_runs(synth.iid(300_000, 61), 0.001, 7).tobytes().decode("latin-1")
    big = {"name": "overlap", "k": 19, "source_n": 3,
           "calls": [(0, [base[:200_000]]), (1, [base[100_000:300_000], base[:5_000]]),
                     (2, [base[250_000:], base[50_000:60_000]])]}
    for case in [c for c, _ in cgold] + [big]:
        oc = O.OracleCounts(case["k"], case["source_n"])
        ptr = None
        for source, seqs in case["calls"]:
            if source < 0:
                with pytest.warns(UserWarning):
                    ptr = count_kmers(seqs, (case["k"], source, case["source_n"]), ptr)
            else:
                ptr = count_kmers(seqs, (case["k"], source, case["source_n"]), ptr)
            oc.add(seqs, source)
            ix = oc.index()
            res = kmer_pos(ptr, 15)
            assert np.array_equal(res["count"], ix.counts), case["name"]
            assert np.array_equal(res["pos"].reshape(-1), ix.pos_rows()), case["name"]
            assert res["kmer"] == ix.kmer_strings(), case["name"]
        ptr.free()


@pytest.mark.gpu
def test_gpu_counts_errors_and_identity(gpu):
    from kmer_hasher_amd import KmerHashError, count_kmers, make_kmer_hash
    p = count_kmers(["ACGTACGTAA"], (4, 0, 2))
    assert count_kmers(["TTTTGGGG"], (4, 1, 2), p) is p          # same pointer comes back
    with pytest.raises(KmerHashError, match="mismatch between specified k"):
        count_kmers(["ACGTACGT"], (5, 0, 2), p)
    with pytest.raises(KmerHashError, match="source_n differs"):
        count_kmers(["ACGTACGT"], (4, 0, 3), p)
    ix = make_kmer_hash("ACGTACGTACGT", 4)
    with pytest.raises(KmerHashError, match="needs a counts pointer"):
        count_kmers(["ACGTACGT"], (4, 0, 1), ix)
    # only sequences of length <= k: a valid, empty counts pointer
    e = count_kmers(["ACG", "AC"], (3, 0, 1))
    assert e.info().n_kmers == 0
    from kmer_hasher_amd import kmer_pos
    r = kmer_pos(e, 15)
    assert r["count"].size == 0 and r["pos"].shape == (0, 2)
    for x in (p, ix, e):
        x.free()


@pytest.mark.gpu
def test_gpu_counts_device_api_and_large(gpu):
    """kmhg_count_device on an HBM-resident sequence; 2 Mbp counted in two sources: every
    window counted once (sum of counts = windows), identical to the host entry point."""
    import ctypes as C

    import torch
    from kmer_hasher_amd import _lib, kmer_pos, synth
    from kmer_hasher_amd.api import ExtPtr
    a = synth.add_n_runs(synth.iid(2_000_000, 31), 0.001, 3)
    b = synth.repeat_rich(1_000_000, 32, n_gap_every=250_000)
    L = _lib.lib()
    h = C.c_void_p()
    for src, arr in ((0, a), (1, b)):
        d = torch.from_numpy(arr).cuda()
        _lib.check(L.kmhg_count_device(C.byref(h), C.c_void_p(d.data_ptr()), arr.size, 25, src,
                                       2, None))
        torch.cuda.synchronize()
    dev = ExtPtr(h.value)
    oc = O.OracleCounts(25, 2)
    oc.add([a.tobytes()], 0)
    oc.add([b.tobytes()], 1)
    res = kmer_pos(dev, 10)
    ix = oc.index()
    assert np.array_equal(res["pos"].reshape(-1), ix.pos_rows())
    M = res["pos"][:, 1].reshape(-1, 2).astype(np.int64)
    assert M[:, 0].sum() == O.windows(a.tobytes(), 25)[0].size
    assert M[:, 1].sum() == O.windows(b.tobytes(), 25)[0].size
    dev.free()

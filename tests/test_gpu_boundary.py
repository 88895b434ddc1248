"""Boundary option / error paths on the GPU: do.sort=TRUE through the
C-ABI, and real results of more than 2^31-1 rows (R's int ncol, reference src/kmer_hash.c:1133,
README.md:80-89) refused with the documented error instead of overflowing."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_do_sort_true_matches_oracle(gpu, testfa):
    from kmer_hasher_amd import kmer_pos, make_kmer_hash, seq_kmer_pos, synth
    rr = synth.add_n_runs(synth.repeat_rich(300_000, 12, n_gap_every=60_000), 0.001, 13)
    for s, k in ((testfa, 15), (rr.tobytes().decode("latin-1"), 21)):
        oi = O.OracleIndex(s, k)
        for ds in (True, 1, False):
            ptr = make_kmer_hash(s, k, do_sort=ds)
            res = kmer_pos(ptr, 15)
            assert np.array_equal(res["count"], oi.counts)
            assert np.array_equal(res["pos"].reshape(-1), oi.pos_rows())
            assert np.array_equal(res["pair.pos"].reshape(-1), oi.pair_rows())
            assert np.array_equal(seq_kmer_pos(ptr, s, k).reshape(-1), oi.query(s, k))
            ptr.free()


def test_pair_rows_over_int_max_raise(gpu):
    """One k-mer seen ~70,000 times: P = C(n, 2) ~ 2.45e9 > 2^31 - 1."""
    from kmer_hasher_amd import kmer_pos, make_kmer_hash
    from kmer_hasher_amd.api import KmerHashError
    ptr = make_kmer_hash("A" * 70_001, 1)
    inf = ptr.info()
    n = inf.n_positions
    assert inf.n_kmers == 1 and inf.n_pairs == n * (n - 1) // 2 > 2**31 - 1
    with pytest.raises(KmerHashError, match="2\\^31-1 columns"):
        kmer_pos(ptr, 4)
    res = kmer_pos(ptr, 10)                     # pos + count alone are fine
    assert res["count"].tolist() == [n]
    ptr.free()


def test_query_rows_over_int_max_raise(gpu):
    """~46,343 windows of one k-mer against an index holding it ~46,342 times: H > 2^31 - 1
    (the device holds the 17 GB of rows; the host copy is refused)."""
    from kmer_hasher_amd import make_kmer_hash, seq_kmer_pos
    from kmer_hasher_amd.api import KmerHashError
    ptr = make_kmer_hash("A" * 46_342, 1)
    n = ptr.info().n_positions
    assert n * len(O.windows("A" * 46_343, 1)[0]) > 2**31 - 1
    with pytest.raises(KmerHashError, match="2\\^31-1 columns"):
        seq_kmer_pos(ptr, "A" * 46_343, 1)
    ptr.free()


@pytest.mark.parametrize("case", ["self", "related", "repeats"])
def test_query_rows_to_host_as_runs(gpu, test_lib, monkeypatch, case):
    """seq.kmer.pos into a host matrix (kmhg_query_fill) from 512 K rows on: the rows cross PCIe
    as diagonal runs and host threads expand them; results equal the oracle's with runs and with
    the plain copy (KMHG_HOST_RUNS=0): a self dot plot (one run per stretch between repeats), a
    related sequence (SNVs, rearrangements, N-runs), and repeat-rich rows that do not shrink
    (the plain copy is taken).  Odd row counts split unevenly over the host threads."""
    from kmer_hasher_amd import make_kmer_hash, seq_kmer_pos, synth
    k = 21
    if case == "repeats":
        a = synth.repeat_rich(700_000, 12, n_gap_every=70_001)
    else:
        a = synth.add_n_runs(synth.iid(1_300_001, 8), 0.0005, 3)
    b = synth.derived(a, 6, 0.01, 3) if case == "related" else a
    A, B = a.tobytes().decode("latin-1"), b.tobytes().decode("latin-1")
    want = O.OracleIndex(A, k).query(B, k)
    assert want.size // 2 >= (1 << 19)
    ptr = make_kmer_hash(A, k)
    for runs in ("1", "0"):
        monkeypatch.setenv("KMHG_HOST_RUNS", runs)
        got = seq_kmer_pos(ptr, B, k)
        assert np.array_equal(got.reshape(-1), want), runs
    ptr.free()


def test_pair_rows_to_host_generated(gpu, test_lib, monkeypatch):
    """kmer.pos pair rows into a host matrix from 4 M rows on are written by host threads from
    the keys' position lists (kmhg_positions_fill): identical to the device-made rows copied over
    (KMHG_HOST_PAIRS=0) and to the oracle, for a 150-copy family, a 20-copy family and a 5 kb
    poly-A run (one key with ~5,000 positions: 12 M pairs), with the stripes of the host threads
    cutting through keys and through one key's rows."""
    from kmer_hasher_amd import kmer_pos, make_kmer_hash, synth
    rng = np.random.default_rng(17)
    s = synth.iid(2_000_000, 21).copy()
    fam = synth.iid(500, 22)
    for at in rng.choice(np.arange(10_000, 1_900_000, 1_000), 150, replace=False):
        s[at:at + 500] = fam
    fam2 = synth.iid(3_000, 23)
    for at in range(1_950_000, 1_950_000 + 20 * 3_001, 3_001)[:16]:
        s[at:at + 3_000] = fam2
    s[5_000:10_000] = ord("A")
    A = s.tobytes().decode("latin-1")
    oi = O.OracleIndex(A, 21)
    want = oi.pair_rows()
    assert want.size // 3 >= (1 << 22)
    ptr = make_kmer_hash(A, 21)
    got = {}
    for hp in ("1", "0"):
        monkeypatch.setenv("KMHG_HOST_PAIRS", hp)
        res = kmer_pos(ptr, 2 + 4 + 8)
        got[hp] = res["pair.pos"].reshape(-1)
        assert np.array_equal(res["pos"].reshape(-1), oi.pos_rows())
        assert np.array_equal(res["count"], oi.counts)
    ptr.free()
    assert np.array_equal(got["0"], want)
    assert np.array_equal(got["1"], want)


def test_large_host_string_ends_at_nul(gpu):
    """kmhg_build / kmhg_query_run of a host string of >= 4 MB: the NUL scan runs beside the
    copy of all L bytes, and the sequence still ends at its first NUL (a C string)."""
    import ctypes as C
    from kmer_hasher_amd import _lib, synth
    k = 21
    s = synth.iid(6_000_000, 41)
    s[3_000_001] = 0
    buf = s.tobytes()
    pre = buf[:3_000_001]
    oi = O.OracleIndex(pre, k)
    out = C.c_void_p()
    _lib.check(_lib.lib().kmhg_build(buf, len(buf), k, 0, C.byref(out)))
    q, h = C.c_void_p(), C.c_int64()
    _lib.check(_lib.lib().kmhg_query_run(out, buf, len(buf), k, C.byref(q), C.byref(h)))
    rows = np.empty(2 * h.value, np.int32)
    _lib.check(_lib.lib().kmhg_query_fill(q, C.c_void_p(rows.ctypes.data)))
    _lib.lib().kmhg_query_free(q)
    want = oi.query(pre, k)
    assert np.array_equal(rows, want)
    _lib.lib().kmhg_free(out)

"""Read counting on the GPU (count.kmers.fq.sh.rp -> seq.kmer.depth.sh / kmer.spec.sh.n,
SURVEY.md §8 f next-4): the HIP path through the C-ABI against the reference's golden vectors
(tests/golden/sh_golden.json, made from the compiled reference core) and against the oracle at
larger sizes.  Keys and counts are compared as the key-sorted table (the suffix hash has no
row order the reference exposes: depth and spectrum are order-free)."""
import ctypes as C

import numpy as np
import pytest

import sh_inputs as I
from kmh_canon import sha
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLD = I.load_golden()


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    return I.materialise(str(tmp_path_factory.mktemp("shg")))


def _params(k, pb, mq, mr, S, src):
    return [k, pb, mq, 1, mr, 1, S, src]


def _sorted_table(ptr):
    from kmer_hasher_amd import api
    keys, M = api.counts_table(ptr)
    o = np.argsort(keys, kind="stable")
    return keys[o], M[o]


@pytest.mark.parametrize("table", ["adopt", "adopt-lb", "rebuild"])
@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: c["name"])
def test_sh_golden(gpu, case, inputs, test_lib, monkeypatch, table):
    """`table`: the first batch's table adopted as the suffix hash (default; rows from
    bucket-aligned tiles, or from the look-back walk with adopt-lb: KMHG_COUNT_WALK=lb) or
    rebuilt from the key list (KMHG_COUNT_TABLE=rebuild, the path of every later batch)."""
    from kmer_hasher_amd import api
    monkeypatch.setenv("KMHG_COUNT_TABLE", table.split("-")[0])
    monkeypatch.setenv("KMHG_COUNT_WALK", "lb" if table.endswith("-lb") else "b")
    files, genome = inputs
    ptr = None
    for f, pb, mq, mr, src in case["calls"]:
        ptr = api.count_kmers_fq_sh_rp(files[f], _params(case["k"], pb, mq, mr, case["source_n"],
                                                         src), ptr)
    inf = ptr.info()
    assert inf.kind == 2 and inf.sources == case["source_n"] and inf.k == case["k"]
    keys, M = _sorted_table(ptr)
    assert len(keys) == case["U"]
    assert sha(keys) == case["keys_sha"]
    assert sha(M.astype(np.int32)) == case["counts_sha"]
    strings = I.depth_strings(genome, case["k"])
    for d in case["depth"]:
        got = api.seq_kmer_depth_sh(ptr, strings[d["string"]], case["k"])   # (S, L)
        assert sha(np.ascontiguousarray(got.T)) == d["sha"], d
    for sp in case["spectra"]:
        got = api.kmer_spec_sh_n(ptr, sp["max_count"], sp["comb"], sp["comb_inner"],
                                 sp["source_min"])
        assert sha(np.ascontiguousarray(got)) == sp["sha"]


def test_sh_depth_short_and_edge_strings(gpu, inputs):
    """Strings the golden set leaves out (L < k: the reference writes before its buffer) and
    NUL-terminated input: all NA where nothing is written, as the oracle defines it."""
    from kmer_hasher_amd import api
    files, genome = inputs
    k = 15
    ptr = api.count_kmers_fq_sh_rp(files["sim.fq"], _params(k, 10, 0, -1, 1, 0))
    o = O.OracleSH(k, 1).add_fastq(files["sim.fq"], 0, 2**62, 0)
    for s in I.depth_strings(genome, k) + [genome[:40] + b"\0" + genome[50:90]]:
        want = o.depth(s.split(b"\0")[0], k)
        got = api.seq_kmer_depth_sh(ptr, s, k).T
        assert np.array_equal(got[:len(want)], want)
        assert (got[len(want):] == np.iinfo(np.int32).min).all()


def test_sh_errors_and_noops(gpu, inputs, tmp_path):
    from kmer_hasher_amd import api
    files, genome = inputs
    E = api.KmerHashError
    with pytest.raises(E, match="k must be a positive integer"):
        api.count_kmers_fq_sh_rp(files["sim.fq"], _params(0, 10, 0, -1, 1, 0))
    with pytest.raises(E, match="Source_n must be in the range 1 - 4"):
        api.count_kmers_fq_sh_rp(files["sim.fq"], _params(15, 10, 0, -1, 5, 0))
    with pytest.raises(E, match="source_i must be less than source_n"):
        api.count_kmers_fq_sh_rp(files["sim.fq"], _params(15, 10, 0, -1, 2, 2))
    with pytest.raises(E, match="k_r must be an integer vector of length 6"):
        api.count_kmers_fq_sh_rp(files["sim.fq"], [15, 10, 0])
    ptr = api.count_kmers_fq_sh_rp(files["sim.fq"], _params(15, 10, 0, 200, 2, 0))
    keys0, M0 = _sorted_table(ptr)
    # into an existing hash: a different k or a source >= its counts_n counts nothing
    api.count_kmers_fq_sh_rp(files["sim.fq"], _params(17, 10, 0, -1, 2, 1), ptr)
    api.count_kmers_fq_sh_rp(files["sim.fq"], _params(15, 10, 0, -1, 4, 3), ptr)
    keys1, M1 = _sorted_table(ptr)
    assert np.array_equal(keys0, keys1) and np.array_equal(M0, M1)
    # a missing file: the reference's reader reads nothing; a new, empty hash
    empty = api.count_kmers_fq_sh_rp(str(tmp_path / "nope.fq"), _params(15, 10, 0, -1, 1, 0))
    assert empty.info().n_kmers == 0
    d = api.seq_kmer_depth_sh(empty, genome[:100], 15)
    assert (d[:, :85] == 0).sum() > 0 and d.shape == (1, 100)
    with pytest.raises(E, match="Receieved error from seq_kmer_counts"):
        api.seq_kmer_depth_sh(ptr, genome[:100], 16)
    with pytest.raises(E, match="unable to obtain suffix_hash_n"):
        api.seq_kmer_depth_sh(api.make_kmer_hash(genome[:100], 15), genome[:100], 15)
    with pytest.raises(E, match="incorrect tag"):
        api.kmer_pos(ptr, 15)
    with pytest.warns(UserWarning, match="returned an error: -3"):
        z = api.kmer_spec_sh_n(ptr, 5, [1], [2], [1, 1])
    assert not z.any()
    with pytest.warns(UserWarning, match="returned an error: -4"):
        api.kmer_spec_sh_n(ptr, 5, [4], [0], [1, 1])


def _pack(torch, seq, qual, hasq=None):
    n, rl = seq.shape
    flat = np.zeros(n * rl + 16, np.uint8)
    flat[:n * rl] = seq.reshape(-1)
    qf = np.zeros(n * rl + 16, np.uint8)
    qf[:n * rl] = qual.reshape(-1)
    off = (np.arange(n + 1, dtype=np.int64) * rl)
    hq = np.ones(n, np.uint8) if hasq is None else hasq
    t = lambda a: torch.from_numpy(a).to("cuda")  # noqa: E731
    return t(flat), t(qf), t(off), t(hq)


def _oracle_counts(seq, qual, hasq, k, mq):
    ks = [O.read_kmers(s.tobytes(), q.tobytes() if h else None, k, mq)
          for s, q, h in zip(seq, qual, hasq)]
    allk = np.concatenate(ks) if ks else np.empty(0, np.uint64)
    return np.unique(allk, return_counts=True)


@pytest.mark.parametrize("k,mq", [(31, 20), (21, 0), (11, 30)])
def test_sh_device_reads_match_oracle(gpu, k, mq):
    """Device-resident packed reads (kmhg_sh_count_reads_device): 60 K reads x 150 bp of an
    iid genome with N calls, one third of them as FASTA records (N-only iterator)."""
    torch = gpu
    from kmer_hasher_amd import _lib, api, synth
    g = synth.add_n_runs(synth.iid(400_000, 41), 0.001, 42, max_run=30)
    seq, qual = synth.reads(g, 60_000, 150, 43 + k)
    hasq = (np.arange(len(seq)) % 3 != 0).astype(np.uint8)
    ds, dq, do, dh = _pack(torch, seq, qual, hasq)
    h = C.c_void_p()
    prm = (C.c_int32 * 8)(k, 10, mq, 1, -1, 1, 1, 0)
    L = _lib.lib()
    _lib.check(L.kmhg_sh_count_reads_device(C.byref(h), ds.data_ptr(), dq.data_ptr(),
                                            do.data_ptr(), dh.data_ptr(), len(seq), prm, None))
    torch.cuda.synchronize()
    ptr = api.ExtPtr(h.value, tag=api.SUFFIX_HASH_N_TAG)
    keys, M = _sorted_table(ptr)
    uk, cnt = _oracle_counts(seq, qual, hasq, k, mq)
    assert np.array_equal(keys, uk)
    assert np.array_equal(M[:, 0], cnt)
    # depth of the genome, device entry point
    dseq = torch.from_numpy(g.copy()).to("cuda")
    out = torch.empty(len(g), dtype=torch.int32, device="cuda")
    _lib.check(L.kmhg_sh_depth_device(ptr.handle, dseq.data_ptr(), len(g), k, out.data_ptr(),
                                      None))
    torch.cuda.synchronize()
    o = O.OracleSH(k, 1)
    o.table = {int(a): np.array([c]) for a, c in zip(uk, cnt)}
    assert np.array_equal(out.cpu().numpy(), o.depth(g.tobytes(), k)[:, 0])


def test_sh_mixed_read_lengths(gpu, tmp_path):
    """Reads of 40..3000 bp: waves whose reads exceed the LDS staging capacity walk them from
    global memory; both paths against the oracle."""
    from kmer_hasher_amd import api, synth
    g = synth.iid(200_000, 71)
    rng = np.random.default_rng(72)
    recs = []
    for i in range(3000):
        ln = int(rng.choice([40, 150, 151, 3000], p=[.3, .4, .2, .1]))
        st = int(rng.integers(0, len(g) - ln))
        s = g[st:st + ln].tobytes()
        q = rng.integers(40, 75, ln).astype(np.uint8).tobytes()
        recs.append(b"@r%d\n%s\n+\n%s\n" % (i, s, q))
    p = str(tmp_path / "mixed.fq")
    open(p, "wb").write(b"".join(recs))
    for k, mq in [(21, 10), (31, 3)]:
        ptr = api.count_kmers_fq_sh_rp(p, [k, 20, mq, 1, -1, 1, 1, 0])
        keys, M = _sorted_table(ptr)
        ok, om = O.OracleSH(k, 1).add_fastq(p, mq, 2**62, 0).arrays()
        assert np.array_equal(keys, ok) and np.array_equal(M, om)


@pytest.mark.parametrize("seed", range(10, 16))
def test_sh_fuzz_fastx(gpu, seed, tmp_path):
    """Random FASTX files (multi-line, CRLF, N runs, random phred, FASTA records first) at
    several k and thresholds against the oracle: the per-base automaton of the kernel equals
    the reference's nested iterator."""
    from kmer_hasher_amd import api
    p = str(tmp_path / "f.fq")
    open(p, "wb").write(I.random_fastx(500, seed))
    for k, mq in [(3, 0), (8, 15), (17, 25), (31, 5)]:
        ptr = api.count_kmers_fq_sh_rp(p, [k, min(8, 2 * k), mq, 1, -1, 1, 2, 1])
        keys, M = _sorted_table(ptr)
        ok, om = O.OracleSH(k, 2).add_fastq(p, mq, 2**62, 1).arrays()
        assert np.array_equal(keys, ok) and np.array_equal(M, om), (k, mq)


def _last_batch(ptr):
    from kmer_hasher_amd import _lib
    est, sp, path = C.c_double(), C.c_int(), C.c_int()
    _lib.check(_lib.lib().kmhg_sh_last_batch(ptr.handle, C.byref(est), C.byref(sp),
                                             C.byref(path)))
    return est.value, sp.value, path.value


def _count_packed(torch, seq, qual, k, mq, ptr=None, source=0, S=1):
    from kmer_hasher_amd import _lib, api
    ds, dq, do, dh = _pack(torch, seq, qual)
    h = C.c_void_p(ptr.handle.value if ptr is not None else None)
    prm = (C.c_int32 * 8)(k, 10, mq, 1, -1, 1, S, source)
    _lib.check(_lib.lib().kmhg_sh_count_reads_device(C.byref(h), ds.data_ptr(), dq.data_ptr(),
                                                     do.data_ptr(), dh.data_ptr(), len(seq), prm,
                                                     None))
    torch.cuda.synchronize()
    return ptr if ptr is not None else api.ExtPtr(h.value, tag=api.SUFFIX_HASH_N_TAG)


@pytest.mark.parametrize("table", ["adopt", "rebuild"])
@pytest.mark.parametrize("env,want_path", [({}, 1), ({"KMHG_CO_SPREAD": "8"}, 2),
                                           ({"KMHG_CO_GLOBAL": "1"}, 3)])
def test_sh_count_only_build_paths(gpu, test_lib, monkeypatch, env, want_path, table):
    """Every path of the count-only batch build, forced, against the oracle: the spread chosen
    from the batch's own HLL estimate (1), a spread too wide for low-coverage reads (distinct /
    stream ~ 0.9: KMHG_CO_SPREAD=8 overflows a sub-table -> the batch is rebuilt at spread 1)
    (2), and the global find-or-insert fallback (3), whose stream-sized table is never adopted."""
    torch = gpu
    from kmer_hasher_amd import synth
    monkeypatch.setenv("KMHG_COUNT_TABLE", table)
    for kk, v in env.items():
        monkeypatch.setenv(kk, v)
    g = synth.iid(3_000_000, 81)
    seq, qual = synth.reads(g, 20_000, 150, 82)
    k, mq = 31, 10
    ptr = _count_packed(torch, seq, qual, k, mq)
    est, sp, path = _last_batch(ptr)
    assert path == want_path, (est, sp, path)
    keys, M = _sorted_table(ptr)
    uk, cnt = _oracle_counts(seq, qual, np.ones(len(seq), np.uint8), k, mq)
    assert np.array_equal(keys, uk) and np.array_equal(M[:, 0], cnt)


def test_sh_spread_per_batch(gpu):
    """The spread comes from each batch's own distinct / stream estimate, not from an earlier
    batch: a deep-coverage batch (spread > 1) followed by a low-coverage batch of another genome
    into the same hash builds at spread 1 without an overflow; the HLL estimate (256 registers:
    standard error 1.04 / 16 = 6.5 %) is within 25 % of the true number of distinct k-mers;
    counts equal the oracle's after both batches."""
    torch = gpu
    from kmer_hasher_amd import synth
    k, mq = 31, 10
    g1 = synth.iid(500_000, 91)
    s1, q1 = synth.reads(g1, 40_000, 150, 92)                 # ~12x coverage
    ptr = _count_packed(torch, s1, q1, k, mq)
    est1, sp1, path1 = _last_batch(ptr)
    u1 = len(_oracle_counts(s1, q1, np.ones(len(s1), np.uint8), k, mq)[0])
    assert sp1 > 1 and path1 == 1
    assert abs(est1 - u1) < 0.25 * u1, (est1, u1)
    g2 = synth.iid(4_000_000, 93)
    s2, q2 = synth.reads(g2, 20_000, 150, 94)                 # ~0.75x coverage
    _count_packed(torch, s2, q2, k, mq, ptr)
    est2, sp2, path2 = _last_batch(ptr)
    assert sp2 == 1 and path2 == 1, (est2, sp2, path2)
    keys, M = _sorted_table(ptr)
    seq = np.concatenate([s1, s2])
    qual = np.concatenate([q1, q2])
    uk, cnt = _oracle_counts(seq, qual, np.ones(len(seq), np.uint8), k, mq)
    assert np.array_equal(keys, uk) and np.array_equal(M[:, 0], cnt)


def test_sh_padded_stream_edges(gpu):
    """The iterator writes each read's k-mers into a range sized by its upper bound
    (length - k + 1) and pads the rest with EMPTY_KEY, which the count-only build skips: a batch
    with 90 % of its reads rejected by quality (mostly padding), and a batch with every window
    rejected (no key at all), fresh and into an existing hash, against the oracle."""
    torch = gpu
    from kmer_hasher_amd import synth
    k, mq = 25, 10
    g = synth.iid(1_000_000, 101)
    seq, qual = synth.reads(g, 30_000, 150, 102)
    bad = qual.copy()
    bad[np.arange(len(seq)) % 10 != 0] = ord("!")        # q = 0: every window rejected
    ptr = _count_packed(torch, seq, bad, k, mq)
    keys, M = _sorted_table(ptr)
    uk, cnt = _oracle_counts(seq, bad, np.ones(len(seq), np.uint8), k, mq)
    assert len(uk) > 0 and np.array_equal(keys, uk) and np.array_equal(M[:, 0], cnt)
    est, sp, path = _last_batch(ptr)
    assert path == 1 and abs(est - len(uk)) < 0.25 * len(uk), (est, len(uk))
    # every window rejected: nothing counted, fresh or into the existing hash
    none = np.full_like(qual, ord("!"))
    empty = _count_packed(torch, seq, none, k, mq)
    assert empty.info().n_kmers == 0
    _count_packed(torch, seq, none, k, mq, ptr)
    keys2, M2 = _sorted_table(ptr)
    assert np.array_equal(keys2, keys) and np.array_equal(M2, M)

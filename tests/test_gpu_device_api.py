"""Device-resident API (inputs in HBM), window-range query shards and index images on one GPU."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _seq(torch, n=300_000, seed=6):
    from kmer_hasher_amd import synth
    s = synth.add_lowercase(synth.add_n_runs(synth.repeat_rich(n, seed, n_gap_every=50_000),
                                             0.002, 3), 0.05, 4)
    return s, torch.from_numpy(s).cuda()


def test_device_build_query_positions_match_oracle(gpu):
    torch = gpu
    from kmer_hasher_amd.device import DeviceIndex
    s, t = _seq(torch)
    for k in (17, 31):
        idx = DeviceIndex.build(t, k)
        oi = O.OracleIndex(s.tobytes(), k)
        inf = idx.info()
        assert (inf["n_kmers"], inf["n_positions"], inf["n_pairs"]) == (oi.U, oi.N, oi.P)
        res = idx.positions(15)
        assert np.array_equal(res["count"].cpu().numpy(), oi.counts)
        assert np.array_equal(res["pos"].cpu().numpy().reshape(-1), oi.pos_rows())
        assert np.array_equal(res["pair.pos"].cpu().numpy().reshape(-1), oi.pair_rows())
        q = idx.query(t, k)
        assert np.array_equal(q.rows().cpu().numpy().reshape(-1), oi.query(s.tobytes(), k))
        q.free()
        idx.free()


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_range_shards_concatenate_to_full_query(gpu, nshards):
    torch = gpu
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd.device import DeviceIndex
    s, t = _seq(torch, 200_000, 8)
    k = 21
    idx = DeviceIndex.build(t, k)
    want = O.OracleIndex(s.tobytes(), k).query(s.tobytes(), 19)
    eng = kd.HipQueryEngine(idx)
    parts = [eng.query_range(t, 19, a, b) for a, b in kd.shard_ranges(t.numel() - 19 + 1, nshards)]
    got = torch.cat(parts).cpu().numpy().reshape(-1)
    assert np.array_equal(got, want)


def test_rows_view_owns_its_query(gpu):
    """DeviceQuery.rows_view: the rows where the emit wrote them, alive after the query object,
    the index and further queries (whose buffers must not reuse the view's) are gone."""
    import gc
    torch = gpu
    from kmer_hasher_amd.device import DeviceIndex
    s, t = _seq(torch, 120_000, 12)
    idx = DeviceIndex.build(t, 23)
    want = O.OracleIndex(s.tobytes(), 23).query(s.tobytes(), 23)
    v = idx.query(t, 23).rows_view()
    gc.collect()
    for _ in range(3):                       # pool traffic while the view is alive
        idx.query(t, 23).rows_view()
    idx.free()
    gc.collect()
    assert v.is_cuda and v.device == t.device
    assert v.dtype == torch.int32 and v.shape == (len(want) // 2, 2)
    assert np.array_equal(v.cpu().numpy().reshape(-1), want)
    empty = DeviceIndex.build(t[:1000], 31)
    z = empty.query(torch.full((500,), ord("N"), dtype=torch.uint8, device=t.device), 31)
    assert z.n_rows == 0 and z.rows_view().shape == (0, 2)
    assert z.device == t.device and z.rows_view().device == t.device   # empty rows: same device
    # ... also when the current device is another one than the query's
    with torch.cuda.device(t.device):
        assert z.rows_view().device == t.device


def test_image_export_import_roundtrip(gpu):
    torch = gpu
    from kmer_hasher_amd.device import DeviceIndex
    s, t = _seq(torch, 150_000, 10)
    a = DeviceIndex.build(t, 25)
    meta, bufs = a.export_image()
    assert int(meta[10]) > 0                 # the diagonal path's code block travels too
    b = DeviceIndex.import_image(meta, [x.clone() for x in bufs])
    qa, qb = a.query(t, 25), b.query(t, 25)
    assert torch.equal(qa.rows(), qb.rows())
    pa, pb = a.positions(15), b.positions(15)
    for f in ("count", "pos", "pair.pos", "kmer"):
        assert torch.equal(pa[f], pb[f])
    # an image without the code block (codes_bytes 0): the importer probes the table only
    meta0 = meta.clone()
    meta0[10] = 0
    c = DeviceIndex.import_image(meta0, [x.clone() for x in bufs])
    assert torch.equal(c.query(t, 25).rows(), qa.rows())
    # an image exported after the first query (unique bits already cleared) imports the same
    meta2, bufs2 = a.export_image()
    d = DeviceIndex.import_image(meta2, [x.clone() for x in bufs2])
    assert torch.equal(d.query(t, 25).rows(), qa.rows())
    # a related query (SNVs) through the imported index vs the oracle
    from kmer_hasher_amd import synth
    B = synth.derived(s, 11)
    want = O.OracleIndex(s.tobytes(), 25).query(B.tobytes(), 25)
    got = d.query(torch.from_numpy(B).cuda(), 25).rows().cpu().numpy().reshape(-1)
    assert np.array_equal(got, want)


def test_full_size_self_query_properties(gpu):
    """Size-independent properties at BASELINE sizes (the oracle is too slow here): every window
    of a self-query matches at least itself, rows are ordered by (i, j), and an i.i.d. 40 Mbp
    sequence (every 31-mer distinct) gives exactly the identity dot plot.  40 M windows take the
    query's multi-block tile scan; the 100 Mbp k = 21 index (config 3) builds with three radix
    passes."""
    torch = gpu
    from kmer_hasher_amd import synth
    from kmer_hasher_amd.device import DeviceIndex
    for L, k in ((40_000_000, 31), (100_000_000, 21)):
        seq = torch.from_numpy(synth.iid(L, 7)).cuda()
        idx = DeviceIndex.build(seq, k)
        inf = idx.info()
        assert inf["n_positions"] == L - k + 1
        q = idx.query(seq, k)
        rows = q.rows().cpu().numpy().astype(np.int64)
        assert rows.shape[0] == q.n_rows >= L - k + 1
        i, j = rows[:, 0], rows[:, 1]
        d = np.diff(i)
        assert np.all(d >= 0) and np.all(np.diff(j)[d == 0] > 0)    # sorted by (i, j)
        assert np.count_nonzero(i - k + 1 == j) == L - k + 1         # each window finds itself
        if inf["n_kmers"] == L - k + 1:
            assert q.n_rows == L - k + 1
            assert np.array_equal(i, np.arange(k, L + 1))
        q.free()
        idx.free()
        del seq
        torch.cuda.empty_cache()

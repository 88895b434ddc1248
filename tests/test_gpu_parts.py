"""Owner-computes build (reference partition pattern src/kmer_reader.c:28-39) on
one GPU: the n parts of kmhg_build_device_part, placed by their part_info and exported with
their list ends rebased (kmhg_part_export), must reassemble into exactly the single-device
index -- the same table and positions bytes -- and answer kmer.pos / seq.kmer.pos as the oracle
does.  Includes parts that own no bucket (more parts than buckets) and the k = 32 side slot."""
import numpy as np
import pytest

from kmh_canon import oracle_index

pytestmark = pytest.mark.gpu


def _assemble_local(parts, torch):
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd.device import SLOT_BYTES, DeviceIndex
    infos = [p.part_info() for p in parts]
    lay = kd.part_layout(infos)
    dev = parts[0].device
    table = torch.full((lay["slots"] * SLOT_BYTES,), 0xAB, dtype=torch.uint8, device=dev)
    positions = torch.empty(max(1, lay["N"] * 4), dtype=torch.uint8, device=dev)
    codes = torch.empty(max(1, lay["codes_bytes"]), dtype=torch.uint8, device=dev)
    capb = lay["capb"]
    code_src = next((r for r, inf in enumerate(infos) if inf["nb"] and inf["codes_bytes"]), 0)
    for r, (p, inf) in enumerate(zip(parts, infos)):
        a = inf["b0"] * capb * SLOT_BYTES
        b = lay["pos_base"][r] * 4
        side = table[-SLOT_BYTES:] if r == lay["side_owner"] else None
        p.export_into(lay["pos_base"][r], table[a:a + inf["nb"] * capb * SLOT_BYTES], side,
                      positions[b:b + inf["n_positions"] * 4], codes if r == code_src else None)
    header = [parts[0].k, parts[0].L, (lay["nb_total"] << 32) | capb, lay["U"], lay["N"],
              lay["P"], lay["max_n"], kd.IMAGE_MAGIC]
    meta = torch.tensor(header + [table.numel(), lay["N"] * 4, lay["codes_bytes"]],
                        dtype=torch.int64)
    torch.cuda.synchronize()
    return DeviceIndex.import_image(meta, [table, positions, codes]), table, positions, lay


def _slot_sets(table, positions, capb):
    """Canonical form of a table: sorted (bucket, key, count, positions) of its occupied slots
    (the side slot is bucket nb)."""
    t = table.cpu().numpy().view(np.uint32).reshape(-1, 4)
    pos = positions.cpu().numpy().view(np.int32)
    key = t[:, 0].astype(np.uint64) | (t[:, 1].astype(np.uint64) << np.uint64(32))
    cnt, aux = t[:, 2], t[:, 3]
    occ = np.nonzero(cnt)[0]
    out = []
    for i in occ:
        c, a = int(cnt[i]), int(aux[i])
        lst = (a,) if c == 1 else tuple(pos[a - c:a].tolist())
        out.append((int(i) // capb, int(key[i]), c, lst))
    return sorted(out)


@pytest.mark.parametrize("stream", ["bid", "keys", "keys-first-pass"])
@pytest.mark.parametrize("n_parts", [1, 2, 3, 5, 8])
def test_parts_reassemble_to_the_single_build(gpu, test_lib, monkeypatch, n_parts, stream):
    """`stream`: bucket-id streams (the default up to 12 M windows), key streams whose parts
    compact their own windows in the first histogram pass and run every radix pass over those
    alone (the default beyond), and key streams with the older first pass over every window
    (KMHG_PART_COMPACT=0)."""
    torch = gpu
    monkeypatch.setenv("KMHG_BUILD_BID", "1" if stream == "bid" else "0")
    monkeypatch.setenv("KMHG_PART_COMPACT", "0" if stream == "keys-first-pass" else "1")
    from kmer_hasher_amd import synth
    from kmer_hasher_amd.device import DeviceIndex
    rr = synth.add_n_runs(synth.repeat_rich(400_000, 31, n_gap_every=70_000), 0.001, 32)
    cases = [(synth.iid(300_000, 33), 31), (rr, 21), (rr, 9),
             (np.frombuffer(b"G" * 40 + b"ACGT" * 800 + b"G" * 35, np.uint8), 32),
             (synth.iid(3_000, 34), 31)]                     # 3 buckets: some parts own none
    for seq_np, k in cases:
        seq = torch.from_numpy(seq_np.copy()).cuda()
        whole = DeviceIndex.build(seq, k)
        meta_w, bufs_w = whole.export_image()
        parts = [DeviceIndex.build_part(seq, k, p, n_parts) for p in range(n_parts)]
        idx, table, positions, lay = _assemble_local(parts, torch)
        inf_w, inf_a = whole.info(), idx.info()
        for f in ("n_kmers", "n_positions", "n_pairs", "max_count", "table_slots"):
            assert inf_w[f] == inf_a[f], (k, n_parts, f)
        # the same slots per bucket (the CAS build's layout inside a bucket depends on which
        # colliding key claimed a slot first, so it is compared as a set): key, count, and the
        # position list of each key
        assert _slot_sets(table, positions, lay["capb"]) == \
            _slot_sets(bufs_w[0][:table.numel()], bufs_w[1], lay["capb"]), (k, n_parts)
        s = seq_np.tobytes()
        oi = oracle_index(s, k)
        res = idx.positions(14)
        assert np.array_equal(res["count"].cpu().numpy(), oi.counts)
        assert np.array_equal(res["pos"].cpu().numpy().reshape(-1), oi.pos_rows())
        assert np.array_equal(res["pair.pos"].cpu().numpy().reshape(-1), oi.pair_rows())
        kq = min(k, 31)
        q = idx.query(seq, kq)
        assert np.array_equal(q.rows().cpu().numpy().reshape(-1), oi.query(s, kq)), (k, n_parts)
        q.free()
        for p in parts:
            p.free()
        idx.free()
        whole.free()


def test_part_index_refuses_queries(gpu):
    torch = gpu
    from kmer_hasher_amd import _lib, synth
    from kmer_hasher_amd.device import DeviceIndex
    seq = torch.from_numpy(synth.iid(50_000, 35)).cuda()
    p = DeviceIndex.build_part(seq, 21, 0, 2)
    with pytest.raises(_lib.KmhgError, match="assembled"):
        p.query(seq, 21)
    with pytest.raises(_lib.KmhgError, match="assembled"):
        p.positions(8)
    with pytest.raises(_lib.KmhgError, match="part out of range"):
        DeviceIndex.build_part(seq, 21, 2, 2)
    p.free()


def test_merge_part_rows_interleaves_by_window(gpu):
    """kmhg_merge_part_rows on hand-made parts: windows dealt to three parts (a window's rows on
    one part, j ascending), ragged tiles (empty tiles, a window with 3,000 rows, a part with no
    rows) -> the rows ordered by window, then by the part's order, as the unsharded query."""
    import torch
    from kmer_hasher_amd.device import merge_part_rows
    rng = np.random.default_rng(5)
    k, nw, T = 21, 3 * 2048 + 77, 2048
    per_window = rng.integers(0, 3, size=nw)
    per_window[100] = 3000                     # a heavy window
    per_window[2048:4096] = 0                  # an empty tile
    owner = rng.integers(0, 2, size=nw)        # part 2 owns nothing
    rows = {0: [], 1: [], 2: []}
    want = []
    for s in range(nw):
        for j in range(per_window[s]):
            r = (s + k, int(rng.integers(1, 10**6)))
            rows[owner[s]].append(r)
            want.append(r)
    nt = (nw + T - 1) // T
    segs, offs, base = [], [], [0]
    for p in range(3):
        a = np.array(rows[p], np.int32).reshape(-1, 2)
        tiles = (a[:, 0].astype(np.int64) - k) // T
        cnt = np.bincount(tiles, minlength=nt)[:nt]
        offs.append(np.concatenate([[0], np.cumsum(cnt)]))
        segs.append(a)
        base.append(base[-1] + a.shape[0])
    allrows = torch.from_numpy(np.concatenate(segs)).cuda()
    tile_off = torch.from_numpy(np.stack(offs).astype(np.int64)).cuda()
    out = merge_part_rows(allrows, base[:3], tile_off, k).cpu().numpy()
    assert out.tolist() == [list(r) for r in want]


def test_rows_runs_round_trip_vs_reference(gpu):
    """kmhg_rows_runs / kmhg_runs_expand (the sharded query's gather format) against the numpy
    reference, run for run: one long diagonal, a shifted one, multi-hit windows (which do not
    compress: None), sorted random rows, runs across 2048-row tiles, i at the int32 edge, and
    the rows of a real related-sequence query."""
    import torch
    import runs_ref
    from test_dist_cpu import _run_cases
    from kmer_hasher_amd import synth
    from kmer_hasher_amd.device import DeviceIndex, rows_to_runs, runs_expand
    cases = _run_cases()
    a = synth.iid(300_000, 3)
    b = synth.derived(a, 4, 0.01, 3)
    idx = DeviceIndex.build(torch.from_numpy(a).cuda(), 21)
    cases["query"] = idx.query(torch.from_numpy(b).cuda(), 21).rows().cpu().numpy()
    idx.free()
    for name, rows in cases.items():
        r = np.asarray(rows, np.int64).astype(np.uint32).view(np.int32).reshape(-1, 2)
        want = runs_ref.encode(r)
        got = rows_to_runs(torch.from_numpy(np.ascontiguousarray(r)).cuda())
        if 3 * want.shape[0] >= 2 * r.shape[0]:
            assert got is None, name           # runs would not be smaller: the rows travel
            got = torch.from_numpy(want).cuda()
        else:
            assert got is not None and np.array_equal(got.cpu().numpy(), want), name
        out = torch.full((r.shape[0], 2), -7, dtype=torch.int32, device="cuda")
        runs_expand(got, r.shape[0], out)
        assert np.array_equal(out.cpu().numpy(), r), name
    assert cases["query"].shape[0] > 100_000


def test_seq_pack_unpack_vs_reference(gpu):
    """kmhg_seq_pack / kmhg_seq_unpack (C1's wire format) against the numpy reference, word for
    word and char for char: arbitrary bytes, N / n, lower case, ragged lengths, slices [a, b)
    with unaligned ends, an unaligned source pointer."""
    import torch
    import runs_ref
    from kmer_hasher_amd.device import seq_pack, seq_unpack
    rng = np.random.default_rng(9)
    for L in (1, 15, 16, 17, 4096, 100_003):
        s = rng.integers(0, 256, L + 1).astype(np.uint8)
        s[::5] = ord("N")
        s[2::13] = ord("n")
        s[1::3] = np.frombuffer(b"acgtACGT", np.uint8)[rng.integers(0, 8, s[1::3].size)]
        for off in (0, 1):                   # off = 1: the sequence starts 1 B past alignment
            src = torch.from_numpy(s).cuda()[off:off + L]
            code, nbit = seq_pack(src)
            rc, rn = runs_ref.seq_pack(s[off:off + L])
            assert np.array_equal(code.cpu().numpy(), rc), (L, off)
            assert np.array_equal(nbit.cpu().numpy(), rn), (L, off)
            for a, b in [(0, L), (min(16, L), L), (L // 3 // 16 * 16, L - L // 5), (L, L),
                         (min(5, L), L)]:
                w0 = a // 16
                out = torch.full((L + 16,), 7, dtype=torch.uint8, device="cuda")
                seq_unpack(code[w0:], nbit[w0:], w0, a, b, out)
                want = np.full(L + 16, 7, np.uint8)
                runs_ref.seq_unpack(rc[w0:], rn[w0:], w0, a, b, want)
                assert np.array_equal(out.cpu().numpy(), want), (L, off, a, b)


@pytest.mark.parametrize("case", ["self", "related", "repeats", "dups"])
def test_query_range_runs_expand_to_rows(gpu, case):
    """kmhg_query_run_device_range_runs (a sharded-query sender's runs, made from the window
    records without writing rows) expands to exactly kmhg_query_run_device_range's rows, for
    ragged window ranges (a range starting mid-tile, one ending at the sequence end, an empty
    one); repeat-rich rows come back as rows (runs would not be smaller); duplicated stretches
    put multi-hit windows (a run per row) among the diagonals."""
    import torch
    from kmer_hasher_amd import synth
    from kmer_hasher_amd.device import DeviceIndex, runs_expand
    k = 21
    a = synth.repeat_rich(400_000, 5, n_gap_every=40_001) if case == "repeats" else \
        synth.add_n_runs(synth.iid(400_000, 31), 0.001, 4)
    if case == "dups":                  # multi-hit windows among long diagonals
        a[200_000:203_000] = a[1_000:4_000]
        a[300_000:300_500] = a[1_200:1_700]
    b = synth.derived(a, 7, 0.01, 3) if case == "related" else a
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    idx = DeviceIndex.build(ta, k)
    nw = b.size - k + 1
    kinds = set()
    for w0, w1 in [(0, nw), (1_000, 250_000), (123_457, nw), (5_000, 5_000), (nw - 3, nw)]:
        want = idx.query_range(tb, k, w0, w1).rows().cpu().numpy()
        kind, t, h = idx.query_range_runs(tb, k, w0, w1)
        kinds.add(kind)
        assert h == want.shape[0], (w0, w1)
        if kind == "runs":
            out = torch.empty((h, 2), dtype=torch.int32, device="cuda")
            runs_expand(t, h, out)
            got = out.cpu().numpy()
        else:
            got = t.cpu().numpy()
        assert np.array_equal(got, want), (case, w0, w1)
    idx.free()
    assert "runs" in kinds if case != "repeats" else True

"""Multi-rank sharded seq.kmer.pos on CPU: gloo, world_size 2 (and 3), the oracle standing in
for the per-rank HIP engine.  Checks that shard edges (N runs, the end-drop rule, query k !=
index k) and the gather order reproduce the unsharded reference rows exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kmer_hasher_amd import dist as kd
from kmer_hasher_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class OracleEngine:
    """Per-rank engine for the CPU test: oracle rows of windows [w0, w1) of the full query."""

    def __init__(self, seq_bytes, k_index):
        from oracle import oracle as O
        self.oi = O.OracleIndex(seq_bytes, k_index)

    def query_range(self, seq, k, w0, w1):
        rows = self.oi.query(seq.numpy().tobytes(), k).reshape(-1, 2)
        ends = rows[:, 0].astype(np.int64)          # i = window start (0-based) + k
        keep = (ends - k >= w0) & (ends - k < w1)
        return torch.from_numpy(np.ascontiguousarray(rows[keep]))


def _worker(rank, world, port, seq_bytes, k_index, kq, out_q, codec=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = OracleEngine(seq_bytes, k_index)
        if codec:                      # rows to the root as diagonal runs (dist.gather_rows)
            import runs_ref
            eng.codec = runs_ref.NumpyRunCodec()
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy())
        # image broadcast path (generic buffer broadcast) round-trips bytes exactly
        meta = torch.tensor([0] * 8 + [7, 3, 5, 11, 13], dtype=torch.int64) if rank == 0 else None
        bufs = [torch.arange(s % 251, dtype=torch.uint8) for s in (7, 3, 5, 11, 13)] \
            if rank == 0 else None
        m, b = kd.broadcast_buffers(meta, bufs, 0, torch.device("cpu"))
        ok_bcast = [x.numel() for x in b] == [7, 3, 5, 11, 13] and m.tolist()[8:] == [7, 3, 5, 11, 13]
        ok_bcast = ok_bcast and all(torch.equal(x, torch.arange(s % 251, dtype=torch.uint8))
                                    for x, s in zip(b, (7, 3, 5, 11, 13)))
        rows = kd.sharded_query(eng, seq, kq, dst=0)
        if rank == 0:
            out_q.put((ok_bcast, rows.numpy().reshape(-1).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k_index,kq,codec", [(2, 15, 15, False), (2, 16, 12, False),
                                                    (3, 31, 31, False), (2, 15, 15, True),
                                                    (3, 31, 31, True)])
def test_sharded_query_matches_unsharded(world, k_index, kq, codec):
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(60_000, 5, n_gap_every=7_001), 0.01, 9)
    s[-k_index - 3] = ord("N")        # an end-drop case near the last shard's edge
    seq_bytes = s.tobytes()
    want = O.OracleIndex(seq_bytes, k_index).query(seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seq_bytes, k_index, kq, q, codec))
             for r in range(world)]
    for p in procs:
        p.start()
    ok_bcast, got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert ok_bcast
    assert got == want


def _c1_worker(rank, world, port, seq_bytes, k_index, kq, c1, host, out_q, codecs=False):
    """The R session's query on rank 0 only: C1 by scatter (each rank receives the slice its
    windows read) or broadcast, rows gathered on rank 0's device or delivered by every rank into
    the shared host matrix; twice through one sink / one receive buffer (reuse).  codecs: the
    sequence travels packed and the rows as diagonal runs (the numpy wire-format references)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sink = kd.HostRowSink(0) if host else None
    try:
        eng = OracleEngine(seq_bytes, k_index)
        if codecs:
            import runs_ref
            eng.codec = runs_ref.NumpyRunCodec()
            eng.seq_codec = runs_ref.NumpySeqCodec()
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()) if rank == 0 else None
        buf = torch.full((len(seq_bytes) + 16,), ord("A"), dtype=torch.uint8) if rank else None
        got = []
        for _ in range(2):
            ph = {}
            rows = kd.sharded_query(eng, seq, kq, dst=0, src=0, c1=c1, sink=sink, seq_buf=buf,
                                    timings=ph)
            assert set(ph) == {"broadcast", "query", "gather"}
            if rank == 0:
                got.append(rows.numpy().reshape(-1).tolist())
            else:
                assert rows is None
        if rank == 0:
            out_q.put(got)
    finally:
        if sink is not None:
            sink.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,c1,host,codecs", [
    (2, "scatter", False, False), (2, "scatter", True, False), (3, "scatter", True, False),
    (3, "broadcast", True, False), (2, "scatter", False, True), (3, "scatter", False, True),
    (3, "broadcast", False, True)])
def test_sharded_query_scatter_and_host_rows(world, c1, host, codecs):
    """C1 as a scatter of slices and rows delivered into one shared host matrix reproduce the
    unsharded reference rows exactly, including an N right at a shard edge and the end-drop
    rule; the shared-memory segment is gone afterwards.  With the wire codecs
    (packed sequence, rows as runs) on a sequence with lower case and IUPAC letters."""
    from oracle import oracle as O
    k = 21
    s = synth.add_n_runs(synth.iid(40_000, 77), 0.01, 9)
    if codecs:
        s = synth.add_ambiguity(synth.add_lowercase(s, 0.1, 3), 0.01, 4)
    n_w = len(s) - k + 1
    for a, _ in kd.shard_ranges(n_w, world)[1:]:
        s[a - 1] = ord("N")            # the char before a shard's first window
        s[a + k - 1] = ord("N")        # the last char of a shard's first window
    s[-k - 1] = ord("N")
    seq_bytes = s.tobytes()
    want = O.OracleIndex(seq_bytes, k).query(seq_bytes, k).tolist()
    before = set(os.listdir("/dev/shm"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c1_worker,
                         args=(r, world, port, seq_bytes, k, k, c1, host, q, codecs))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got[0] == want and got[1] == want
    assert not [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("kmhg_rows")]


def _run_cases():
    rng = np.random.default_rng(5)
    diag = np.stack([np.arange(100, 5100), np.arange(7, 5007)], 1)       # one long diagonal
    cut = diag.copy()
    cut[1000:] += [0, 3]                                                 # a shifted diagonal
    rep = np.repeat(np.arange(50, 90), 3)                                # 3 hits per window
    reps = np.stack([rep, np.tile([5, 900, 77_000], 40)], 1)
    rnd = np.sort(rng.integers(1, 1 << 30, (3000, 2)), 0)
    big = np.stack([np.arange(1 << 20), np.arange(1 << 20)], 1) + [31, 1]
    big[::4097] += [0, 11]
    return {"empty": np.zeros((0, 2)), "one": np.array([[40, 9]]), "diag": diag, "cut": cut,
            "repeats": reps, "random": rnd, "tiles": big,
            "wrap": np.array([[2**31 - 2, 5], [2**31 - 1, 6], [-2**31, 7]])}


def test_seq_codec_reference():
    """The numpy sequence packing keeps what the reference reads of every char: the 2-bit code
    and the N test (lower case, IUPAC letters, other bytes), for every slice [a, b)."""
    import runs_ref
    rng = np.random.default_rng(3)
    s = rng.integers(0, 256, 1000).astype(np.uint8)
    s[::7] = ord("N")
    s[3::11] = ord("n")
    code, nbit = runs_ref.seq_pack(s)
    for a, b in [(0, 1000), (0, 1), (16, 999), (5, 37), (992, 1000), (500, 500)]:
        out = np.zeros(1000, np.uint8)
        w0 = a // 16
        runs_ref.seq_unpack(code[w0:], nbit[w0:], w0, a, b, out)
        got, orig = out[a:b], s[a:b]
        isn = (orig | 0x20) == ord("n")
        assert np.array_equal((got | 0x20) == ord("n"), isn)
        assert np.array_equal(((got >> 1) & 3)[~isn], ((orig >> 1) & 3)[~isn])


def test_run_codec_reference():
    """The numpy run reference round-trips every shape of row set: one long diagonal, a shifted
    one, multi-hit windows (runs of one row), sorted random rows, runs across 2048-row tiles, i
    at the int32 edge."""
    import runs_ref
    for name, rows in _run_cases().items():
        r = np.asarray(rows, np.int64).astype(np.uint32).view(np.int32).reshape(-1, 2)
        runs = runs_ref.encode(r)
        assert np.array_equal(runs_ref.decode(runs, r.shape[0]), r), name
    assert runs_ref.encode(_run_cases()["diag"]).shape == (1, 3)
    assert runs_ref.encode(_run_cases()["cut"]).shape == (2, 3)


def _codec_gather_worker(rank, world, port, out_q):
    """gather_rows with the run codec: every rank's rows of another shape (a diagonal, repeats
    that do not compress, nothing), concatenated on rank 0 in rank order."""
    import runs_ref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cases = _run_cases()
        mine = [cases["diag"], cases["repeats"], cases["empty"], cases["cut"]][rank]
        local = torch.from_numpy(np.ascontiguousarray(mine, np.int32).reshape(-1, 2))
        out = kd.gather_rows(local, 0, None, runs_ref.NumpyRunCodec())
        if rank == 0:
            out_q.put(out.numpy().tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gather_rows_with_run_codec(world):
    cases = _run_cases()
    parts = [cases["diag"], cases["repeats"], cases["empty"], cases["cut"]][:world]
    want = np.concatenate([np.asarray(p, np.int32).reshape(-1, 2) for p in parts]).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_codec_gather_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got == want


def test_slice_bounds_cover_window_rule():
    """A range's slice holds the char before its first window and the last char of its last
    window (the window rule's reads), clipped to the sequence."""
    for L, k, w0, w1 in [(1000, 31, 0, 500), (1000, 31, 500, 970), (10**6, 21, 123_457, 654_321)]:
        a, b = kd.slice_bounds(L, k, w0, w1)
        assert a <= max(0, w0 - 1) and b >= min(L, w1 + k - 1)
        assert 0 <= a and b <= L
    assert kd.slice_bounds(100, 5, 7, 7) == (0, 0)


def test_shard_ranges():
    assert kd.shard_ranges(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert kd.shard_ranges(0, 2) == [(0, 0), (0, 0)]
    r = kd.shard_ranges(1_000_003, 8)
    assert r[0][0] == 0 and r[-1][1] == 1_000_003
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))


# ------------------------------------------------------------ owner-computes assembly (gloo)
class FakePart:
    """A part of a synthetic whole index (nb_total buckets x capb 16-B slots, N positions): owns
    buckets [b0, b1) and the positions of its elements; list ends (count >= 2) are stored
    part-local and rebased by export_into, as kmhg_part_export does."""

    def __init__(self, rank, world, nb_total=11, capb=4, seed=5):
        from kmer_hasher_amd.device import SLOT_BYTES
        rng = np.random.default_rng(seed)
        self.k, self.L = 21, 5000
        slots = rng.integers(0, 2**31, size=(nb_total * capb + 1, 4), dtype=np.int64).astype(
            np.uint32)
        slots[:, 2] = rng.integers(0, 4, size=nb_total * capb + 1)          # counts 0..3
        per_bucket = rng.integers(0, 9, size=nb_total)                       # positions / bucket
        self.whole_pos = rng.integers(1, 10**6, size=int(per_bucket.sum()), dtype=np.int32)
        self.b0 = nb_total * rank // world
        self.b1 = nb_total * (rank + 1) // world
        starts = np.concatenate([[0], np.cumsum(per_bucket)])
        self.base = int(starts[self.b0])
        self.n = int(starts[self.b1] - starts[self.b0])
        self.whole_table = slots
        local = slots.copy()
        multi = local[:, 2] > 1
        local[multi, 3] = (local[multi, 3] % 1000).astype(np.uint32)
        self.whole_table[multi, 3] = local[multi, 3]           # keep aux + base in range
        self.local = local
        self.capb, self.nb_total, self.slot_bytes = capb, nb_total, SLOT_BYTES
        side_b = 3
        self.side_owner = int(self.b0 <= side_b < self.b1)
        self.codes = np.arange(24, dtype=np.uint8)

    def expected(self, world):
        t = self.whole_table.copy()
        # every part rebases its own slots by its own base
        for r in range(world):
            p = FakePart(r, world, self.nb_total, self.capb)
            a, b = p.b0 * self.capb, p.b1 * self.capb
            m = t[a:b, 2] > 1
            t[a:b][m, 3] += np.uint32(p.base)
        side_part = next(FakePart(r, world, self.nb_total, self.capb) for r in range(world)
                         if FakePart(r, world, self.nb_total, self.capb).side_owner)
        t[-1] = side_part.local[-1]
        m = t[-1, 2] > 1
        if m:
            t[-1, 3] += np.uint32(side_part.base)
        return t.view(np.uint8).reshape(-1), self.whole_pos.view(np.uint8)

    def part_info(self):
        return {"b0": self.b0, "nb": self.b1 - self.b0, "nb_total": self.nb_total,
                "capb": self.capb, "n_positions": self.n, "n_kmers": 7 * (self.b1 - self.b0),
                "n_pairs": self.n, "max_count": 3, "side_owner": self.side_owner,
                "codes_bytes": 24}

    def export_into(self, pos_base, table, side, positions, codes, stream=None):
        assert pos_base == self.base
        sl = self.local[self.b0 * self.capb:self.b1 * self.capb].copy()
        m = sl[:, 2] > 1
        sl[m, 3] += np.uint32(pos_base)
        if table is not None and table.numel():
            table.copy_(torch.from_numpy(sl.view(np.uint8).reshape(-1)))
        if side is not None:
            s = self.local[-1:].copy()
            if s[0, 2] > 1:
                s[0, 3] += np.uint32(pos_base)
            side.copy_(torch.from_numpy(s.view(np.uint8).reshape(-1)))
        if positions is not None and positions.numel():
            positions.copy_(torch.from_numpy(
                self.whole_pos[self.base:self.base + self.n].view(np.uint8).copy()))
        if codes is not None:
            codes.copy_(torch.from_numpy(self.codes))


def _assemble_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        part = FakePart(rank, world)
        meta, bufs = kd.assemble_parts(part, torch.device("cpu"),
                                       import_fn=lambda m, b: (m, b))
        want_t, want_p = part.expected(world)
        ok = (np.array_equal(bufs[0].numpy(), want_t)
              and np.array_equal(bufs[1].numpy()[:want_p.size], want_p)
              and np.array_equal(bufs[2].numpy(), part.codes)
              and meta.tolist()[:8] == [21, 5000, (11 << 32) | 4, 7 * 11, want_p.size // 4,
                                        want_p.size // 4, 3, kd.IMAGE_MAGIC])
        out_q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_assemble_parts_places_and_rebases(world):
    """assemble_parts (the all-gather of owner-computes parts) puts every part's slots at its
    bucket range, its positions at its base, rebased list ends, the side slot from its owner and
    the code block -- on every rank.  world 5 over 11 buckets: uneven parts."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_assemble_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(res[r] for r in range(world)), res


class FailingPart(FakePart):
    """A part whose build failed on its own rank (kmhg_part_info raising KMHG_EOVERFLOW)."""

    def part_info(self):
        from kmer_hasher_amd import _lib
        raise _lib.KmhgError(_lib.KMHG_EOVERFLOW, "a bucket of a part build overflowed its LDS table")


def _failing_worker(rank, world, port, bad, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        part = FailingPart(rank, world) if rank == bad else FakePart(rank, world)
        try:
            kd.assemble_parts(part, torch.device("cpu"), import_fn=lambda m, b: (m, b))
            out_q.put((rank, "assembled"))
        except Exception as e:                       # every rank must land here, none may hang
            out_q.put((rank, type(e).__name__ + ": " + str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad", [(2, 1), (3, 0)])
def test_assemble_parts_failure_reaches_every_rank(world, bad):
    """A part build that fails on one rank (its bucket overflowed: part_info raises there only)
    makes every rank raise before the first collective of the assembly, instead of the other
    ranks blocking forever in the all-gather (dist.part_info_all all-reduces the status first)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, bad, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert "overflowed" in res[bad], res
    for r in range(world):
        if r != bad:
            assert "another rank's part build failed" in res[r], res


# ------------------------------------------------------------ owner-routed query (gloo, CPU)
TILE = 2048


class FakePartEngine:
    """Rank r's part for the CPU test: the oracle's rows of the windows this rank "owns" (here a
    hash of the window index: every window's rows on exactly one rank, as the real parts own a
    window by its key), with their per-tile offsets (tiles of 2048 windows); the merge is a
    stable sort by window end (the HIP merge is tested on the GPU)."""

    def __init__(self, seq_bytes, k_index, rank, world):
        from oracle import oracle as O
        self.oi = O.OracleIndex(seq_bytes, k_index)
        self.rank, self.world = rank, world

    def query_part(self, seq, k):
        rows = self.oi.query(seq.numpy().tobytes(), k).reshape(-1, 2)
        i = rows[:, 0].astype(np.int64)
        own = ((i * 2654435761) >> 7) % self.world == self.rank
        mine = np.ascontiguousarray(rows[own])
        nw = seq.numel() - k + 1
        nt = (nw + TILE - 1) // TILE
        tiles = (mine[:, 0].astype(np.int64) - k) // TILE
        cnt = np.bincount(tiles, minlength=nt)[:nt]
        off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        return torch.from_numpy(mine), torch.from_numpy(off)

    def merge(self, rows, seg_base, tile_off, k):
        r = rows.numpy()
        assert tile_off.shape[0] == self.world and seg_base[0] == 0
        o = np.argsort(r[:, 0], kind="stable")
        return torch.from_numpy(np.ascontiguousarray(r[o]))


def _owner_worker(rank, world, port, seq_bytes, k, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = FakePartEngine(seq_bytes, k, rank, world)
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()) if rank == 0 else None
        ph = {}
        rows = kd.owner_query(eng, seq, k, dst=0, src=0, timings=ph)
        assert set(ph) == {"broadcast", "query", "gather", "merge"}
        if rank == 0:
            out_q.put(rows.numpy().reshape(-1).tolist())
        else:
            assert rows is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_owner_query_orchestration(world):
    """owner_query: the query broadcast from rank 0, every rank's owned rows and tile offsets
    gathered to rank 0 and merged back into the unsharded seq.kmer.pos rows."""
    from oracle import oracle as O
    k = 17
    s = synth.add_n_runs(synth.repeat_rich(30_000, 6, n_gap_every=7_001), 0.01, 9)
    seq_bytes = s.tobytes()
    want = O.OracleIndex(seq_bytes, k).query(seq_bytes, k).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, seq_bytes, k, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got == want

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


def _worker(rank, world, port, seq_bytes, k_index, kq, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = OracleEngine(seq_bytes, k_index)
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


@pytest.mark.parametrize("world,k_index,kq", [(2, 15, 15), (2, 16, 12), (3, 31, 31)])
def test_sharded_query_matches_unsharded(world, k_index, kq):
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(60_000, 5, n_gap_every=7_001), 0.01, 9)
    s[-k_index - 3] = ord("N")        # an end-drop case near the last shard's edge
    seq_bytes = s.tobytes()
    want = O.OracleIndex(seq_bytes, k_index).query(seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seq_bytes, k_index, kq, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ok_bcast, got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert ok_bcast
    assert got == want


def test_shard_ranges():
    assert kd.shard_ranges(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert kd.shard_ranges(0, 2) == [(0, 0), (0, 0)]
    r = kd.shard_ranges(1_000_003, 8)
    assert r[0][0] == 0 and r[-1][1] == 1_000_003
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))

"""Multi-rank seq.kmer.pos with the HIP engine, rehearsed on ONE GPU: two ranks
share cuda:0 over gloo (RCCL refuses two ranks on one device).  Rank 0 builds the index; its device
image goes to rank 1 by broadcast of HBM buffers (kmer_hasher_amd/dist.py broadcast_index); each
rank queries its window range with libkmhgpu; the rows are gathered in rank order and must equal
the oracle's unsharded seq.kmer.pos rows.  gloo moves device tensors for broadcast/all_gather but
not for point-to-point, so the per-rank rows are handed to gather_rows on the host here; on the
8-GPU node the same code runs over RCCL with the rows left in HBM."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _HostRows:
    def __init__(self, eng):
        self.eng = eng

    def query_range(self, seq, k, w0, w1):
        return self.eng.query_range(seq, k, w0, w1).cpu()


def _worker(rank, world, port, seq_bytes, k_index, kq, out_q, device_rows=False):
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd.device import DeviceIndex
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()).to(dev)
        built = DeviceIndex.build(seq, k_index) if rank == 0 else None
        idx = kd.broadcast_index(built, dev, src=0)
        info = idx.info()
        eng = kd.HipQueryEngine(idx)
        # device_rows: the engine itself, so the sender's rows leave as runs made from its
        # window records (query_range_runs) or as rows where runs would not be smaller
        rows = kd.sharded_query(eng if device_rows else _HostRows(eng), seq, kq, dst=0)
        torch.cuda.synchronize()
        if rank == 0:
            out_q.put(((info["n_kmers"], info["n_positions"]),
                       rows.cpu().numpy().reshape(-1).tolist()))
        dist.barrier()
        idx.free()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k_index,kq,seq_kind,device_rows",
                         [(2, 31, 31, "repeats", False), (2, 21, 19, "repeats", False),
                          (2, 31, 31, "repeats", True), (3, 21, 21, "dups", True)])
def test_two_ranks_one_gpu_sharded_query(gpu, world, k_index, kq, seq_kind, device_rows):
    import torch.multiprocessing as mp
    from kmer_hasher_amd import synth
    from oracle import oracle as O
    if seq_kind == "repeats":
        s = synth.add_n_runs(synth.repeat_rich(120_000, 5, n_gap_every=9_001), 0.005, 3)
    else:                               # mostly unique, a few duplicated stretches
        s = synth.add_n_runs(synth.iid(120_000, 5), 0.002, 3)
        s[70_000:71_500] = s[10_000:11_500]
        s[90_000:90_400] = s[10_200:10_600]
    s[-k_index - 2] = ord("N")          # an end-drop case in the last shard
    seq_bytes = s.tobytes()
    oi = O.OracleIndex(seq_bytes, k_index)
    want = oi.query(seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, seq_bytes, k_index, kq, q, device_rows))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        (nk, npos), got = q.get(timeout=100)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert (nk, npos) == (oi.U, oi.N)
    assert got == want


def _owner_worker(rank, world, port, seq_bytes, k, kq, out_q):
    """Owner-computes build over `world` ranks sharing cuda:0 (gloo): the sequence and the query
    live on rank 0 only and are broadcast (C1); each rank builds its bucket range
    (kmhg_build_device_part); assemble_parts all-gathers the parts into the whole index on every
    rank; then the sharded seq.kmer.pos with the query broadcast from rank 0."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import dist as kd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()).to(dev) \
            if rank == 0 else None
        part, seq_all = kd.owner_build(seq, k, dev, src=0)
        idx = kd.assemble_parts(part, dev)
        info = idx.info()
        part.free()
        timings = {}
        rows = kd.sharded_query(_HostRows(kd.HipQueryEngine(idx)), seq if rank == 0 else None,
                                kq, dst=0, src=0, timings=timings)
        torch.cuda.synchronize()
        if rank == 0:
            out_q.put(((info["n_kmers"], info["n_positions"], info["n_pairs"]),
                       rows.numpy().reshape(-1).tolist(), sorted(timings)))
        dist.barrier()
        idx.free()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,kq", [(2, 31, 31), (3, 21, 17)])
def test_owner_computes_build_and_broadcast_query(gpu, world, k, kq):
    import torch.multiprocessing as mp
    from kmer_hasher_amd import synth
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(150_000, 8, n_gap_every=11_003), 0.004, 6)
    s[-k - 2] = ord("N")
    seq_bytes = s.tobytes()
    oi = O.OracleIndex(seq_bytes, k)
    want = oi.query(seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, seq_bytes, k, kq, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        (nk, npos, npair), got, phases = q.get(timeout=100)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert (nk, npos, npair) == (oi.U, oi.N, oi.P)
    assert got == want
    assert phases == ["broadcast", "gather", "query"]


def _nccl_worker(port, seq_bytes, k, kq, out_q):
    """World size 1 over RCCL (backend "nccl"): every collective of the N > 1 path runs on the
    real backend with device tensors -- the sequence broadcast (C1), the owner-computes part build
    and its all-gather assembly, the index image broadcast, the sharded query's count all-gather
    and row gather -- so an RCCL-only constraint surfaces on the one-GPU box, not first on the
    driver's 8-GPU node."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd.device import DeviceIndex
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()).to(dev)
        part, _ = kd.owner_build(seq, k, dev, src=0)
        idx = kd.assemble_parts(part, dev)
        part.free()
        idx = kd.broadcast_index(idx, dev, src=0)
        info = idx.info()
        timings = {}
        rows = kd.sharded_query(kd.HipQueryEngine(idx), seq, kq, dst=0, src=0, timings=timings)
        torch.cuda.synchronize()
        # the receiving side of an image broadcast: import the exported image
        meta, bufs = idx.export_image()
        torch.cuda.synchronize()
        rep = DeviceIndex.import_image(meta.cpu(), bufs)
        rows2 = kd.sharded_query(kd.HipQueryEngine(rep), seq, kq, dst=0)
        torch.cuda.synchronize()
        out_q.put(((info["n_kmers"], info["n_positions"], info["n_pairs"]),
                   rows.cpu().numpy().reshape(-1).tolist(),
                   rows2.cpu().numpy().reshape(-1).tolist(), sorted(timings),
                   dist.get_backend(), str(rows.device)))
        rep.free()
        idx.free()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("k,kq", [(31, 31), (21, 17)])
def test_nccl_world1_owner_build_assemble_sharded_query(gpu, k, kq):
    import torch.multiprocessing as mp
    from kmer_hasher_amd import synth
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(150_000, 9, n_gap_every=10_007), 0.004, 8)
    s[-k - 2] = ord("N")
    seq_bytes = s.tobytes()
    oi = O.OracleIndex(seq_bytes, k)
    want = oi.query(seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), seq_bytes, k, kq, q))
    p.start()
    try:
        (nk, npos, npair), got, got2, phases, backend, where = q.get(timeout=100)
        p.join(60)
        assert p.exitcode == 0
    finally:
        if p.is_alive():
            p.kill()
    assert backend == "nccl" and where == "cuda:0"
    assert (nk, npos, npair) == (oi.U, oi.N, oi.P)
    assert got == want and got2 == want
    assert phases == ["broadcast", "gather", "query"]


def _scatter_worker(rank, world, port, seq_bytes, k, backend, out_q):
    """The R session's query on rank 0 only (config 5's step): C1 scatters each rank the slice
    its windows read (dist.scatter_sequence, into a reused buffer), every rank runs the HIP range
    query, and the rows are gathered into rank 0's device buffer, then delivered into the
    node-shared host matrix (dist.HostRowSink, hipHostRegister'ed)."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd.device import DeviceIndex
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    sink = kd.HostRowSink(0)
    try:
        seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()).to(dev) \
            if rank == 0 else None
        built = DeviceIndex.build(seq, k) if rank == 0 else None
        idx = kd.broadcast_index(built, dev, src=0)
        eng = kd.HipQueryEngine(idx)
        buf = torch.empty(len(seq_bytes) + 16, dtype=torch.uint8, device=dev) if rank else None
        res = []
        for to_host in (False, True, True):
            rows = kd.sharded_query(eng, seq, k, dst=0, src=0, c1="scatter",
                                    sink=sink if to_host else None, seq_buf=buf)
            torch.cuda.synchronize()
            if rank == 0:
                res.append((str(rows.device), rows.cpu().numpy().reshape(-1).tolist()))
        if rank == 0:
            out_q.put((res, sink.registered is not None))
        dist.barrier()
        idx.free()
    finally:
        sink.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,backend", [(2, 31, "gloo"), (3, 21, "gloo"), (1, 31, "nccl")])
def test_scatter_query_rows_to_device_and_host(gpu, world, k, backend):
    import torch.multiprocessing as mp
    from kmer_hasher_amd import synth
    from kmer_hasher_amd import dist as kd
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(130_000, 4, n_gap_every=8_009), 0.004, 5)
    n_w = len(s) - k + 1
    for a, _ in kd.shard_ranges(n_w, world)[1:]:
        s[a - 1] = ord("N")              # an N just before a shard's first window
    s[-k - 2] = ord("N")
    seq_bytes = s.tobytes()
    want = O.OracleIndex(seq_bytes, k).query(seq_bytes, k).tolist()
    before = set(os.listdir("/dev/shm"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, seq_bytes, k, backend, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res, registered = q.get(timeout=100)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert [r[0] for r in res] == ["cuda:0", "cpu", "cpu"]
    assert all(r[1] == want for r in res)
    assert registered                   # the host matrix is DMA-registered
    assert not [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("kmhg_rows")]


def _owner_query_worker(rank, world, port, seq_bytes, k, kq, backend, out_q, qbytes=None,
                        knobs=None):
    """Owner-computes build over `world` ranks sharing cuda:0 and the owner-routed query over the
    resident parts (no assembly): the query (`qbytes`, default the indexed sequence) broadcast
    from rank 0, every rank probing the windows its part owns (kmhg_query_run_device_part: the
    diagonal path where kq == k), rows and tile offsets to rank 0, merged there by
    kmhg_merge_part_rows.  `knobs`: path selectors for the test build (libkmhgpu_test.so)."""
    import contextlib
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import _lib
    from kmer_hasher_amd import dist as kd
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(knobs or {})
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with (_lib.using_test_build() if knobs else contextlib.nullcontext()):
            seq = torch.from_numpy(np.frombuffer(seq_bytes, np.uint8).copy()).to(dev) \
                if rank == 0 else None
            qry = seq if qbytes is None or rank != 0 else \
                torch.from_numpy(np.frombuffer(qbytes, np.uint8).copy()).to(dev)
            part, _ = kd.owner_build(seq, k, dev, src=0)
            kd.part_info_all(part, dev)
            eng = kd.HipPartEngine(part)
            res = []
            for _ in range(2):               # twice: the second reuses the pools and the tags
                ph = {}
                rows = kd.owner_query(eng, qry if rank == 0 else None, kq, dst=0, src=0,
                                      timings=ph)
                torch.cuda.synchronize()
                if rank == 0:
                    res.append(rows.cpu().numpy().reshape(-1).tolist())
            if rank == 0:
                out_q.put((res, sorted(ph)))
            dist.barrier()
            part.free()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,kq,backend,query", [
    (2, 31, 31, "gloo", "self"), (3, 21, 17, "gloo", "self"), (3, 31, 31, "gloo", "self"),
    (1, 21, 21, "nccl", "self"), (3, 31, 31, "gloo", "related"), (2, 21, 21, "gloo", "nodiag"),
    (3, 31, 31, "gloo", "buildtags")])
def test_owner_routed_query_over_parts(gpu, world, k, kq, backend, query):
    """Owner-routed rows equal the oracle's: self dot plots of a repeat-rich sequence (diagonal
    path at kq == k, table probes at kq != k), a related query (config 5's shape: SNVs,
    inversions / translocations and N-runs, so verifications fail and windows probe), the
    table-probe path forced at kq == k, and the parts' slot tags and repeated-key bits written by
    their builds (what parts beyond the cache do) instead of the first query."""
    knobs = {"nodiag": {"KMHG_QUERY_DIAG": "0"},
             "buildtags": {"KMHG_BUILD_TAGS": "1", "KMHG_BUILD_BID": "0"}}.get(query)
    import torch.multiprocessing as mp
    from kmer_hasher_amd import synth
    from oracle import oracle as O
    s = synth.add_n_runs(synth.repeat_rich(160_000, 12, n_gap_every=10_009), 0.004, 13)
    s[-k - 2] = ord("N")
    seq_bytes = s.tobytes()
    qbytes = synth.derived(s, 9, 0.01, 4).tobytes() if query in ("related", "buildtags") \
        else None
    want = O.OracleIndex(seq_bytes, k).query(qbytes or seq_bytes, kq).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_query_worker,
                         args=(r, world, port, seq_bytes, k, kq, backend, q, qbytes, knobs))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res, phases = q.get(timeout=100)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert len(want) > 0 and all(r == want for r in res)
    assert phases == ["broadcast", "gather", "merge", "query"]

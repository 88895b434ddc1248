"""Multi-GPU seq.kmer.pos: one process per GPU over torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X).

  * the index is built once (rank 0) and its device image is broadcast to every rank
    (two ncclBroadcast calls: the hash table and the positions);
  * the query's windows are split into `world` contiguous ranges; the query, held by one rank,
    is scattered (each rank receives the chars its range reads, at their absolute positions) or
    broadcast; each rank runs the HIP query on its range -- validity at a range edge is decided
    from the same chars as on the full sequence, so no halo logic leaks into the result;
  * per-rank row counts are all-gathered (8 B each) and the rows are gathered to the root with
    point-to-point send/recv (RCCL has no gatherv) -- as diagonal runs, 12 B per run of rows
    (i, j), (i + 1, j + 1), ..., expanded on the root -- or every rank copies its rows into one
    node-shared host matrix (HostRowSink); concatenation in rank order is exactly the
    reference's row order (window end ascending, then index position ascending).

The collective layer is engine-agnostic: anything with ``query_range(seq, k, w0, w1) -> (h, 2)
int32 tensor`` works, which is how tests exercise the sharding + gather logic with gloo on CPU.
The product engine is ``HipQueryEngine`` (libkmhgpu.so).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_ranges(n: int, world: int) -> list[tuple[int, int]]:
    """Balanced contiguous [w0, w1) ranges covering [0, n)."""
    q, r = divmod(max(n, 0), world)
    out, a = [], 0
    for i in range(world):
        b = a + q + (1 if i < r else 0)
        out.append((a, b))
        a = b
    return out


def broadcast_buffers(meta: torch.Tensor | None, bufs: list[torch.Tensor] | None, src: int,
                      device: torch.device, group=None) -> tuple[torch.Tensor, list[torch.Tensor]]:
    """Broadcast an int64 meta vector (after the 8-word header: one byte size per buffer) and the
    byte buffers it describes from `src`.  Non-src ranks pass None and receive fresh tensors."""
    rank = dist.get_rank(group)
    n_meta = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n_meta[0] = meta.numel()
    dist.broadcast(n_meta, src, group=group)
    m = meta.to(device) if rank == src else torch.empty(int(n_meta.item()), dtype=torch.int64,
                                                        device=device)
    dist.broadcast(m, src, group=group)
    sizes = [int(x) for x in m[8:].tolist()]
    if rank != src:
        bufs = [torch.empty(max(1, s), dtype=torch.uint8, device=device) for s in sizes]
    for b in bufs:
        dist.broadcast(b, src, group=group)
    return m, bufs


def gather_rows(local, dst: int = 0, group=None, codec=None) -> torch.Tensor | None:
    """Concatenate every rank's (h_r, 2) int32 rows on `dst` in rank order.

    codec: rows travel as diagonal runs where that is smaller ("Rows as diagonal
    runs"): codec.encode(rows) -> an (n, 3) int32 runs tensor or None (send the rows), and
    codec.decode(runs, h, out) on `dst` writes the h rows into `out`.  A dot plot's rows are
    long diagonals (config 5: 133 rows per 12-B run), so the link carries ~1/89 of the bytes.
    `local` may also come encoded already, as ('runs', (n, 3) runs, h) or ('rows', rows, h) (a
    sender's HipQueryEngine.query_range_runs, whose rows were never written)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if isinstance(local, tuple):
        kind, t, h_local = local
        runs = t if kind == "runs" else None
        local = t if kind == "rows" else None
        dev = t.device
    else:
        h_local = local.shape[0]
        dev = local.device
        runs = codec.encode(local) if codec is not None and rank != dst and h_local else None
    cnt = torch.tensor([h_local, -1 if runs is None else runs.shape[0]], dtype=torch.int64,
                       device=dev)
    metas = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(metas, cnt, group=group)
    counts = [int(m[0].item()) for m in metas]
    n_runs = [int(m[1].item()) for m in metas]
    if rank == dst:
        if world == 1 and local is not None:
            return local                     # the rows are already where they belong
        out = torch.empty((sum(counts), 2), dtype=torch.int32, device=dev)
        offs = [0]
        for c in counts:
            offs.append(offs[-1] + c)
        # the peers' rows (or runs) arrive (the backend's stream) while the root copies its own
        bufs = {r: torch.empty((n_runs[r], 3), dtype=torch.int32, device=dev)
                for r in range(world) if r != dst and counts[r] and n_runs[r] >= 0}
        works = p2p([("recv", bufs[r] if r in bufs else out[offs[r]:offs[r + 1]], r)
                     for r in range(world) if r != dst and counts[r]], group, wait=False)
        if local is not None:
            out[offs[rank]:offs[rank + 1]] = local
        elif counts[rank]:
            codec.decode(runs, counts[rank], out[offs[rank]:offs[rank + 1]])
        p2p_wait(works)
        for r, b in bufs.items():
            codec.decode(b, counts[r], out[offs[r]:offs[r + 1]])
        return out
    if counts[rank]:
        p2p([("send", local.contiguous() if runs is None else runs, dst)], group)
    return None


def p2p(ops: list, group=None, wait: bool = True):
    """One batch of point-to-point transfers, ("send" | "recv", tensor, group rank) each, waited
    for (wait=False: returned, for p2p_wait).  gloo moves device tensors in its collectives but
    not point to point: there (the one-GPU rehearsals) device tensors are staged through host
    copies."""
    if not ops:
        return ([], [])
    stage = dist.get_backend(group) == "gloo"
    batch, post = [], []
    for kind, t, peer in ops:
        if stage and t.is_cuda:
            h = t.cpu() if kind == "send" else torch.empty(t.shape, dtype=t.dtype)
            if kind == "recv":
                post.append((t, h))
            t = h
        batch.append(dist.P2POp(dist.isend if kind == "send" else dist.irecv, t,
                                _global(peer, group), group=group))
    works = (dist.batch_isend_irecv(batch), post)
    if wait:
        p2p_wait(works)
    return works


def p2p_wait(works) -> None:
    """Wait for a p2p(..., wait=False) batch (and land its host-staged receives)."""
    reqs, post = works
    for w in reqs:
        w.wait()
    for t, h in post:
        t.copy_(h)


def broadcast_sequence(seq: torch.Tensor | None, src: int, device: torch.device,
                       group=None, codec=None) -> torch.Tensor:
    """C1: the root's uint8 sequence on every rank (its length first, then one
    broadcast of the bytes; over RCCL the root fans out on its xGMI links).  codec: the bytes
    travel packed (codec.pack -> (code words, N-flag words), 6 B per 16 chars; HipSeqCodec) and
    are unpacked on arrival."""
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = seq.numel()
    dist.broadcast(n, src, group=group)
    L = int(n.item())
    if codec is None or L == 0 or dist.get_world_size(group) == 1:
        out = seq if rank == src else torch.empty(L, dtype=torch.uint8, device=device)
        if L:
            dist.broadcast(out, src, group=group)
        return out
    words = (L + 15) // 16
    if rank == src:
        code, nbit = codec.pack(seq)
    else:
        code = torch.empty(words, dtype=torch.int32, device=device)
        nbit = torch.empty(words, dtype=torch.int16, device=device)
    dist.broadcast(code, src, group=group)
    dist.broadcast(nbit.view(torch.uint8), src, group=group)   # (no int16 in gloo or RCCL)
    if rank == src:
        return seq
    out = torch.empty(L, dtype=torch.uint8, device=device)
    codec.unpack(code, nbit, 0, 0, L, out)
    return out


def slice_bounds(n_chars: int, k: int, w0: int, w1: int) -> tuple[int, int]:
    """The chars [a, b) a range query of windows [w0, w1) reads: the window rule needs chars
    [w0 - 1, w1 + k - 1) (src/kmer_pos.c:121-134: the N before a window, the end-drop test); the
    probe's aligned tile loads and halo read a few more around them, which feed only windows
    outside the range (the same bounds as the one-process multi-device split,
    kmhg_engine.cpp query_multi_device)."""
    if w1 <= w0:
        return 0, 0
    return max(0, (w0 & ~15) - 64), min(n_chars, w1 + k + 64)


def scatter_sequence(seq: torch.Tensor | None, k: int, src: int, device: torch.device,
                     group=None, out: torch.Tensor | None = None, codec=None) -> torch.Tensor:
    """C1 as a scatter: rank `src` holds the query; every other rank receives only the chars its
    window range reads (slice_bounds), in place in a full-length buffer, so the range query
    addresses the sequence by its absolute positions.  (N - 1)/N of L leaves the root, one slice
    per link, instead of the whole L on every link (broadcast_sequence).  `out`: a buffer of at
    least L + 16 bytes to reuse across calls.  Chars outside the slice are undefined (on CPU
    they read 'A': the gloo tests' oracle engine reads the whole buffer).  codec: the slices
    travel packed (the code and N-flag words covering them), unpacked into `out` on arrival."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        n[0] = seq.numel()
    dist.broadcast(n, src, group=group)
    L = int(n.item())
    ranges = shard_ranges(max(0, L - k + 1), world)
    if rank == src:
        ops = []
        packed = codec.pack(seq) if codec is not None and L and world > 1 else None
        for r in range(world):
            a, b = slice_bounds(L, k, *ranges[r])
            if r != src and b > a:
                if packed is None:
                    ops.append(("send", seq[a:b], r))
                else:
                    wa, wb = a // 16, (b + 15) // 16     # (u16 words as bytes: no int16 in RCCL)
                    ops += [("send", packed[0][wa:wb], r),
                            ("send", packed[1][wa:wb].view(torch.uint8), r)]
        p2p(ops, group)
        return seq
    if out is None or out.numel() < L + 16 or out.device != device:
        out = torch.empty(L + 16, dtype=torch.uint8, device=device)
        if device.type == "cpu":
            out.fill_(ord("A"))
    a, b = slice_bounds(L, k, *ranges[rank])
    if b > a:
        if codec is None:
            p2p([("recv", out[a:b], src)], group)
        else:
            wa, wb = a // 16, (b + 15) // 16
            code = torch.empty(wb - wa, dtype=torch.int32, device=device)
            nbit = torch.empty(wb - wa, dtype=torch.int16, device=device)
            p2p([("recv", code, src), ("recv", nbit.view(torch.uint8), src)], group)
            codec.unpack(code, nbit, wa, a, b, out)
    return out[:L]


def _global(r: int, group) -> int:
    """P2POp peers are global ranks."""
    return r if group is None else dist.get_global_rank(group, r)


class HostRowSink:
    """ONE host matrix shared by the ranks of a node (POSIX shared memory), into which every
    rank copies its own rows D2H at its row offset: each GPU uses its own PCIe link, and no row
    crosses xGMI ("Where the rows go").  The buffer is grown, never shrunk, and
    registered with the HIP runtime (hipHostRegister) so the copies are direct DMA; reuse one
    sink across queries.  close() on every rank releases it (the owner unlinks the segment)."""

    def __init__(self, owner: int = 0, group=None):
        self.owner, self.group = owner, group
        self.rank = dist.get_rank(group)
        self.cap = 0
        self.gen = 0
        self.shm = None
        self.t = None
        self.registered = None
        self.token = None

    def _name(self) -> str:
        return f"kmhg_rows_{self.token}_{self.gen}"

    def _release(self):
        if self.registered is not None:
            torch.cuda.cudart().cudaHostUnregister(self.registered)
            self.registered = None
        self.t = None
        if self.shm is not None:
            self.shm.close()
            if self.rank == self.owner:
                self.shm.unlink()
            self.shm = None

    def ensure(self, rows: int, device: torch.device):
        """A buffer of at least `rows` rows on every rank (collective: same `rows` everywhere)."""
        from multiprocessing import shared_memory
        if self.token is None:
            import os
            tok = torch.tensor([os.getpid() if self.rank == self.owner else 0], dtype=torch.int64,
                               device=device)
            dist.broadcast(tok, _global(self.owner, self.group), group=self.group)
            self.token = int(tok.item())
        if rows <= self.cap and self.t is not None:
            return
        nbytes = max(8, rows * 8)
        # room in /dev/shm (a tmpfs: writing past its size would SIGBUS every rank), decided by
        # the owner for every rank, before anything is created
        import os
        ok = torch.tensor([1], dtype=torch.int32, device=device)
        if self.rank == self.owner:
            try:
                st = os.statvfs("/dev/shm")
                free = st.f_bavail * st.f_frsize + (self.cap * 8 if self.t is not None else 0)
                ok[0] = 1 if free >= nbytes + (64 << 20) else 0
            except OSError:
                ok[0] = 0
        dist.broadcast(ok, _global(self.owner, self.group), group=self.group)
        if not int(ok.item()):
            raise RuntimeError(f"HostRowSink: /dev/shm has no room for {nbytes} bytes of rows")
        dist.barrier(group=self.group)             # nobody still writes the old buffer
        self._release()
        self.gen += 1
        if self.rank == self.owner:
            self.shm = shared_memory.SharedMemory(name=self._name(), create=True, size=nbytes)
        dist.barrier(group=self.group)
        if self.rank != self.owner:
            self.shm = shared_memory.SharedMemory(name=self._name())
            # only the owner unlinks: keep Python's resource tracker from unlinking the
            # segment again when this process exits (it registers every attachment)
            from multiprocessing import resource_tracker
            try:
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
        self.t = torch.frombuffer(self.shm.buf, dtype=torch.int32, count=nbytes // 4)
        if device.type == "cuda":
            ptr = self.t.data_ptr()
            if int(torch.cuda.cudart().cudaHostRegister(ptr, nbytes, 0)) == 0:
                self.registered = ptr
        self.cap = nbytes // 8

    def close(self):
        self._release()
        self.cap = 0


def deliver_rows_host(local: torch.Tensor, sink: HostRowSink, group=None, codec=None):
    """Every rank's (h_r, 2) int32 rows into the sink's shared host matrix, rank r's at row
    offset h_0 + ... + h_{r-1} (= the reference's row order), each rank copying its own rows
    D2H (codec.to_host when the codec has one: HipRunCodec sends them over PCIe as diagonal
    runs, expanded by host threads).  Returns the (H, 2) matrix (a view of the shared buffer)
    on the sink's owner, else None.  The matrix is valid until the next delivery into the same
    sink."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local.device
    cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    H = sum(counts)
    sink.ensure(H, dev)
    off = sum(counts[:rank])
    if counts[rank]:
        dst = sink.t[2 * off:2 * (off + counts[rank])].view(-1, 2)
        if codec is not None and hasattr(codec, "to_host") and local.is_cuda:
            codec.to_host(local, dst)
        else:
            dst.copy_(local)
    dist.barrier(group=group)                       # every rank's copy has landed
    if rank == sink.owner:
        return sink.t[:2 * H].view(-1, 2)
    return None


def sharded_query(engine, seq: torch.Tensor | None, k: int, dst: int = 0, group=None,
                  src: int | None = None, timings: dict | None = None, c1: str = "scatter",
                  sink: HostRowSink | None = None, seq_buf: torch.Tensor | None = None):
    """seq.kmer.pos with the query windows split across ranks; rows gathered on `dst`.

    src=None: every rank already holds the whole query.  src=r: only rank r holds it (the R
    session's query string arrives on one process): c1="scatter" sends each rank the slice its
    windows read (scatter_sequence), c1="broadcast" the whole sequence (broadcast_sequence).
    sink=None: rows gathered into one device buffer on `dst` (gather_rows, over xGMI; as
    diagonal runs when the engine has a `codec`); a HostRowSink: every rank copies its rows into
    the shared host matrix (deliver_rows_host).
    `seq_buf`: scatter receive buffer to reuse.  `timings` (optional) receives the seconds of
    each phase as seen by this rank: 'broadcast' (C1), 'query' (the HIP range query) and
    'gather'."""
    import time
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = seq.device if seq is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
        else torch.device("cpu"))

    def mark():
        if timings is not None and dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return time.perf_counter()

    t0 = mark()
    sc = getattr(engine, "seq_codec", None)
    if src is not None:
        if c1 == "scatter":
            seq = scatter_sequence(seq, k, src, dev, group, out=seq_buf, codec=sc)
        else:
            seq = broadcast_sequence(seq, src, dev, group, sc)
    t1 = mark()
    n_windows = max(0, seq.numel() - k + 1)
    w0, w1 = shard_ranges(n_windows, world)[rank]
    codec = getattr(engine, "codec", None)
    if sink is None and rank != dst and codec is not None and hasattr(engine, "query_range_runs"):
        local = engine.query_range_runs(seq, k, w0, w1)    # a sender: its runs, no rows
    else:
        local = engine.query_range(seq, k, w0, w1)
    t2 = mark()
    rows = gather_rows(local, dst, group, codec) if sink is None \
        else deliver_rows_host(local, sink, group, codec)
    t3 = mark()
    if timings is not None:
        for name, dt in (("broadcast", t1 - t0), ("query", t2 - t1), ("gather", t3 - t2)):
            timings[name] = timings.get(name, 0.0) + dt
    return rows


# ------------------------------------------------------------------ owner-computes build (§8e)
IMAGE_MAGIC = 0x6B6D6867          # 'kmhg', kmhg_image_import's header word 7


def part_layout(infos: list[dict]) -> dict:
    """Where each rank's part lands in the whole index: its first slot (bucket b0 x capb), its
    first position index (the positions of the parts before it), and the totals."""
    capb, nbt = infos[0]["capb"], infos[0]["nb_total"]
    bases, acc = [], 0
    for inf in infos:
        bases.append(acc)
        acc += inf["n_positions"]
    owners = [r for r, inf in enumerate(infos) if inf["side_owner"]]
    return {"capb": capb, "nb_total": nbt, "slots": nbt * capb + 1, "pos_base": bases,
            "N": acc, "U": sum(i["n_kmers"] for i in infos),
            "P": sum(i["n_pairs"] for i in infos),
            "max_n": max(i["max_count"] for i in infos), "side_owner": owners[0] if owners else 0,
            "codes_bytes": max(i["codes_bytes"] for i in infos)}


def owner_build(seq: torch.Tensor | None, k: int, device: torch.device, src: int | None = 0,
                group=None, stream=None, codec="auto"):
    """make.kmer.hash over G ranks, owner-computes (the reference's reader pool
    gives each thread the k-mers it owns, src/kmer_reader.c:28-39): the sequence is broadcast
    from `src` (C1; src=None: every rank holds it already; packed by HipSeqCodec on a GPU),
    every rank walks all windows and builds only the k-mers of its bucket range
    (kmhg_build_device_part).  Returns this rank's DevicePart and the sequence it built from;
    assemble_parts() makes the whole index on every rank."""
    from .device import DeviceIndex
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if codec == "auto":
        codec = HipSeqCodec() if device.type == "cuda" else None
    if src is not None:
        seq = broadcast_sequence(seq, src, device, group, codec)
    return DeviceIndex.build_part(seq, k, rank, world, stream), seq


def part_info_all(part, device: torch.device, group=None) -> dict:
    """part.part_info() (which waits for the part build) on every rank, or an error on EVERY
    rank: a part whose bucket overflowed raises on its own rank only, and the other ranks would
    otherwise block forever in the next collective.  The status goes round first (all-reduce
    MIN), so all ranks raise together."""
    err = None
    try:
        mine = part.part_info()
    except Exception as e:                  # KmhgError (overflow) or a device error
        err, mine = e, None
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if err is not None:
        raise err
    if not int(ok.item()):
        raise RuntimeError("owner-computes build: another rank's part build failed")
    return mine


def assemble_parts(part, device: torch.device, group=None, import_fn=None):
    """All ranks' parts -> the whole index on every rank (all-gather of the rebased slot ranges
    and of the positions, the side slot and code block from their owners), imported with
    kmhg_image_import.  Bit-identical to the single-device build of the same sequence."""
    from .device import PART_FIELDS, SLOT_BYTES, DeviceIndex
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    mine = part_info_all(part, device, group)
    t = torch.tensor([mine[f] for f in PART_FIELDS], dtype=torch.int64, device=device)
    got = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(got, t, group=group)
    infos = [dict(zip(PART_FIELDS, g.tolist())) for g in got]
    lay = part_layout(infos)
    capb = lay["capb"]
    slot_b = [inf["nb"] * capb * SLOT_BYTES for inf in infos]
    pos_b = [inf["n_positions"] * 4 for inf in infos]
    ms, mp = max(1, max(slot_b)), max(1, max(pos_b))
    # padded all-gathers: every rank contributes max-sized buffers (one collective each)
    send_t = torch.empty(ms, dtype=torch.uint8, device=device)
    send_p = torch.empty(mp, dtype=torch.uint8, device=device)
    side = torch.zeros(SLOT_BYTES, dtype=torch.uint8, device=device)
    codes = torch.empty(max(1, lay["codes_bytes"]), dtype=torch.uint8, device=device)
    code_src = next((r for r, inf in enumerate(infos) if inf["nb"] and inf["codes_bytes"]), 0)
    part.export_into(lay["pos_base"][rank], send_t[:slot_b[rank]], side, send_p[:pos_b[rank]],
                     codes if rank == code_src else None)
    recv_t = torch.empty((world, ms), dtype=torch.uint8, device=device)
    recv_p = torch.empty((world, mp), dtype=torch.uint8, device=device)
    dist.all_gather(list(recv_t.unbind(0)), send_t, group=group)
    dist.all_gather(list(recv_p.unbind(0)), send_p, group=group)
    dist.broadcast(side, lay["side_owner"], group=group)
    dist.broadcast(codes, code_src, group=group)
    table = torch.empty(lay["slots"] * SLOT_BYTES, dtype=torch.uint8, device=device)
    positions = torch.empty(max(1, lay["N"] * 4), dtype=torch.uint8, device=device)
    for r, inf in enumerate(infos):
        a = inf["b0"] * capb * SLOT_BYTES
        table[a:a + slot_b[r]] = recv_t[r, :slot_b[r]]
        b = lay["pos_base"][r] * 4
        positions[b:b + pos_b[r]] = recv_p[r, :pos_b[r]]
    table[-SLOT_BYTES:] = side
    del recv_t, recv_p, send_t, send_p
    header = [int(part.k), part.L, (lay["nb_total"] << 32) | capb, lay["U"], lay["N"], lay["P"],
              lay["max_n"], IMAGE_MAGIC]
    sizes = [table.numel(), lay["N"] * 4, lay["codes_bytes"]]
    meta = torch.tensor(header + sizes, dtype=torch.int64)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    return (import_fn or DeviceIndex.import_image)(meta, [table, positions, codes])


class HipSeqCodec:
    """C1's sequence codec on the GPU: kmhg_seq_pack / kmhg_seq_unpack (2-bit codes + N flags,
    6 B per 16 chars on the wire)."""

    @staticmethod
    def pack(seq: torch.Tensor):
        from .device import seq_pack
        return seq_pack(seq)

    @staticmethod
    def unpack(code: torch.Tensor, nbit: torch.Tensor, word0: int, a: int, b: int,
               out: torch.Tensor):
        from .device import seq_unpack
        seq_unpack(code, nbit, word0, a, b, out)


class HipRunCodec:
    """gather_rows' run codec on the GPU: kmhg_rows_runs / kmhg_runs_expand."""

    @staticmethod
    def encode(rows: torch.Tensor):
        from .device import rows_to_runs
        return rows_to_runs(rows)

    @staticmethod
    def decode(runs: torch.Tensor, n_rows: int, out: torch.Tensor):
        from .device import runs_expand
        runs_expand(runs, n_rows, out)

    @staticmethod
    def to_host(rows: torch.Tensor, out: torch.Tensor):
        from .device import rows_to_host
        rows_to_host(rows, out)


class HipQueryEngine:
    """Adapter: a DeviceIndex (libkmhgpu) as a sharded-query engine; its rows travel to the
    root as diagonal runs (HipRunCodec)."""

    codec = HipRunCodec()
    seq_codec = HipSeqCodec()

    def __init__(self, index):
        self.index = index

    def query_range(self, seq: torch.Tensor, k: int, w0: int, w1: int) -> torch.Tensor:
        # the rows stay where the emit kernel wrote them (a 3 GB device copy per query at
        # config 5 otherwise); the tensor owns the query
        return self.index.query_range(seq, k, w0, w1).rows_view()

    def query_range_runs(self, seq: torch.Tensor, k: int, w0: int, w1: int):
        """A sender's range of the gather: ('runs', runs, H) made from the query's window
        records without writing its rows, or ('rows', rows, H)."""
        return self.index.query_range_runs(seq, k, w0, w1)


def broadcast_index(index, device: torch.device, src: int = 0, group=None):
    """Replicate rank `src`'s DeviceIndex on every rank (index image over RCCL)."""
    from .device import DeviceIndex
    rank = dist.get_rank(group)
    if rank == src:
        meta, bufs = index.export_image()
        torch.cuda.synchronize(device)
        broadcast_buffers(meta, bufs, src, device, group)
        return index
    meta, bufs = broadcast_buffers(None, None, src, device, group)
    torch.cuda.synchronize(device)
    return DeviceIndex.import_image(meta.cpu(), bufs)


# ------------------------------------------------------- owner-routed query over resident parts
class HipPartEngine:
    """Adapter: this rank's DevicePart (libkmhgpu) as an owner-routed query engine."""

    seq_codec = HipSeqCodec()

    def __init__(self, part):
        self.part = part

    def query_part(self, seq: torch.Tensor, k: int):
        """(rows of the windows this part owns, in window order; their n_tiles + 1 per-tile row
        offsets) -- kmhg_query_run_device_part."""
        q = self.part.query_part(seq, k)
        return q.rows_view(), q.tile_offsets()

    def merge(self, rows: torch.Tensor, seg_base: list[int], tile_off: torch.Tensor, k: int):
        from .device import merge_part_rows
        return merge_part_rows(rows, seg_base, tile_off, k)


def owner_query(engine, seq: torch.Tensor | None, k: int, dst: int = 0, src: int | None = 0,
                group=None, timings: dict | None = None):
    """seq.kmer.pos against an index that stays split in its owner-computes parts, one per rank
    (the reference's reader-pool partition src/kmer_reader.c:28-39): no assembly
    and no index broadcast.  The query is broadcast (C1: every rank walks every window), each
    rank probes only the windows whose k-mer it owns and emits their rows in window order with
    its per-tile row offsets; the rows and offsets go to `dst`, whose merge
    (kmhg_merge_part_rows) interleaves them by window into exactly the unsharded rows (a
    window's rows all come from its key's owner).  Returns the (H, 2) rows on `dst`, None
    elsewhere.  `timings` receives 'broadcast', 'query', 'gather' and 'merge' seconds."""
    import time
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = seq.device if seq is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
        else torch.device("cpu"))

    def mark():
        if timings is not None and dev.type == "cuda":
            torch.cuda.synchronize(dev)
        return time.perf_counter()

    t0 = mark()
    if src is not None:
        seq = broadcast_sequence(seq, src, dev, group, getattr(engine, "seq_codec", None))
    t1 = mark()
    local, toff = engine.query_part(seq, k)
    t2 = mark()
    toff = toff.to(torch.int64)
    offs = [torch.empty_like(toff) for _ in range(world)]
    dist.all_gather(offs, toff, group=group)
    rows = gather_rows(local, dst, group)
    t3 = mark()
    out = None
    if rank == dst:
        if world == 1:
            out = rows                        # one part owns every window: already in order
        else:
            totals = [int(o[-1].item()) for o in offs]
            seg_base = [sum(totals[:r]) for r in range(world)]
            out = engine.merge(rows, seg_base, torch.stack(offs), k)
    t4 = mark()
    if timings is not None:
        for name, dt in (("broadcast", t1 - t0), ("query", t2 - t1), ("gather", t3 - t2),
                         ("merge", t4 - t3)):
            timings[name] = timings.get(name, 0.0) + dt
    return out

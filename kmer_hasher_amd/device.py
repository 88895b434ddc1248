"""Device-resident entry points (inputs already in HBM as torch uint8 tensors).

These drive the same C-ABI as ``api`` (kmhg_*_device variants) on the caller's current torch
stream, so bench.py can time the hot path with inputs resident in HBM and the multi-GPU layer
(``dist``) can move index images and hit rows with RCCL.  torch is plumbing here (device memory,
streams, torch.distributed); every result is computed by the HIP kernels in libkmhgpu.so.
"""
from __future__ import annotations

import ctypes as C
import json

import torch

from . import _lib


def _stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _check_seq(t: torch.Tensor):
    if not (t.is_cuda and t.dtype == torch.uint8 and t.dim() == 1 and t.is_contiguous()):
        raise TypeError("sequence must be a contiguous 1-D torch.uint8 CUDA tensor")


class DeviceIndex:
    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @classmethod
    def build(cls, seq: torch.Tensor, k: int, stream=None) -> "DeviceIndex":
        _check_seq(seq)
        with torch.cuda.device(seq.device):
            out = C.c_void_p()
            _lib.check(_lib.lib().kmhg_build_device(C.c_void_p(seq.data_ptr()), seq.numel(), k, 0,
                                                    _stream_ptr(stream), C.byref(out)))
        return cls(out.value)

    @classmethod
    def build_part(cls, seq: torch.Tensor, k: int, part: int, n_parts: int,
                   stream=None) -> "DevicePart":
        """Part `part` of `n_parts` of an owner-computes build (kmhg_build_device_part): the
        k-mers whose hash bucket lies in this part's range of the whole table, from every
        window of `seq`."""
        _check_seq(seq)
        with torch.cuda.device(seq.device):
            out = C.c_void_p()
            _lib.check(_lib.lib().kmhg_build_device_part(C.c_void_p(seq.data_ptr()), seq.numel(),
                                                         k, part, n_parts, _stream_ptr(stream),
                                                         C.byref(out)))
        p = DevicePart(out.value)
        p.k, p.L, p.device = k, seq.numel(), seq.device
        return p

    @classmethod
    def count(cls, seq: torch.Tensor, k: int, source: int, source_n: int,
              into: "DeviceIndex | None" = None, stream=None) -> "DeviceIndex":
        """count.kmers of one HBM-resident sequence (kmhg_count_device): adds to `into`, or
        makes a new counts index.  Synchronous (the merge reads the number of new k-mers)."""
        _check_seq(seq)
        h = C.c_void_p(into._h.value if into is not None else None)
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_count_device(C.byref(h), C.c_void_p(seq.data_ptr()),
                                                    seq.numel(), k, source, source_n,
                                                    _stream_ptr(stream)))
        return into if into is not None else cls(h.value)

    @classmethod
    def count_reads(cls, reads: "DeviceReads", params, into: "DeviceIndex | None" = None,
                    stream=None) -> "DeviceIndex":
        """count.kmers.fq.sh.rp over HBM-resident packed reads (kmhg_sh_count_reads_device):
        params = (k, prefix_bits, min_q, thread_n, max_reads, max_mem, source_n, source)."""
        h = C.c_void_p(into._h.value if into is not None else None)
        prm = (C.c_int32 * 8)(*[int(x) for x in params])
        with torch.cuda.device(reads.seq.device):
            _lib.check(_lib.lib().kmhg_sh_count_reads_device(
                C.byref(h), C.c_void_p(reads.seq.data_ptr()), C.c_void_p(reads.qual.data_ptr()),
                C.c_void_p(reads.off.data_ptr()), C.c_void_p(reads.hasq.data_ptr()), reads.n,
                prm, _stream_ptr(stream)))
        return into if into is not None else cls(h.value)

    def depth(self, seq: torch.Tensor, k: int, out: torch.Tensor | None = None,
              stream=None) -> torch.Tensor:
        """seq.kmer.depth.sh of an HBM-resident sequence: (L, counts_n) int32 (INT_MIN = NA)."""
        _check_seq(seq)
        S = self.info()["sources"]
        if out is None:
            out = torch.empty((seq.numel(), S), dtype=torch.int32, device=seq.device)
        if out.dtype != torch.int32 or not out.is_contiguous() or out.numel() < seq.numel() * S:
            raise ValueError(f"out must be a contiguous int32 tensor of >= {seq.numel() * S} "
                             "elements (L x counts_n)")
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_sh_depth_device(self._h, C.c_void_p(seq.data_ptr()),
                                                       seq.numel(), k, C.c_void_p(out.data_ptr()),
                                                       _stream_ptr(stream)))
        return out

    @property
    def handle(self):
        return self._h

    def wait(self) -> "DeviceIndex":
        """Block until the (asynchronous) build has finished; info/queries/readout also wait."""
        _lib.check(_lib.lib().kmhg_index_wait(self._h))
        return self

    def info(self) -> dict:
        inf = _lib.Info()
        _lib.check(_lib.lib().kmhg_index_info(self._h, C.byref(inf)))
        return {f: getattr(inf, f) for f, _ in _lib.Info._fields_}

    def query(self, seq: torch.Tensor, k: int, stream=None) -> "DeviceQuery":
        _check_seq(seq)
        q = C.c_void_p()
        h = C.c_int64()
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_query_run_device(self._h, C.c_void_p(seq.data_ptr()),
                                                        seq.numel(), k, _stream_ptr(stream),
                                                        C.byref(q), C.byref(h)))
        return DeviceQuery(q.value, h.value, seq.device)

    def query_range(self, seq: torch.Tensor, k: int, w0: int, w1: int, stream=None) -> "DeviceQuery":
        """Windows [w0, w1) of `seq` (the multi-GPU shard unit, see dist.py)."""
        _check_seq(seq)
        q = C.c_void_p()
        h = C.c_int64()
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_query_run_device_range(
                self._h, C.c_void_p(seq.data_ptr()), seq.numel(), k, w0, w1, _stream_ptr(stream),
                C.byref(q), C.byref(h)))
        return DeviceQuery(q.value, h.value, seq.device)

    def query_range_runs(self, seq: torch.Tensor, k: int, w0: int, w1: int, stream=None):
        """Windows [w0, w1) with the rows left as diagonal runs
        (kmhg_query_run_device_range_runs): ('runs', (n_runs, 3) int32 tensor, H), or
        ('rows', (H, 2) int32 tensor, H) where runs would not be smaller.  Either tensor owns
        the query."""
        _check_seq(seq)
        q = C.c_void_p()
        h, nr = C.c_int64(), C.c_int64()
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_query_run_device_range_runs(
                self._h, C.c_void_p(seq.data_ptr()), seq.numel(), k, w0, w1, _stream_ptr(stream),
                C.byref(q), C.byref(h), C.byref(nr)))
        dq = DeviceQuery(q.value, h.value, seq.device)
        if nr.value < 0:
            return "rows", dq.rows_view(), h.value
        return "runs", dq.runs_view(nr.value), h.value

    def positions(self, opt: int, stream=None) -> dict:
        """kmer.pos into device tensors: {'kmer': uint8 (U, k+1), 'pos': int32 (N, 2),
        'pair.pos': int32 (P, 3), 'count': int32 (U,)} for the requested bits."""
        L = _lib.lib()
        nk, npos, npair, ncnt = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check(L.kmhg_positions_size(self._h, opt, C.byref(nk), C.byref(npos),
                                         C.byref(npair), C.byref(ncnt)))
        inf = self.info()
        dev = torch.device("cuda", inf["device"])
        out = {"kmer": None, "pos": None, "pair.pos": None, "count": None}
        if opt & 1:
            out["kmer"] = torch.empty((nk.value, inf["k"] + 1), dtype=torch.uint8, device=dev)
        if opt & 2:
            out["pos"] = torch.empty((npos.value, 2), dtype=torch.int32, device=dev)
        if opt & 4:
            out["pair.pos"] = torch.empty((npair.value, 3), dtype=torch.int32, device=dev)
        if opt & 8:
            out["count"] = torch.empty((ncnt.value,), dtype=torch.int32, device=dev)

        def p(t):
            return C.c_void_p(t.data_ptr()) if t is not None and t.numel() else None

        with torch.cuda.device(dev):
            _lib.check(L.kmhg_positions_fill_device(self._h, opt, p(out["kmer"]), p(out["pos"]),
                                                    p(out["pair.pos"]), p(out["count"]),
                                                    _stream_ptr(stream)))
        return out

    # ---- index image (multi-GPU replication) ---------------------------------------------
    def export_image(self, stream=None) -> tuple[torch.Tensor, list[torch.Tensor]]:
        sz = _lib.ImageSizes()
        hdr = (C.c_int64 * 8)()
        _lib.check(_lib.lib().kmhg_image_sizes_get(self._h, C.byref(sz), hdr))
        dev = torch.device("cuda", self.info()["device"])
        bufs = [torch.empty(max(1, getattr(sz, f)), dtype=torch.uint8, device=dev)
                for f, _ in _lib.ImageSizes._fields_]
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().kmhg_image_export(self._h,
                                                    *[C.c_void_p(b.data_ptr()) for b in bufs],
                                                    _stream_ptr(stream)))
        header = torch.tensor(list(hdr), dtype=torch.int64)
        sizes = torch.tensor([getattr(sz, f) for f, _ in _lib.ImageSizes._fields_],
                             dtype=torch.int64)
        return torch.cat([header, sizes]), bufs

    @classmethod
    def import_image(cls, meta: torch.Tensor, bufs: list[torch.Tensor], stream=None):
        hdr = (C.c_int64 * 8)(*[int(x) for x in meta[:8].tolist()])
        sizes = [int(x) for x in meta[8:].tolist()]
        out = C.c_void_p()
        # a buffer of size 0 (no positions, no code block) is passed as NULL
        ptrs = [C.c_void_p(b.data_ptr() if i >= len(sizes) or sizes[i] else None)
                for i, b in enumerate(bufs)]
        with torch.cuda.device(bufs[0].device):
            _lib.check(_lib.lib().kmhg_image_import(hdr, *ptrs, _stream_ptr(stream), C.byref(out)))
        return cls(out.value)

    def free(self):
        if self._h:
            _lib.lib().kmhg_free(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


PART_FIELDS = ("b0", "nb", "nb_total", "capb", "n_positions", "n_kmers", "n_pairs", "max_count",
               "side_owner", "codes_bytes")
SLOT_BYTES = 16


class DevicePart(DeviceIndex):
    """One part of an owner-computes build (DeviceIndex.build_part); dist.assemble_parts turns
    the parts of all ranks into the whole index."""

    def part_info(self) -> dict:
        a = (C.c_int64 * 10)()
        _lib.check(_lib.lib().kmhg_part_info(self._h, a))
        return dict(zip(PART_FIELDS, list(a)))

    def export_into(self, pos_base: int, table: torch.Tensor | None, side: torch.Tensor | None,
                    positions: torch.Tensor | None, codes: torch.Tensor | None, stream=None):
        """Write this part's rebased slots / side slot / positions / code block into the given
        uint8 device views (None = skip)."""
        def p(t):
            return C.c_void_p(t.data_ptr()) if t is not None and t.numel() else None
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().kmhg_part_export(self._h, pos_base, p(table), p(side),
                                                   p(positions), p(codes), _stream_ptr(stream)))


    def query_part(self, seq: torch.Tensor, k: int, stream=None) -> "DeviceQuery":
        """seq.kmer.pos of every window of `seq` against this part only
        (kmhg_query_run_device_part): the rows of the windows whose k-mer the part owns, in
        window order; merge_part_rows interleaves every part's rows."""
        _check_seq(seq)
        q = C.c_void_p()
        h = C.c_int64()
        with torch.cuda.device(seq.device):
            _lib.check(_lib.lib().kmhg_query_run_device_part(
                self._h, C.c_void_p(seq.data_ptr()), seq.numel(), k, _stream_ptr(stream),
                C.byref(q), C.byref(h)))
        return DeviceQuery(q.value, h.value, seq.device)


def merge_part_rows(rows: torch.Tensor, seg_base: list[int], tile_off: torch.Tensor, k: int,
                    w0: int = 0, stream=None) -> torch.Tensor:
    """kmhg_merge_part_rows: `rows` (H, 2) int32 holds every part's rows (part r's from row
    seg_base[r]), `tile_off` (n_parts, n_tiles + 1) uint64 their per-tile offsets; returns the
    (H, 2) rows in the unsharded seq.kmer.pos order."""
    dev = rows.device
    n_parts, nt1 = tile_off.shape
    out = torch.empty_like(rows)
    base = torch.tensor(seg_base, dtype=torch.int64, device=dev)
    toff = tile_off.to(device=dev, dtype=torch.int64).contiguous()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().kmhg_merge_part_rows(
            C.c_void_p(rows.data_ptr()), C.c_void_p(base.data_ptr()),
            C.c_void_p(toff.data_ptr()), n_parts, nt1 - 1, k, w0, C.c_void_p(out.data_ptr()),
            _stream_ptr(stream)))
    return out


def seq_pack(seq: torch.Tensor, stream=None) -> tuple[torch.Tensor, torch.Tensor]:
    """kmhg_seq_pack: a uint8 device sequence as (code u32 words, N-flag u16 words), 16 chars
    each -- what crosses xGMI in place of the chars (6 B per 16)."""
    _check_seq(seq)
    words = (seq.numel() + 15) // 16
    code = torch.empty(max(1, words), dtype=torch.int32, device=seq.device)
    nbit = torch.empty(max(1, words), dtype=torch.int16, device=seq.device)
    with torch.cuda.device(seq.device):
        _lib.check(_lib.lib().kmhg_seq_pack(
            C.c_void_p(seq.data_ptr()), seq.numel(), C.c_void_p(code.data_ptr()),
            C.c_void_p(nbit.data_ptr()), _stream_ptr(stream)))
    return code[:words], nbit[:words]


def seq_unpack(code: torch.Tensor, nbit: torch.Tensor, word0: int, a: int, b: int,
               out: torch.Tensor, stream=None) -> torch.Tensor:
    """kmhg_seq_unpack: chars [a, b) of `out` (uint8, device) from words held from word0 on."""
    if b <= a:
        return out
    if out.numel() < b or out.dtype != torch.uint8 or not out.is_cuda:
        raise ValueError("out must be a uint8 CUDA tensor of at least b chars")
    if code.numel() < (b + 15) // 16 - word0 or nbit.numel() < (b + 15) // 16 - word0:
        raise ValueError("the packed words do not cover [a, b)")
    with torch.cuda.device(out.device):
        _lib.check(_lib.lib().kmhg_seq_unpack(
            C.c_void_p(code.data_ptr()), C.c_void_p(nbit.data_ptr()), word0, a, b,
            C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return out


def rows_to_host(rows: torch.Tensor, out: torch.Tensor, stream=None) -> torch.Tensor:
    """kmhg_rows_to_host: (H, 2) int32 device rows into `out`, a contiguous host (H, 2) int32
    tensor (pinned or not), as kmhg_query_fill delivers a query: diagonal runs over PCIe,
    expanded by host threads.  Synchronous."""
    H = rows.shape[0]
    if out.shape != (H, 2) or out.dtype != torch.int32 or out.is_cuda or not out.is_contiguous():
        raise ValueError("out must be a contiguous host (H, 2) int32 tensor")
    if H == 0:
        return out
    rows = rows.contiguous()
    with torch.cuda.device(rows.device):
        _lib.check(_lib.lib().kmhg_rows_to_host(C.c_void_p(rows.data_ptr()), H,
                                                C.c_void_p(out.data_ptr()), _stream_ptr(stream)))
    return out


def rows_to_runs(rows: torch.Tensor, stream=None) -> torch.Tensor | None:
    """kmhg_rows_runs: the (H, 2) int32 rows as diagonal runs, an (n_runs, 3) int32 tensor of
    {first row index, i, j} -- or None when runs would not be smaller than the rows (12 B per
    run against 8 B per row)."""
    H = rows.shape[0]
    if H == 0:
        return None
    dev = rows.device
    rows = rows.contiguous()
    n = C.c_int64()
    cap = max(1, H // 16)                    # a dot plot's runs: tens of rows each
    with torch.cuda.device(dev):
        for _ in range(2):
            runs = torch.empty((cap, 3), dtype=torch.int32, device=dev)
            _lib.check(_lib.lib().kmhg_rows_runs(
                C.c_void_p(rows.data_ptr()), H, C.c_void_p(runs.data_ptr()), cap, C.byref(n),
                _stream_ptr(stream)))
            if 3 * n.value >= 2 * H:
                return None
            if n.value <= cap:
                return runs[:n.value]
            cap = n.value
    raise RuntimeError("kmhg_rows_runs: run count changed between calls")


def runs_expand(runs: torch.Tensor, n_rows: int, out: torch.Tensor, stream=None) -> torch.Tensor:
    """kmhg_runs_expand: (n_runs, 3) int32 runs back to their n_rows (i, j) rows in `out` (a
    contiguous (n_rows, 2) int32 device tensor)."""
    if n_rows == 0:
        return out
    if out.shape != (n_rows, 2) or out.dtype != torch.int32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous (n_rows, 2) int32 tensor")
    runs = runs.to(device=out.device, dtype=torch.int32).contiguous()
    with torch.cuda.device(out.device):
        _lib.check(_lib.lib().kmhg_runs_expand(
            C.c_void_p(runs.data_ptr()), runs.shape[0], n_rows, C.c_void_p(out.data_ptr()),
            _stream_ptr(stream)))
    return out


class DeviceQuery:
    def __init__(self, handle: int, n_rows: int, device: torch.device | None = None):
        self._h = C.c_void_p(handle)
        self.n_rows = n_rows
        # the device the query ran on (the query sequence's): rows_view of an empty result lands
        # there too, like a non-empty one
        self.device = device if device is not None else \
            torch.device("cuda", torch.cuda.current_device())

    def copy_to(self, dst: torch.Tensor, stream=None) -> torch.Tensor:
        """Copy the (H, 2) int32 rows into `dst` (device, >= 2*H int32)."""
        if dst.numel() < 2 * self.n_rows or dst.dtype != torch.int32 or not dst.is_cuda:
            raise ValueError("destination too small or not an int32 CUDA tensor")
        with torch.cuda.device(dst.device):
            _lib.check(_lib.lib().kmhg_query_copy_device(self._h, C.c_void_p(dst.data_ptr()),
                                                         _stream_ptr(stream)))
        return dst

    def rows(self, device=None) -> torch.Tensor:
        dev = device or torch.device("cuda", torch.cuda.current_device())
        t = torch.empty((self.n_rows, 2), dtype=torch.int32, device=dev)
        if self.n_rows:
            self.copy_to(t)
        return t

    def tile_offsets(self, stream=None) -> torch.Tensor:
        """A part query's n_tiles + 1 per-tile row offsets (uint64 as int64, on its device)."""
        n = C.c_int64()
        _lib.check(_lib.lib().kmhg_query_tile_offsets(self._h, None, C.byref(n), None))
        out = torch.empty(n.value + 1, dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().kmhg_query_tile_offsets(self._h, C.c_void_p(out.data_ptr()),
                                                          C.byref(n), _stream_ptr(stream)))
        return out

    def rows_view(self) -> torch.Tensor:
        """The (H, 2) int32 rows where the emit kernel wrote them (kmhg_query_rows_device), as a
        tensor that owns this query: no copy, and the rows' buffer goes back to the library's pool
        (stream-ordered on the query's stream) when the last tensor using it is gone.  Used on
        the query's stream, as every result of the library is."""
        if not self.n_rows:
            return torch.empty((0, 2), dtype=torch.int32, device=self.device)
        d = C.c_void_p()
        _lib.check(_lib.lib().kmhg_query_rows_device(self._h, C.byref(d)))
        return torch.as_tensor(_RowsBuffer(self, d.value))   # on the rows' own device

    def runs_view(self, n_runs: int) -> torch.Tensor:
        """The (n_runs, 3) int32 runs of a runs query (kmhg_query_runs_device), as a tensor that
        owns this query (rows_view's contract)."""
        if not n_runs:
            return torch.empty((0, 3), dtype=torch.int32, device=self.device)
        d = C.c_void_p()
        _lib.check(_lib.lib().kmhg_query_runs_device(self._h, C.byref(d)))
        return torch.as_tensor(_RowsBuffer(self, d.value, (n_runs, 3)))

    def free(self):
        if self._h:
            _lib.lib().kmhg_query_free(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class _RowsBuffer:
    """__cuda_array_interface__ of a query's device rows; torch keeps this object (and so the
    query) alive for as long as the tensor made from it."""

    def __init__(self, q: DeviceQuery, ptr: int, shape: tuple | None = None):
        self.q = q
        self.__cuda_array_interface__ = {"shape": shape or (q.n_rows, 2), "typestr": "<i4",
                                         "data": (ptr, False), "version": 3, "strides": None,
                                         "stream": None}


def timing_enable(on: bool = True):
    _lib.check(_lib.lib().kmhg_timing_enable(1 if on else 0))


def timing_select(kernel: str | None):
    """Record events only around `kernel` (None = every kernel)."""
    _lib.check(_lib.lib().kmhg_timing_select(kernel.encode() if kernel else None))


def timing_reset():
    _lib.check(_lib.lib().kmhg_timing_reset())


def timing_report() -> dict:
    buf = C.create_string_buffer(1 << 16)
    _lib.check(_lib.lib().kmhg_timing_report(buf, len(buf)))
    return json.loads(buf.value.decode())


class DeviceReads:
    """Packed reads in HBM for kmhg_sh_count_reads_device: bases and qualities (8-B aligned,
    16 B of padding), int64 offsets[n + 1], has_qual[n] (0 = FASTA record)."""

    def __init__(self, seq, qual, off, hasq):
        self.seq, self.qual, self.off, self.hasq = seq, qual, off, hasq
        self.n = int(hasq.numel())

    @classmethod
    def from_arrays(cls, seq, qual, device, has_qual=None) -> "DeviceReads":
        """seq / qual: (n_reads, read_len) uint8 numpy arrays (synth.reads)."""
        import numpy as np
        n, rl = seq.shape
        flat = np.zeros(n * rl + 16, np.uint8)
        flat[:n * rl] = seq.reshape(-1)
        qf = np.zeros(n * rl + 16, np.uint8)
        qf[:n * rl] = qual.reshape(-1)
        off = np.arange(n + 1, dtype=np.int64) * rl
        hq = np.ones(n, np.uint8) if has_qual is None else has_qual.astype(np.uint8)
        t = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
        return cls(t(flat), t(qf), t(off), t(hq))

    @property
    def n_bases(self) -> int:
        return int(self.off[-1].item())

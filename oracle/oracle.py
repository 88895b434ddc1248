"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

ctypes front-ends to
  * ``liboracle.so``        -- the clean-room C restatement in ``kmer_oracle.c``
  * ``_ref/libkmh_ref.so``  -- the reference's own index core (src/kmer_pos.c,
                               src/kmer_util.c, klib) compiled by ``oracle/Makefile``
                               behind the R-free harness ``ref_harness.c``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  Arrays follow the reference's R layouts (column-major 2 x N / 3 x P,
i.e. row-interleaved) so they compare 1:1 with what ``kmer.pos`` / ``seq.kmer.pos`` return.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ORC = None
_REF = None

i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")


def build(force: bool = False) -> None:
    """Compile liboracle.so (and _ref/ when /root/reference is present)."""
    if force or not os.path.exists(os.path.join(_HERE, "liboracle.so")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _orc():
    global _ORC
    if _ORC is None:
        build()
        lib = C.CDLL(os.path.join(_HERE, "liboracle.so"))
        lib.orc_windows.restype = C.c_long
        lib.orc_windows.argtypes = [C.c_char_p, C.c_long, C.c_int, u64p, i32p, i32p]
        lib.orc_index_build.restype = C.c_long
        lib.orc_index_build.argtypes = [C.c_char_p, C.c_long, C.c_int, u64p, i32p, i64p, i32p,
                                        C.POINTER(C.c_long), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int32)]
        lib.orc_query.restype = C.c_int64
        lib.orc_query.argtypes = [u64p, i32p, i64p, i32p, C.c_long, C.c_char_p, C.c_long, C.c_int,
                                  C.c_void_p]
        lib.orc_pairs.restype = C.c_int64
        lib.orc_pairs.argtypes = [i32p, i64p, i32p, C.c_long, C.c_void_p, i32p]
        lib.orc_khash_order.restype = C.c_long
        lib.orc_khash_order.argtypes = [u64p, C.c_long, i64p]
        _ORC = lib
    return _ORC


def ref_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libkmh_ref.so"))


class _RefPos(C.Structure):
    _fields_ = [("n_kmers", C.c_long), ("kmers", C.c_void_p),
                ("n_pos", C.c_long), ("pos", C.c_void_p),
                ("n_pairs", C.c_long), ("pairs", C.c_void_p),
                ("n_counts", C.c_long), ("counts", C.c_void_p)]


def _ref():
    global _REF
    if _REF is None:
        lib = C.CDLL(os.path.join(_HERE, "_ref", "libkmh_ref.so"))
        lib.ref_build.restype = C.c_void_p
        lib.ref_build.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_long),
                                  C.POINTER(C.c_int)]
        lib.ref_size.restype = C.c_long
        lib.ref_size.argtypes = [C.c_void_p]
        lib.ref_free_index.argtypes = [C.c_void_p]
        lib.ref_free.argtypes = [C.c_void_p]
        lib.ref_positions.argtypes = [C.c_void_p, C.c_uint, C.POINTER(_RefPos)]
        lib.ref_query.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.POINTER(C.c_long),
                                  C.POINTER(C.POINTER(C.c_int))]
        lib.ref_count.restype = C.c_void_p
        lib.ref_count.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.POINTER(C.c_int)]
        lib.ref_kmer_count.restype = C.c_long
        lib.ref_kmer_count.argtypes = [C.c_void_p]
        lib.ref_rows_chunk.restype = C.c_long
        lib.ref_rows_chunk.argtypes = [C.c_void_p, C.c_uint, i64p, i32p, C.c_long]
        lib.ref_totals.argtypes = [C.c_void_p, C.POINTER(C.c_long), C.POINTER(C.c_long),
                                   C.POINTER(C.c_long)]
        _REF = lib
    return _REF


def _as_bytes(seq) -> bytes:
    if isinstance(seq, str):
        return seq.encode("latin-1")
    if isinstance(seq, np.ndarray):
        return seq.astype(np.uint8, copy=False).tobytes()
    return bytes(seq)


# --------------------------------------------------------------------------- restatement
def windows(seq, k: int):
    """(keys u64, start1 i32, end1 i32) of every window the reference visits."""
    b = _as_bytes(seq)
    L = len(b)
    keys = np.empty(L + 1, np.uint64)
    s = np.empty(L + 1, np.int32)
    e = np.empty(L + 1, np.int32)
    n = _orc().orc_windows(b, L, k, keys, s, e)
    return keys[:n], s[:n], e[:n]


class OracleIndex:
    """Canonical CSR: key ids rank distinct keys by first position; positions ascend."""

    def __init__(self, seq, k: int):
        b = _as_bytes(seq)
        L = len(b)
        self.k = k
        cap = L + 1
        keys = np.empty(cap, np.uint64)
        counts = np.empty(cap, np.int32)
        offs = np.empty(cap + 1, np.int64)
        pos = np.empty(cap, np.int32)
        n = C.c_long(0)
        p = C.c_int64(0)
        mx = C.c_int32(0)
        U = _orc().orc_index_build(b, L, k, keys, counts, offs, pos, C.byref(n), C.byref(p),
                                   C.byref(mx))
        if U < 0:
            raise MemoryError("oracle allocation failed")
        self.U, self.N, self.P, self.max_n = int(U), int(n.value), int(p.value), int(mx.value)
        self.keys = keys[:U].copy()
        self.counts = counts[:U].copy()
        self.offsets = offs[:U + 1].copy()
        self.positions = pos[:self.N].copy()

    # kmer.pos pieces in canonical order -----------------------------------------------
    def pos_rows(self) -> np.ndarray:
        """2 x N data (i, pos) interleaved, i 1-based in canonical order."""
        out = np.empty((self.N, 2), np.int32)
        out[:, 0] = np.repeat(np.arange(1, self.U + 1, dtype=np.int32), self.counts)
        out[:, 1] = self.positions
        return out.reshape(-1)

    def pair_rows(self, order=None) -> np.ndarray:
        out = np.empty(3 * self.P + 1, np.int32)
        o = None if order is None else np.ascontiguousarray(order, np.int64)
        n = _orc().orc_pairs(self.counts, self.offsets, self.positions, self.U,
                             None if o is None else o.ctypes.data, out)
        assert n == self.P
        return out[:3 * self.P]

    def pairs_with(self, other: "OracleIndex", order=None) -> np.ndarray:
        """kmer_pair_pos (src/kmer_hash.c:1174-1203) as intended: for each live k-mer of self (in
        canonical order, or `order`), if `other` holds it, all (pos_self, pos_other) with self's
        positions outer.  2 x M interleaved int32."""
        ids = np.arange(self.U) if order is None else np.asarray(order)
        srt = np.argsort(other.keys, kind="stable")
        sk = other.keys[srt]
        at = np.searchsorted(sk, self.keys[ids]) if len(sk) else np.zeros(len(ids), np.int64)
        out = []
        for c, p in zip(ids, at):
            if p < len(sk) and sk[p] == self.keys[c]:
                o = srt[p]
                pa = self.positions[self.offsets[c]:self.offsets[c + 1]]
                pb = other.positions[other.offsets[o]:other.offsets[o + 1]]
                out.append(np.stack([np.repeat(pa, len(pb)), np.tile(pb, len(pa))], 1))
        if not out:
            return np.empty(0, np.int32)
        return np.concatenate(out).astype(np.int32).reshape(-1)

    def kmer_strings(self) -> list[str]:
        return [decode(int(x), self.k) for x in self.keys]

    def khash_order(self) -> np.ndarray:
        """ids in the bucket order khash 0.2.8 gives the reference (kmer_positions' row order)."""
        out = np.empty(self.U, np.int64)
        r = _orc().orc_khash_order(self.keys, self.U, out)
        assert r == self.U
        return out

    def query(self, seq, kq: int) -> np.ndarray:
        b = _as_bytes(seq)
        lib = _orc()
        h = lib.orc_query(self.keys, self.counts, self.offsets, self.positions, self.U, b, len(b),
                          kq, None)
        rows = np.empty(2 * h + 1, np.int32)
        h2 = lib.orc_query(self.keys, self.counts, self.offsets, self.positions, self.U, b, len(b),
                           kq, rows.ctypes.data)
        assert h2 == h
        return rows[:2 * h]


class OracleCounts:
    """count.kmers restated (reference src/kmer_hash.c:548-591, seq_to_counts :220-251,
    kmer_count_insert :185-208): distinct keys in first-insertion order, each with a vector of
    `source_n` per-source window counts.  add() is one count.kmers call."""

    def __init__(self, k: int, source_n: int):
        self.k, self.S = k, source_n
        self.keys: list[int] = []
        self.row: dict[int, int] = {}
        self.M: list[np.ndarray] = []
        self.kmer_count = 0

    def add(self, seqs, source: int) -> None:
        if source < 0 or source >= self.S:      # every insert warns and fails: nothing counted
            return
        for seq in seqs:
            b = _as_bytes(seq)
            if len(b) <= self.k:
                continue
            keys, _, _ = windows(b, self.k)
            uk, first, cnt = np.unique(keys, return_index=True, return_counts=True)
            for j in np.argsort(first, kind="stable"):
                key = int(uk[j])
                r = self.row.get(key)
                if r is None:
                    r = self.row[key] = len(self.keys)
                    self.keys.append(key)
                    self.M.append(np.zeros(self.S, np.int32))
                    self.kmer_count += 1
                self.M[r][source] += int(cnt[j])

    @property
    def U(self) -> int:
        return len(self.keys)

    def index(self) -> "OracleIndex":
        """The counts as an OracleIndex-shaped CSR (positions = per-source counts)."""
        ix = OracleIndex.__new__(OracleIndex)
        U, S = self.U, self.S
        ix.k, ix.U, ix.N, ix.P, ix.max_n = self.k, U, U * S, U * S * (S - 1) // 2, S if U else 0
        ix.keys = np.array(self.keys, np.uint64)
        ix.counts = np.full(U, S, np.int32)
        ix.offsets = np.arange(U + 1, dtype=np.int64) * S
        ix.positions = (np.stack(self.M).reshape(-1) if U else np.empty(0, np.int32)).astype(
            np.int32)
        return ix


_NUC = "ACTG"


def decode(key: int, k: int) -> str:
    """kmer_seq (reference src/kmer_hash.c:123-133): LSB pair is the last base."""
    out = []
    for _ in range(k):
        out.append(_NUC[key & 3])
        key >>= 2
    return "".join(reversed(out))


# --------------------------------------------------------------------------- reference
class RefIndex:
    """The compiled reference index (khash order, exactly what the R API would return)."""

    def __init__(self, seq, k: int, do_sort: int = 0):
        lib = _ref()
        self._b = _as_bytes(seq)
        cnt = C.c_long(0)
        err = C.c_int(0)
        self.k = k
        self.h = lib.ref_build(self._b, k, do_sort, C.byref(cnt), C.byref(err))
        if err.value == 1:
            raise ValueError("k must be a positive integer less than 1+MAX_K")
        if err.value == 2:
            raise ValueError("the length of the sequence must be at least k")
        self.kmer_count = int(cnt.value)

    def positions(self, opt: int) -> dict:
        lib = _ref()
        r = _RefPos()
        lib.ref_positions(self.h, opt, C.byref(r))
        out = {"kmer": None, "pos": None, "pair.pos": None, "count": None}

        def take(ptr, n, dt):
            a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_int32)), shape=(n,)).copy() \
                if n else np.empty(0, dt)
            lib.ref_free(ptr)
            return a

        if opt & 1:
            raw = C.string_at(r.kmers, r.n_kmers * (self.k + 1)) if r.n_kmers else b""
            lib.ref_free(r.kmers)
            out["kmer"] = [raw[i * (self.k + 1):i * (self.k + 1) + self.k].decode()
                           for i in range(r.n_kmers)]
        if opt & 2:
            out["pos"] = take(r.pos, 2 * r.n_pos, np.int32)
        if opt & 4:
            out["pair.pos"] = take(r.pairs, 3 * r.n_pairs, np.int32)
        if opt & 8:
            out["count"] = take(r.counts, r.n_counts, np.int32)
        return out

    def time_positions(self, opt: int) -> tuple[float, int, int]:
        """kmer_positions(opt) timed alone (the C bucket walk into flat arrays, as the R
        matrices are filled); the arrays are freed without being copied.  Returns (seconds,
        pos rows, pair rows)."""
        import time
        lib = _ref()
        r = _RefPos()
        t0 = time.perf_counter()
        lib.ref_positions(self.h, opt, C.byref(r))
        t = time.perf_counter() - t0
        for p in (r.kmers, r.pos, r.pairs, r.counts):
            if p:
                lib.ref_free(p)
        return t, int(r.n_pos), int(r.n_pairs)

    def totals(self) -> tuple[int, int, int]:
        """(N, P, max n) over the live buckets."""
        n, p, m = C.c_long(0), C.c_long(0), C.c_long(0)
        _ref().ref_totals(self.h, C.byref(n), C.byref(p), C.byref(m))
        return int(n.value), int(p.value), int(m.value)

    def rows_sha256(self, opt: int, chunk_rows: int = 1 << 24) -> tuple[str, int]:
        """sha256 of kmer.pos's $pos (opt 2) or $pair.pos (opt 4) R-matrix data in the
        reference's khash order, streamed from the bucket walk (ref_rows_chunk) so pair tables
        of many GB are digested without being held.  Returns (hexdigest, rows)."""
        import hashlib
        width = 2 if opt == 2 else 3
        st = np.zeros(5, np.int64)
        buf = np.empty(width * chunk_rows, np.int32)
        h = hashlib.sha256()
        rows = 0
        while True:
            n = _ref().ref_rows_chunk(self.h, opt, st, buf, chunk_rows)
            if n == 0:
                break
            h.update(memoryview(buf[:width * n]))
            rows += n
        return h.hexdigest(), rows

    @classmethod
    def counts(cls, seqs, k: int, source: int, source_n: int, into: "RefIndex | None" = None):
        """count.kmers(seqs, c(k, source, source_n), into) on the compiled reference core."""
        lib = _ref()
        self = into if into is not None else cls.__new__(cls)
        if into is None:
            self.k, self.h = k, None
        bs = [_as_bytes(x) for x in seqs]
        arr = (C.c_char_p * len(bs))(*bs)
        err = C.c_int(0)
        h = lib.ref_count(self.h, arr, len(bs), k, source, source_n, C.byref(err))
        msgs = {1: "k must be a positive integer less than 1+MAX_K",
                4: "source_n must be larger than 1 and larger than source",
                5: "mismatch between specified k and that given in the external pointer"}
        if err.value:
            raise ValueError(msgs[err.value])
        self.h = h
        self.kmer_count = int(lib.ref_kmer_count(h))
        return self

    def query(self, seq, kq: int) -> np.ndarray:
        lib = _ref()
        n = C.c_long(0)
        rows = C.POINTER(C.c_int)()
        rc = lib.ref_query(self.h, _as_bytes(seq), kq, C.byref(n), C.byref(rows))
        if rc:
            raise ValueError("the sequence should be longer than k and k should not be longer "
                             "than 31")
        a = np.ctypeslib.as_array(rows, shape=(2 * n.value,)).copy() if n.value else \
            np.empty(0, np.int32)
        lib.ref_free(rows)
        return a

    def close(self):
        if self.h:
            _ref().ref_free_index(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------------------------------------- read counting
# count.kmers.fq.sh.rp / seq.kmer.depth.sh / kmer.spec.sh.n (SURVEY.md §8 f next-4, depth half)
def _orc_sh():
    lib = _orc()
    if not hasattr(lib, "_sh_ready"):
        d256 = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        lib.orc_qll.argtypes = [d256]
        lib.orc_read_kmers.restype = C.c_long
        lib.orc_read_kmers.argtypes = [C.c_char_p, C.c_char_p, C.c_long, C.c_int, C.c_int, u64p]
        lib.orc_depth.restype = C.c_int
        lib.orc_depth.argtypes = [u64p, i32p, C.c_long, C.c_int, C.c_char_p, C.c_long, C.c_int,
                                  i32p]
        lib._sh_ready = True
    return lib


def qll_table() -> np.ndarray:
    """q_to_ll (src/Q_to_log_likelihood.h) regenerated from its formula (sh_oracle.c)."""
    out = np.zeros(256, np.float64)
    _orc_sh().orc_qll(out)
    return out


def fastx_records(data: bytes):
    """kseq_read (klib kseq.h bundled as src/kseq.h, __KSEQ_READ) restated over a decompressed
    byte string: yields (seq, qual) where qual is None for a FASTA record, and stops at the end
    of the file (-1) or at the first record whose quality length differs from its sequence (-2),
    as kmer_reader_read's loop does (src/kmer_reader.c:55)."""
    n = len(data)
    pos = 0
    last_char = 0

    def line_from(p):                      # rest of the line, the '\n' consumed
        e = data.find(b"\n", p)
        return (data[p:], n) if e < 0 else (data[p:e], e + 1)

    while True:
        if last_char == 0:                 # jump to the next header
            while pos < n and data[pos] not in b">@":
                pos += 1
            if pos >= n:
                return
            pos += 1
        if pos >= n:                       # name: EOF with nothing read
            return
        e = pos
        while e < n and data[e] not in b" \t\n\v\f\r":
            e += 1
        delim = data[e] if e < n else 0
        pos = min(e + 1, n)
        if delim != 0x0A and pos < n:      # comment: rest of the header line
            _, pos = line_from(pos)
        seq = bytearray()
        c = -1
        while pos < n:
            c = data[pos]
            pos += 1
            if c in b">+@":
                break
            if c == 0x0A:
                c = -1
                continue
            seq.append(c)
            if pos < n:                    # ks_getuntil2 strips '\r' only when it read bytes
                rest, pos = line_from(pos)
                seq += rest
                if len(seq) > 1 and seq[-1] == 0x0D:
                    seq.pop()
            c = -1
        last_char = c if c in (0x3E, 0x40) else 0
        if c != 0x2B:                      # FASTA
            yield bytes(seq), None
            continue
        while pos < n and data[pos] != 0x0A:   # rest of the '+' line
            pos += 1
        if pos >= n:
            return                         # -2: no quality string
        pos += 1
        qual = bytearray()
        while pos < n:                     # at least one line, then while shorter than seq
            rest, pos = line_from(pos)
            qual += rest
            if len(qual) > 1 and qual[-1] == 0x0D:
                qual.pop()
            if len(qual) >= len(seq):
                break
        last_char = 0
        if len(qual) != len(seq):
            return                         # -2
        yield bytes(seq), bytes(qual)


def read_fastx(path: str) -> bytes:
    raw = open(path, "rb").read()
    if raw[:2] == b"\x1f\x8b":
        import gzip
        raw = gzip.decompress(raw)
    return raw


def read_kmers(seq: bytes, qual, k: int, min_q: int) -> np.ndarray:
    """Canonical k-mers of one read in iteration order (orc_read_kmers)."""
    out = np.zeros(max(len(seq) - k + 1, 1), np.uint64)
    n = _orc_sh().orc_read_kmers(seq, qual, len(seq), k, min_q, out)
    return out[:n]


class OracleSH:
    """suffix_hash_n restated as {canonical key: counts[counts_n]} (src/suffix_hash.c:179-285),
    filled by count.kmers.fq.sh.rp's reader (src/kmer_reader.c:41-76)."""

    def __init__(self, k: int, counts_n: int):
        self.k, self.S = k, counts_n
        self.table: dict[int, np.ndarray] = {}

    def add_fastq(self, path_or_bytes, min_q: int, max_reads: int, source: int) -> "OracleSH":
        data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else \
            read_fastx(path_or_bytes)
        chunks = []
        for i, (s, q) in enumerate(fastx_records(bytes(data))):
            if i >= max_reads:
                break
            if len(s) <= self.k:
                continue
            chunks.append(read_kmers(s, q, self.k, min_q))
        if chunks:
            allk = np.concatenate(chunks)
            uk, cnt = np.unique(allk, return_counts=True)
            for key, c in zip(uk.tolist(), cnt.tolist()):
                v = self.table.get(key)
                if v is None:
                    v = self.table[key] = np.zeros(self.S, np.int64)
                v[source] += c
        return self

    def arrays(self):
        """(keys ascending, counts U x S int32)"""
        keys = np.array(sorted(self.table), np.uint64)
        M = np.array([self.table[int(x)] for x in keys], np.int64).reshape(-1, self.S)
        return keys, M.astype(np.int32)

    def depth(self, seq, k: int) -> np.ndarray:
        """seq.kmer.depth.sh: (L, counts_n) int32; NA = INT_MIN"""
        b = _as_bytes(seq)
        keys, M = self.arrays()
        out = np.zeros(len(b) * self.S, np.int32)
        _orc_sh().orc_depth(keys, np.ascontiguousarray(M.reshape(-1)), len(keys), self.S, b,
                            len(b), k, out)
        return out.reshape(len(b), self.S)

    def spectrum(self, max_count: int, comb, comb_inner, source_min) -> np.ndarray:
        """sh_count_spectrum_nc (src/suffix_hash.c:338-421): (comb_n * S, max_count + 1)."""
        comb = [int(c) & 0xFFFFFFFF for c in comb]
        inner = [int(c) & 0xFFFFFFFF for c in comb_inner]
        smin = np.array([int(c) & 0xFFFFFFFF for c in source_min], np.int64)
        cn, S = len(comb), self.S
        out = np.zeros((max_count + 1, cn * S), np.float64)
        if any(x > 1 for x in inner) or any(c >= (1 << S) for c in comb):
            return out.T.copy()
        _, M = self.arrays()
        M = M.astype(np.int64) & 0xFFFFFFFF
        flag = np.zeros(len(M), np.int64)
        for j in range(S):
            flag |= (M[:, j] >= smin[j]).astype(np.int64) << j
        capped = np.minimum(M, max_count)
        for jj in range(cn):
            sel = (flag == comb[jj]) if inner[jj] else ((flag & comb[jj]) > 0)
            for kk in range(S):
                np.add.at(out[:, jj * S + kk], capped[sel, kk], 1.0)
        return out.T.copy()


def _ref_sh():
    lib = C.CDLL(os.path.join(_HERE, "_ref", "libkmh_ref_sh.so"))
    lib.ref_sh_count_fastq.restype = C.c_void_p
    lib.ref_sh_count_fastq.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_long, C.c_int, C.c_int]
    lib.ref_sh_size.restype = C.c_long
    lib.ref_sh_size.argtypes = [C.c_void_p]
    lib.ref_sh_counts_n.argtypes = [C.c_void_p]
    lib.ref_sh_dump.restype = C.c_long
    lib.ref_sh_dump.argtypes = [C.c_void_p, u64p, i32p]
    lib.ref_sh_depth.argtypes = [C.c_void_p, C.c_char_p, C.c_long, C.c_int, i32p]
    lib.ref_sh_spectrum.argtypes = [C.c_void_p, C.c_int, i32p, i32p, C.c_int, i32p,
                                    np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")]
    lib.ref_sh_free.argtypes = [C.c_void_p]
    return lib


def ref_sh_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libkmh_ref_sh.so"))


class RefSH:
    """The compiled reference suffix_hash_n (count_kmers_fastq_sh_rp & co., ref_sh_harness.c)."""

    def __init__(self):
        self.lib = _ref_sh()
        self.h = None

    def add_fastq(self, path: str, k: int, prefix_bits: int, min_q: int, max_reads: int,
                  source_n: int, source: int, thread_n: int = 1) -> "RefSH":
        # the reference's reader threads printf progress ("thread: 0 exit. ...") to stdout;
        # send it to stderr so a caller's stdout (bench.py's one JSON line) stays clean
        libc = C.CDLL(None)
        sys.stdout.flush()
        saved = os.dup(1)
        try:
            os.dup2(2, 1)
            self.h = self.lib.ref_sh_count_fastq(self.h, path.encode(), k, prefix_bits, min_q,
                                                 thread_n, max_reads, source_n, source)
            libc.fflush(None)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        return self

    def arrays(self):
        n = self.lib.ref_sh_size(self.h)
        S = self.lib.ref_sh_counts_n(self.h)
        keys = np.zeros(max(n, 1), np.uint64)
        M = np.zeros(max(n, 1) * S, np.int32)
        n2 = self.lib.ref_sh_dump(self.h, keys, M)
        assert n2 == n
        o = np.argsort(keys[:n], kind="stable")
        return keys[:n][o], M[:n * S].reshape(n, S)[o]

    def depth(self, seq, k: int) -> np.ndarray:
        b = _as_bytes(seq)
        S = self.lib.ref_sh_counts_n(self.h)
        out = np.zeros(max(len(b), 1) * S, np.int32)
        rc = self.lib.ref_sh_depth(self.h, b, len(b), k, out)
        if rc != 1:
            raise ValueError("Receieved error from seq_kmer_counts")
        return out[:len(b) * S].reshape(len(b), S)

    def spectrum(self, max_count, comb, comb_inner, source_min) -> np.ndarray:
        S = self.lib.ref_sh_counts_n(self.h)
        cn = len(comb)
        out = np.zeros(cn * S * (max_count + 1), np.float64)
        self.lib.ref_sh_spectrum(self.h, max_count, np.array(comb, np.int32),
                                 np.array(comb_inner, np.int32), cn,
                                 np.array(source_min, np.int32), out)
        return out.reshape(max_count + 1, cn * S).T.copy()

    def close(self):
        if self.h:
            self.lib.ref_sh_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

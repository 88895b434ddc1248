"""Host-side mirror of the reference's R API for the index hot path (reference kmer_hash.R:5-28).

    make_kmer_hash(seq, k, do_sort=False)  <- make.kmer.hash  (kmer_hash.R:5-8)
    kmer_pos(ex_ptr, opt_flag)             <- kmer.pos        (kmer_hash.R:10-21)
    seq_kmer_pos(ex_ptr, seq, k)           <- seq.kmer.pos    (kmer_hash.R:23-28)
    kmer_pairs(ptr_a, ptr_b)               <- kmer.pairs      (kmer_hash.R:30-34), fixed
    count_kmers(seq, params, hash_ptr)     <- count.kmers     (kmer_hash.R:43-46)
    count_kmers_fq_sh_rp(fq, params, ptr)  <- count.kmers.fq.sh.rp (kmer_hash.R:75-78)
    seq_kmer_depth_sh(ptr, seq, k)         <- seq.kmer.depth.sh    (kmer_hash.R:80-83)
    kmer_spec_sh_n(ptr, max_count, comb, comb_inner, source_min)
                                           <- kmer.spec.sh.n       (kmer_hash.R:93-96)
    set_row_order(ex_ptr, "khash")         kmer.pos rows in the reference's khash order (opt-in)

Same argument meaning, same validation order and the reference's own error messages (raised as
``KmerHashError``, the analogue of R's error()).  Results follow the R wrappers after their
``t()``: ``pos`` is an (N, 2) int32 matrix with columns (i, pos), ``pair.pos`` (P, 3) with
(i, x, y), the query an (H, 2) matrix with (i, j).  Everything runs through libkmhgpu.so on the
GPU; nothing here computes a result on the CPU.

The external pointer is an ``ExtPtr`` carrying the reference's tag "kmer_hash_250930"
(src/kmer_hash.c:22) and a finaliser that frees the device index (finalise_khash_ptr,
src/kmer_hash.c:56-66).
"""
from __future__ import annotations

import ctypes as C
import warnings
import weakref

import numpy as np

from . import _lib

KMER_HASH_TAG = "kmer_hash_250930"
SUFFIX_HASH_N_TAG = "suffix_hash_n_250930"          # src/kmer_hash.c:25
OPT_KMER, OPT_POS, OPT_PAIRS, OPT_COUNT = 1, 2, 4, 8
FIELDS = ("kmer", "pos", "pair.pos", "count")          # src/kmer_hash.c:18
INT_MAX = 2**31 - 1


class KmerHashError(ValueError):
    """R error() raised by the .Call bridge."""


class ExtPtr:
    """Analogue of the EXTPTRSXP returned by make_kmer_h_index."""

    def __init__(self, handle: int, tag: str = KMER_HASH_TAG):
        self._h = C.c_void_p(handle)
        self.tag = tag
        self._fin = weakref.finalize(self, ExtPtr._finalise, handle)

    @staticmethod
    def _finalise(handle):
        if handle:
            _lib.lib().kmhg_free(C.c_void_p(handle))

    @property
    def handle(self) -> C.c_void_p:
        if not self._h:
            raise KmerHashError("external pointer has been freed")
        return self._h

    def info(self) -> _lib.Info:
        inf = _lib.Info()
        _lib.check(_lib.lib().kmhg_index_info(self.handle, C.byref(inf)))
        return inf

    def free(self):
        if self._h:
            self._fin()
            self._h = C.c_void_p(0)


def _as_seq_bytes(seq, what: str) -> bytes:
    # as.character(seq); STRING_ELT(seq_r, 0) -- only the first element is used
    if isinstance(seq, (list, tuple)):
        if len(seq) < 1:
            raise KmerHashError(what)
        seq = seq[0]
    if isinstance(seq, str):
        return seq.encode("latin-1")
    if isinstance(seq, (bytes, bytearray)):
        return bytes(seq)
    if isinstance(seq, np.ndarray) and seq.dtype == np.uint8:
        return seq.tobytes()
    raise KmerHashError(what)


def _as_int(x, what: str) -> int:
    if isinstance(x, (list, tuple, np.ndarray)):
        if len(x) < 1:
            raise KmerHashError(what)
        x = x[0]
    try:
        return int(x)
    except (TypeError, ValueError):
        raise KmerHashError(what) from None


def make_kmer_hash(seq, k, do_sort=False) -> ExtPtr:
    """make.kmer.hash -> .Call("make_kmer_h_index", ...)  (src/kmer_hash.c:506-540)."""
    b = _as_seq_bytes(seq, "seq_r should be a character vector of length at least one")
    kk = _as_int(k, "k_r must be an integer vector of length at least one")
    ds = _as_int(do_sort, "sort_pos_r must be an integer vector of length at least one")
    out = C.c_void_p()
    rc = _lib.lib().kmhg_build(b, len(b), kk, ds, C.byref(out))
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(_lib.lib().kmhg_last_error().decode())
    _lib.check(rc)
    return ExtPtr(out.value)


def _extract(ptr) -> ExtPtr:
    # extract_khash_ptr, src/kmer_hash.c:491-503
    if not isinstance(ptr, ExtPtr):
        raise KmerHashError("ptr_r should be an external pointer")
    if ptr.tag != KMER_HASH_TAG:
        raise KmerHashError("External pointer has incorrect tag")
    return ptr


def kmer_pos(ex_ptr, opt_flag) -> dict:
    """kmer.pos -> .Call("kmer_positions", ...)  (src/kmer_hash.c:1054-1147).

    Returns {"kmer", "pos", "pair.pos", "count"}; unset flags give None (R's NULL)."""
    p = _extract(ex_ptr)
    if isinstance(opt_flag, (list, tuple, np.ndarray)) and len(opt_flag) != 1:
        raise KmerHashError("opt_flag_r should be an integer vector of length 1")
    opt = _as_int(opt_flag, "opt_flag_r should be an integer vector of length 1") & 0xFFFFFFFF
    L = _lib.lib()
    nk, npos, npair, ncnt = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    _lib.check(L.kmhg_positions_size(p.handle, opt, C.byref(nk), C.byref(npos), C.byref(npair),
                                     C.byref(ncnt)))
    # R's allocMatrix takes an int ncol: the reference overflows silently; we refuse cleanly.
    if npair.value > INT_MAX or npos.value > INT_MAX:
        raise KmerHashError("result has more than 2^31-1 columns (R matrix limit)")
    k = p.info().k
    kb = np.empty(nk.value * (k + 1), np.uint8) if opt & OPT_KMER else None
    pos = np.empty(2 * npos.value, np.int32) if opt & OPT_POS else None
    pairs = np.empty(3 * npair.value, np.int32) if opt & OPT_PAIRS else None
    cnt = np.empty(ncnt.value, np.int32) if opt & OPT_COUNT else None

    def ptr(a):
        return a.ctypes.data if a is not None and a.size else None

    _lib.check(L.kmhg_positions_fill(p.handle, opt, ptr(kb), ptr(pos), ptr(pairs), ptr(cnt)))
    out = dict.fromkeys(FIELDS)
    if kb is not None:
        out["kmer"] = [x.decode() for x in kb.reshape(-1, k + 1)[:, :k].view(f"S{k}").ravel()] \
            if nk.value else []
    if pos is not None:
        out["pos"] = pos.reshape(-1, 2)          # t(tmp$pos): columns i, pos
    if pairs is not None:
        out["pair.pos"] = pairs.reshape(-1, 3)   # t(tmp$pair.pos): columns i, x, y
    if cnt is not None:
        out["count"] = cnt
    return out


def kmer_pairs(ptr_a, ptr_b) -> np.ndarray:
    """kmer.pairs -> .Call("kmer_pair_pos", ...)  (src/kmer_hash.c:1174-1203, kmer_hash.R:30-34).

    Returns an (M, 2) int32 matrix with columns (a, b): for every k-mer held by both indices,
    each position in a paired with each position in b (a outer, b inner), k-mers in a's kmer.pos
    row order.  Defined where the reference crashes (empty buckets of a, out-of-bounds kh_exist
    on b); the indices must share k."""
    a, b = _extract(ptr_a), _extract(ptr_b)
    L = _lib.lib()
    q = C.c_void_p()
    h = C.c_int64()
    rc = L.kmhg_pairs_run(a.handle, b.handle, C.byref(q), C.byref(h))
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    try:
        if h.value > INT_MAX:
            raise KmerHashError("result has more than 2^31-1 columns (R matrix limit)")
        rows = np.empty(2 * h.value, np.int32)
        if h.value:
            _lib.check(L.kmhg_query_fill(q, rows.ctypes.data))
    finally:
        L.kmhg_query_free(q)
    return rows.reshape(-1, 2)


def set_row_order(ex_ptr, order: str = "first") -> None:
    """Label kmer.pos k-mers by first occurrence ("first", the default) or in the reference's own
    khash bucket order ("khash": byte-identical kmer.pos output, src/kmer_hash.c:1096-1124).
    KMHG_ROW_ORDER=khash in the environment makes "khash" the default for new indices."""
    p = _extract(ex_ptr)
    code = {"first": _lib.KMHG_ORDER_FIRST, "khash": _lib.KMHG_ORDER_KHASH}.get(order)
    if code is None:
        raise KmerHashError("order must be 'first' or 'khash'")
    _lib.check(_lib.lib().kmhg_set_row_order(p.handle, code))


def seq_kmer_pos(ex_ptr, seq, k) -> np.ndarray:
    """seq.kmer.pos -> .Call("sequence_kmer_positions", ...)  (src/kmer_hash.c:1151-1172).

    Returns an (H, 2) int32 matrix with columns (i, j): i = 1-based end of the query window,
    j = 1-based start of the indexed occurrence; rows ordered by i then j."""
    p = _extract(ex_ptr)
    if isinstance(seq, (list, tuple)) and len(seq) != 1:
        raise KmerHashError("seq_r should be a single sequence")
    b = _as_seq_bytes(seq, "seq_r should be a single sequence")
    if isinstance(k, (list, tuple, np.ndarray)) and len(k) != 1:
        raise KmerHashError("k should be an integer of length 1")
    kk = _as_int(k, "k should be an integer of length 1")
    L = _lib.lib()
    q = C.c_void_p()
    h = C.c_int64()
    rc = L.kmhg_query_run(p.handle, b, len(b), kk, C.byref(q), C.byref(h))
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    try:
        if h.value > INT_MAX:
            raise KmerHashError("result has more than 2^31-1 columns (R matrix limit)")
        rows = np.empty(2 * h.value, np.int32)
        if h.value:
            _lib.check(L.kmhg_query_fill(q, rows.ctypes.data))
    finally:
        L.kmhg_query_free(q)
    return rows.reshape(-1, 2)


def count_kmers(seq, params, hash_ptr=None) -> ExtPtr:
    """count.kmers -> .Call("count_kmers", hash.ptr, params, seq)  (src/kmer_hash.c:548-591).

    seq: a character vector (str or list of str); params = (k, source, source_n).  Every valid
    window of every sequence adds one to entry `source` of its k-mer's vector of source_n
    counts.  hash_ptr None makes a new counts pointer; otherwise the counts are added to it and
    the same pointer is returned.  kmer.pos / seq.kmer.pos read the count vectors as positions,
    as the reference does (test.R:340-343)."""
    if isinstance(seq, (str, bytes, bytearray)):
        seq = [seq]
    if not isinstance(seq, (list, tuple)) or len(seq) < 1 or \
            not all(isinstance(x, (str, bytes, bytearray)) for x in seq):
        raise KmerHashError("seq_r should be a character vector of length at least one")
    try:
        prm = [int(x) for x in params]
    except (TypeError, ValueError):
        raise KmerHashError("k_r must be an integer vector of length 3") from None
    if len(prm) != 3:
        raise KmerHashError("k_r must be an integer vector of length 3")
    k, source, source_n = prm
    if k < 1 or k > 32:
        raise KmerHashError("k must be a positive integer less than 1+MAX_K")
    if source_n < 1 or source >= source_n:
        raise KmerHashError("source_n must be larger than 1 and larger than source")
    if hash_ptr is not None and (not isinstance(hash_ptr, ExtPtr) or
                                 hash_ptr.tag != KMER_HASH_TAG or not hash_ptr._h):
        # extract_ext_ptr returns NULL (src/kmer_hash.c:574-577)
        raise KmerHashError("failed to extract kmer_hash from external pointer")
    bs = [x.encode("latin-1") if isinstance(x, str) else bytes(x) for x in seq]
    arr = (C.c_char_p * len(bs))(*bs)
    lens = (C.c_size_t * len(bs))(*[len(b) for b in bs])
    h = C.c_void_p(hash_ptr._h.value if hash_ptr is not None and hash_ptr._h else None)
    L = _lib.lib()
    rc = L.kmhg_count(C.byref(h), arr, lens, len(bs), k, source, source_n)
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    if source < 0:   # kmer_count_insert: one warning() per window, nothing counted
        warnings.warn(f"source ({source % 2**64}) equal to or larger than source_n ({source_n})")
    if hash_ptr is not None:
        return hash_ptr
    return ExtPtr(h.value)


# ------------------------------------------------------------------ read counting (suffix hash)
def _int_vec(x, n: int | None, what: str) -> list[int]:
    if isinstance(x, (int, np.integer)):
        x = [x]
    try:
        v = [int(a) for a in x]
    except (TypeError, ValueError):
        raise KmerHashError(what) from None
    if n is not None and len(v) != n:
        raise KmerHashError(what)
    return v


def _extract_sh(ptr):
    # extract_ext_ptr(hash_ptr_r, suffix_hash_n_tag): NULL for anything else (src/kmer_hash.c:41-52)
    if isinstance(ptr, ExtPtr) and ptr.tag == SUFFIX_HASH_N_TAG and ptr._h:
        return ptr
    return None


def count_kmers_fq_sh_rp(fq_file, params, hash_ptr=None) -> ExtPtr:
    """count.kmers.fq.sh.rp -> .Call("count_kmers_fastq_sh_rp", hash.ptr, params, fq.file)
    (src/kmer_hash.c:810-857; reader src/kmer_reader.c:41-147).

    params = (k, prefix_bits, min_q, thread_n, max_reads, max_mem, source_n, source).  Counts the
    canonical k-mers of the FASTA/FASTQ file (plain or gzip) the reference's quality iterator
    accepts into entry `source` of a suffix hash of source_n counts.  A hash_ptr that is not a
    suffix hash is ignored and a new one returned, as extract_ext_ptr yields NULL for it."""
    if isinstance(fq_file, (list, tuple)):
        if len(fq_file) != 1:
            raise KmerHashError("fq_file should be a character vector of length at least one")
        fq_file = fq_file[0]
    if not isinstance(fq_file, (str, bytes)):
        raise KmerHashError("fq_file should be a character vector of length at least one")
    prm = _int_vec(params, 8, "k_r must be an integer vector of length 6 (k, prefix_bits, min_q, "
                              "thread_n, max_reads, max_mem, source_n, source")
    sh = _extract_sh(hash_ptr)
    h = C.c_void_p(sh._h.value if sh is not None else None)
    arr = (C.c_int32 * 8)(*[((x + 2**31) % 2**32) - 2**31 for x in prm])
    path = fq_file.encode() if isinstance(fq_file, str) else fq_file
    L = _lib.lib()
    rc = L.kmhg_sh_count_fastq(C.byref(h), path, arr)
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    if sh is not None:
        return sh
    return ExtPtr(h.value, tag=SUFFIX_HASH_N_TAG)


def seq_kmer_depth_sh(hash_ptr, seq, k) -> np.ndarray:
    """seq.kmer.depth.sh -> .Call("seq_kmer_depth_sh", hash.ptr, seq, k)
    (src/kmer_hash.c:859-879, seq_kmer_counts src/kmer_reader.c:155-193).

    Returns the (counts_n, L) int32 matrix R gets (no t() in the wrapper); NA is INT_MIN."""
    sh = _extract_sh(hash_ptr)
    if sh is None:
        raise KmerHashError("unable to obtain suffix_hash_n from external pointer")
    if isinstance(k, (list, tuple, np.ndarray)) and len(k) != 1:
        raise KmerHashError("k_r should be a single integer")
    kk = _as_int(k, "k_r should be a single integer")
    if isinstance(seq, (list, tuple)) and len(seq) != 1:
        raise KmerHashError("seq_r should be a character vector of length 1")
    b = _as_seq_bytes(seq, "seq_r should be a character vector of length 1")
    S = sh.info().sources
    out = np.empty(max(len(b) * S, 1), np.int32)
    L = _lib.lib()
    rc = L.kmhg_sh_depth(sh.handle, b, len(b), kk, out.ctypes.data)
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    return out[:len(b) * S].reshape(len(b), S).T


def kmer_spec_sh_n(hash_ptr, max_count, comb, comb_inner, source_min) -> np.ndarray:
    """kmer.spec.sh.n -> .Call("kmer_spectrum_suffix_hash_n", ...)  (src/kmer_hash.c:1010-1039,
    sh_count_spectrum_nc src/suffix_hash.c:338-421).

    Returns the (comb_n * counts_n, max_count + 1) float64 matrix; an invalid comb / comb_inner
    gives zeros and the reference's message, as its Rprintf branch does."""
    sh = _extract_sh(hash_ptr)
    if sh is None:
        raise KmerHashError("unable to obtain suffix_hash_n from external pointer")
    mc = _int_vec(max_count, 1, "max_count_r should be a single integer")[0]
    cb = _int_vec(comb, None, "comb_r should be an integer vector of length > 0")
    if len(cb) < 1:
        raise KmerHashError("comb_r should be an integer vector of length > 0")
    ci = _int_vec(comb_inner, None,
                  "comb_inner_r should be an integer vector of the same length as comb_r")
    if len(ci) != len(cb):
        raise KmerHashError("comb_inner_r should be an integer vector of the same length as comb_r")
    S = sh.info().sources
    sm = _int_vec(source_min, None,
                  "source_min_r should be an integer vector of length sh->counts_n")
    if len(sm) != S:
        raise KmerHashError("source_min_r should be an integer vector of length sh->counts_n")
    a32 = lambda v: np.array([((x + 2**31) % 2**32) - 2**31 for x in v], np.int32)  # noqa: E731
    cb_a, ci_a, sm_a = a32(cb), a32(ci), a32(sm)
    if mc < 0:
        raise KmerHashError("max_count must be >= 0")
    out = np.zeros(max((mc + 1) * len(cb) * S, 1), np.float64)
    st = C.c_int(0)
    L = _lib.lib()
    rc = L.kmhg_sh_spectrum(sh.handle, mc, cb_a.ctypes.data, ci_a.ctypes.data, len(cb),
                            sm_a.ctypes.data, len(sm), out.ctypes.data, C.byref(st))
    if rc == _lib.KMHG_EINVAL:
        raise KmerHashError(L.kmhg_last_error().decode())
    _lib.check(rc)
    if st.value != 1:
        warnings.warn(f"sh_count_spectrum_nc returned an error: {st.value}")
    return out[:(mc + 1) * len(cb) * S].reshape(mc + 1, len(cb) * S).T


def counts_table(ptr):
    """(keys, counts) rows of a counts pointer or suffix hash (tests and inspection)."""
    if not isinstance(ptr, ExtPtr):
        raise KmerHashError("ptr_r should be an external pointer")
    inf = ptr.info()
    keys = np.zeros(max(inf.n_kmers, 1), np.uint64)
    M = np.zeros(max(inf.n_kmers * inf.sources, 1), np.int32)
    _lib.check(_lib.lib().kmhg_counts_export(ptr.handle, keys.ctypes.data, M.ctypes.data))
    return keys[:inf.n_kmers], M[:inf.n_kmers * inf.sources].reshape(inf.n_kmers, inf.sources)

"""The R glue (kmer_hasher_amd/R/kmer_hash_glue.c), compiled and driven without R.

R is not installed in this image, so tests/rshim holds declaration-only stand-ins for R.h,
Rinternals.h and R_ext/Rdynload.h (R's public API signatures) and fake_r.c, a tiny R runtime:
error() unwinds to the .Call like R's longjmp, PROTECT depth is counted, external pointers carry
tag / address / finaliser, and R_registerRoutines records the table.  The glue and the runtime
link into tests/rshim/_build/librglue.so (tests/rshim/Makefile, run by __graft_entry__.build()),
which these tests load with ctypes.

CPU: the glue type-checks under -Wall -Wextra -pedantic -Werror; its registration matches the
reference's names and arities (src/kmer_hash.c:1205-1224); every validation branch raises the
reference's message (src/kmer_hash.c:491-520, 548-591, 1054-1060, 1151-1164) before any device
work.  GPU: make_kmer_h_index -> kmer_positions / sequence_kmer_positions / kmer_pair_pos /
count_kmers through the glue, against the oracle and the reference's own raw digests.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from kmh_canon import sha

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SHIM = os.path.join(HERE, "rshim")
LIB = os.path.join(SHIM, "_build", "librglue.so")
GLUE = os.path.join(ROOT, "kmer_hasher_amd", "R", "kmer_hash_glue.c")
TAG = "kmer_hash_250930"
INTSXP, REALSXP, STRSXP, VECSXP, EXTPTRSXP = 13, 14, 16, 19, 22


def _build():
    from kmer_hasher_amd import _lib
    _lib.lib()                                   # libkmhgpu.so exists (built by build())
    subprocess.run(["make", "-s", "-C", SHIM], check=True)


class FakeR:
    def __init__(self):
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(GLUE):
            _build()
        L = C.CDLL(LIB)
        S = C.c_void_p
        for name, res, args in [
                ("fr_init", C.c_int, []), ("fr_routine", C.c_char_p, [C.c_int, C.POINTER(C.c_int)]),
                ("fr_nil", S, []),
                ("fr_str", S, [C.POINTER(C.c_char_p), C.POINTER(C.c_int64), C.c_int64]),
                ("fr_int", S, [C.POINTER(C.c_int), C.c_int64]),
                ("fr_real", S, [C.POINTER(C.c_double), C.c_int64]),
                ("fr_extptr", S, [S, C.c_char_p]), ("fr_type", C.c_int, [S]),
                ("fr_len", C.c_int64, [S]), ("fr_nrow", C.c_int, [S]), ("fr_ncol", C.c_int, [S]),
                ("fr_ints", C.POINTER(C.c_int), [S]), ("fr_reals", C.POINTER(C.c_double), [S]),
                ("fr_elt", S, [S, C.c_int64]), ("fr_chars", C.c_char_p, [S]), ("fr_names", S, [S]),
                ("fr_addr", S, [S]), ("fr_tag", C.c_char_p, [S]),
                ("fr_has_finalizer", C.c_int, [S]), ("fr_last_error", C.c_char_p, []),
                ("fr_last_warning", C.c_char_p, []), ("fr_warnings", C.c_int, []),
                ("fr_call", C.c_int, [C.c_char_p, C.c_int, C.POINTER(S), C.POINTER(S)]),
                ("fr_finalize", C.c_int, [S]), ("fr_reset", None, [])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L
        self.n_routines = L.fr_init()

    # R values
    def s(self, *strs):
        b = [x.encode("latin-1") if isinstance(x, str) else x for x in strs]
        arr = (C.c_char_p * len(b))(*b)
        lens = (C.c_int64 * len(b))(*[len(x) for x in b])
        return self.L.fr_str(arr, lens, len(b))

    def i(self, *v):
        return self.L.fr_int((C.c_int * len(v))(*v), len(v))

    def d(self, *v):
        return self.L.fr_real((C.c_double * len(v))(*v), len(v))

    def nil(self):
        return self.L.fr_nil()

    def call(self, name, *args):
        """.Call(name, ...) -> result; RError(message) if the entry point called error()."""
        out = C.c_void_p()
        a = (C.c_void_p * len(args))(*args)
        rc = self.L.fr_call(name.encode(), len(args), a, C.byref(out))
        if rc == 1:
            raise RError(self.L.fr_last_error().decode())
        assert rc == 0, f"{name}: rc {rc} (2 = unknown name / arity, 3 = PROTECT imbalance)"
        return out.value

    def int_matrix(self, x):
        n = self.L.fr_len(x)
        a = np.ctypeslib.as_array(self.L.fr_ints(x), shape=(n,)).copy() if n else np.zeros(0, np.int32)
        return a.reshape(self.L.fr_ncol(x), self.L.fr_nrow(x)) if self.L.fr_nrow(x) >= 0 else a

    def strings(self, x):
        return [self.L.fr_chars(self.L.fr_elt(x, j)).decode() for j in range(self.L.fr_len(x))]

    def kmer_pos(self, ptr, opt):
        r = self.call("kmer_positions", ptr, self.i(opt))
        names = self.strings(self.L.fr_names(r))
        out = {}
        for j, nm in enumerate(names):
            e = self.L.fr_elt(r, j)
            t = self.L.fr_type(e)
            out[nm] = (None if t == 0 else self.strings(e) if t == STRSXP else self.int_matrix(e))
        return out


class RError(Exception):
    pass


@pytest.fixture(scope="module")
def R():
    r = FakeR()
    yield r
    r.L.fr_reset()


def test_glue_type_checks_pedantic():
    inc = ["-I" + SHIM, "-I" + os.path.join(ROOT, "include")]
    subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-Wno-cast-function-type"] + inc + [GLUE], check=True)
    # and as C++ (R packages are sometimes built with a C++ compiler front end)
    subprocess.run(["g++", "-fsyntax-only", "-x", "c++", "-Wall", "-Werror",
                    "-Wno-cast-function-type"] + inc + [GLUE], check=True)


def test_registration_matches_reference(R):
    got = {}
    for j in range(R.n_routines):
        n = C.c_int()
        name = R.L.fr_routine(j, C.byref(n)).decode()
        got[name] = n.value
    # the reference's callMethods (src/kmer_hash.c:1205-1219) for the symbols this path replaces
    ref = {"make_kmer_h_index": 3, "kmer_positions": 2, "sequence_kmer_positions": 3,
           "kmer_pair_pos": 2, "count_kmers": 3, "count_kmers_fastq_sh_rp": 3,
           "seq_kmer_depth_sh": 3, "kmer_spectrum_suffix_hash_n": 5}
    for name, n in ref.items():
        assert got.get(name) == n, name
    assert set(got) - set(ref) == {"kmer_row_order"}          # the one addition (documented)


@pytest.mark.parametrize("args,msg", [
    (lambda R: (R.i(1), R.i(5), R.i(0)), "seq_r should be a character vector of length at least one"),
    (lambda R: (R.s(), R.i(5), R.i(0)), "seq_r should be a character vector of length at least one"),
    (lambda R: (R.s("ACGTACGT"), R.d(5.0), R.i(0)), "k_r must be an integer vector of length at least one"),
    (lambda R: (R.s("ACGTACGT"), R.i(), R.i(0)), "k_r must be an integer vector of length at least one"),
    (lambda R: (R.s("ACGTACGT"), R.i(5), R.s("x")), "sort_pos_r must be an integer vector of length at least one"),
    (lambda R: (R.s("ACGTACGT"), R.i(0), R.i(0)), "k must be a positive integer less than 1+MAX_K"),
    (lambda R: (R.s("ACGTACGT"), R.i(33), R.i(0)), "k must be a positive integer less than 1+MAX_K"),
    (lambda R: (R.s("ACGTA"), R.i(5), R.i(0)), "the length of the sequence must be at least k"),
])
def test_make_kmer_h_index_validation(R, args, msg):
    """src/kmer_hash.c:506-520, in the reference's order (the sequence check first)."""
    with pytest.raises(RError) as e:
        R.call("make_kmer_h_index", *args(R))
    assert str(e.value) == msg


def test_pointer_checks(R):
    """extract_khash_ptr (src/kmer_hash.c:491-503) and a finalised pointer."""
    for entry, extra in [("kmer_positions", lambda: (R.i(15),)),
                         ("sequence_kmer_positions", lambda: (R.s("ACGTACGT"), R.i(3)))]:
        with pytest.raises(RError, match="^ptr_r should be an external pointer$"):
            R.call(entry, R.i(1), *extra())
        with pytest.raises(RError, match="^External pointer has incorrect tag$"):
            R.call(entry, R.L.fr_extptr(None, b"suffix_hash_n_250930"), *extra())
        with pytest.raises(RError, match="^External pointer has incorrect tag$"):
            R.call(entry, R.L.fr_extptr(None, None), *extra())
        # a pointer whose finaliser already ran: refused, not dereferenced
        with pytest.raises(RError, match="^external pointer has been finalised$"):
            R.call(entry, R.L.fr_extptr(None, TAG.encode()), *extra())
    with pytest.raises(RError, match="^ptr_r should be an external pointer$"):
        R.call("kmer_pair_pos", R.s("x"), R.s("y"))


def test_count_kmers_validation(R):
    """count_kmers, src/kmer_hash.c:548-570 (messages and order)."""
    with pytest.raises(RError, match="^seq_r should be a character vector of length at least one$"):
        R.call("count_kmers", R.nil(), R.i(15, 0, 1), R.i(1))
    with pytest.raises(RError, match="^k_r must be an integer vector of length 3$"):
        R.call("count_kmers", R.nil(), R.i(15, 0), R.s("ACGT"))
    with pytest.raises(RError, match="^k must be a positive integer less than 1\\+MAX_K$"):
        R.call("count_kmers", R.nil(), R.i(0, 0, 1), R.s("ACGT"))
    with pytest.raises(RError, match="^source_n must be larger than 1 and larger than source$"):
        R.call("count_kmers", R.nil(), R.i(15, 1, 1), R.s("ACGT"))
    with pytest.raises(RError, match="^failed to extract kmer_hash from external pointer$"):
        R.call("count_kmers", R.i(3), R.i(15, 0, 1), R.s("ACGT"))


def test_suffix_hash_validation(R):
    with pytest.raises(RError, match="^unable to obtain suffix_hash_n from external pointer$"):
        R.call("seq_kmer_depth_sh", R.nil(), R.s("ACGT"), R.i(3))
    with pytest.raises(RError, match="^unable to obtain suffix_hash_n from external pointer$"):
        R.call("kmer_spectrum_suffix_hash_n", R.L.fr_extptr(None, TAG.encode()), R.i(10),
               R.i(1), R.i(1), R.i(0))
    with pytest.raises(RError, match="^fq_file should be a character vector"):
        R.call("count_kmers_fastq_sh_rp", R.nil(), R.i(*[0] * 8), R.i(1))
    with pytest.raises(RError, match="^k_r must be an integer vector of length 6"):
        R.call("count_kmers_fastq_sh_rp", R.nil(), R.i(1, 2), R.s("x.fq"))


def test_device_errors_reach_r_error(R):
    """Valid arguments on a host without a GPU: the library's error text comes back through R's
    error() (no crash, no leaked PROTECT)."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the gpu tests cover this path)")
    with pytest.raises(RError) as e:
        R.call("make_kmer_h_index", R.s("ACGTACGTACGTAAAC"), R.i(5), R.i(0))
    assert str(e.value)


# ---------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_glue_end_to_end_vs_reference(gpu, R, golden, testfa):
    """make.kmer.hash -> kmer.pos(15) / seq.kmer.pos / kmer.pairs / count.kmers through the R
    glue: test.fa rows equal the oracle's (first-occurrence order) and, in khash order, the
    reference's own raw digests byte for byte."""
    from oracle import oracle as O
    recs = [r for r in golden[0]["records"] if r["name"] == "test.fa" and r["k"] in (10, 15, 31)]
    assert recs
    for r in recs:
        k = r["k"]
        ptr = R.call("make_kmer_h_index", R.s(testfa), R.i(k), R.i(1))
        assert R.L.fr_tag(ptr).decode() == TAG and R.L.fr_has_finalizer(ptr)
        res = R.kmer_pos(ptr, 15)
        oi = O.OracleIndex(testfa, k)
        assert np.array_equal(res["count"], oi.counts)
        assert np.array_equal(res["pos"].reshape(-1), oi.pos_rows())
        assert np.array_equal(res["pair.pos"].reshape(-1), oi.pair_rows())
        assert res["kmer"] == oi.kmer_strings()
        assert R.kmer_pos(ptr, 8)["pos"] is None                  # unset flags -> NULL
        R.call("kmer_row_order", ptr, R.s("khash"))
        raw = R.kmer_pos(ptr, 15)
        for f in ("count", "pos", "pair.pos", "kmer"):
            v = raw[f] if f == "kmer" else raw[f].reshape(-1)
            assert sha(v) == r["raw_sha"][f], (k, f)
        R.call("kmer_row_order", ptr, R.s("first"))     # kmer.pairs follows a's row order
        for kq, qv in r.get("query", {}).items():
            q = R.int_matrix(R.call("sequence_kmer_positions", ptr, R.s(testfa), R.i(int(kq))))
            assert q.shape == (qv["H"], 2) and sha(q.reshape(-1)) == qv["sha"], (k, kq)
        sub = testfa[:5000]
        p2 = R.call("make_kmer_h_index", R.s(sub), R.i(k), R.i(0))
        pairs = R.int_matrix(R.call("kmer_pair_pos", ptr, p2))
        assert np.array_equal(pairs.reshape(-1), oi.pairs_with(O.OracleIndex(sub, k)))
        assert R.L.fr_finalize(p2) == 1
        with pytest.raises(RError, match="^external pointer has been finalised$"):
            R.kmer_pos(p2, 15)
        assert R.L.fr_finalize(ptr) == 1
    # count.kmers into a new pointer, then into the same pointer from a second source
    seqs = [testfa[:20000], testfa[20000:45000]]
    cp = R.call("count_kmers", R.nil(), R.i(15, 0, 2), R.s(*seqs))
    assert R.call("count_kmers", cp, R.i(15, 1, 2), R.s(testfa[45000:])) == cp
    oc = O.OracleCounts(15, 2)
    oc.add(seqs, 0)
    oc.add([testfa[45000:]], 1)
    res = R.kmer_pos(cp, 15)
    want = oc.index()
    assert np.array_equal(res["count"], want.counts)
    assert np.array_equal(res["pos"].reshape(-1), want.pos_rows())
    R.L.fr_finalize(cp)

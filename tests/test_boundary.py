"""Boundary error / option paths without a GPU.

* do.sort (src/kmer_hash.c:528-529 -> sort_kmer_pos, src/kmer_pos.c:21-33): the reference's own
  sort is a semantic no-op on an index (positions are pushed in sequence order); pinned here on
  the compiled reference, so the engine's "accepted, positions already ascending" is exact.
* results of >= 2^31 rows: R's allocMatrix takes an int ncol (reference src/kmer_hash.c:1133,
  README.md:80-89).  The Python mirror (api.kmer_pos / api.seq_kmer_pos / api.kmer_pairs)
  refuses them with the documented KmerHashError before allocating anything; sizes are injected
  through a stand-in for the C-ABI's size entry points (the GPU twin in test_gpu_boundary.py
  produces real > 2^31 results).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O
from kmh_canon import sha

pytestmark = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")


def test_reference_do_sort_is_a_no_op(testfa):
    from kmer_hasher_amd import synth
    rr = synth.add_n_runs(synth.repeat_rich(200_000, 8, n_gap_every=40_000), 0.002, 9).tobytes()
    for s, k in ((testfa, 15), (rr, 21), (rr, 9)):
        a = O.RefIndex(s, k, do_sort=0).positions(15)
        b = O.RefIndex(s, k, do_sort=1).positions(15)
        for f in ("pos", "pair.pos", "count"):
            assert sha(a[f]) == sha(b[f]), (k, f)
        assert a["kmer"] == b["kmer"]


class _FakeLib:
    """Stands in for libkmhgpu's size / run entry points with injected result sizes."""

    def __init__(self, npos=0, npair=0, h=0):
        self.npos, self.npair, self.h = npos, npair, h
        self.filled = False

    def kmhg_positions_size(self, handle, opt, nk, npos, npair, ncnt):
        for p, v in ((nk, 1), (npos, self.npos), (npair, self.npair), (ncnt, 1)):
            C.cast(p, C.POINTER(C.c_int64))[0] = v if v is not None else 0
        return 0

    def kmhg_positions_fill(self, *a):
        self.filled = True
        return 0

    def kmhg_query_run(self, handle, seq, n, k, q, h):
        C.cast(h, C.POINTER(C.c_int64))[0] = self.h
        return 0

    def kmhg_pairs_run(self, a, b, q, h):
        C.cast(h, C.POINTER(C.c_int64))[0] = self.h
        return 0

    def kmhg_query_fill(self, *a):
        self.filled = True
        return 0

    def kmhg_query_free(self, q):
        return 0

    def kmhg_index_info(self, handle, inf):
        return 0

    def kmhg_free(self, h):
        return 0


@pytest.mark.parametrize("npos,npair", [(2**31, 0), (5, 2**31), (5, 2**33 + 7)])
def test_kmer_pos_refuses_2_31_rows(monkeypatch, npos, npair):
    from kmer_hasher_amd import _lib, api
    fake = _FakeLib(npos=npos, npair=npair)
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    ptr = api.ExtPtr(1)
    ptr._fin.detach()
    with pytest.raises(api.KmerHashError, match="2\\^31-1 columns"):
        api.kmer_pos(ptr, 15)
    assert not fake.filled


def test_kmer_pos_accepts_2_31_minus_1(monkeypatch):
    """INT_MAX columns is still a valid R matrix: the check is > INT_MAX, not >=."""
    from kmer_hasher_amd import _lib, api
    fake = _FakeLib(npos=3, npair=2**31 - 1)
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    monkeypatch.setattr(api.ExtPtr, "info", lambda self: type("I", (), {"k": 5})())
    monkeypatch.setattr(api.np, "empty", lambda n, dt: np.zeros(min(n, 6), dt))   # no 24 GB buffer
    ptr = api.ExtPtr(1)
    ptr._fin.detach()
    api.kmer_pos(ptr, 14)
    assert fake.filled


@pytest.mark.parametrize("fn", ["seq_kmer_pos", "kmer_pairs"])
def test_query_and_pairs_refuse_2_31_rows(monkeypatch, fn):
    from kmer_hasher_amd import _lib, api
    fake = _FakeLib(h=2**31)
    monkeypatch.setattr(_lib, "lib", lambda: fake)
    ptr = api.ExtPtr(1)
    ptr._fin.detach()
    with pytest.raises(api.KmerHashError, match="2\\^31-1 columns"):
        if fn == "seq_kmer_pos":
            api.seq_kmer_pos(ptr, "ACGTACGT", 3)
        else:
            api.kmer_pairs(ptr, ptr)
    assert not fake.filled

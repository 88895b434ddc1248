"""Multi-device seq.kmer.pos through the R API's own entry point (KMHG_DEVICES, SURVEY.md §5
"Config / flags"; reference .Call("sequence_kmer_positions"), src/kmer_hash.c:1151-1172).

With KMHG_DEVICES=d0,d1,... the host-pointer kmhg_query_run splits the query's windows over the
listed devices in one process: the index is peer-copied to each other device once (one replica
per device, shared by that device's parts, which run in order on its host thread; the index's
own device uses the index itself -- KMHG_TEST_REPLICA makes its later parts use a same-device
copy, so the copy path runs on a one-GPU box too), each device receives only its slice of the
host sequence, and kmhg_query_fill writes every part straight into the caller's buffer.  KMHG_SLICE_POISON fills each device's
sequence buffer with 'A' outside its slice, so a window that read past its slice would show.
Rows must equal the oracle's unsharded rows, order included."""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _devices_list(torch, reps):
    n = torch.cuda.device_count()
    return ",".join(str(i % n) for i in range(reps))


@pytest.mark.parametrize("replica", ["copy", "home"])
@pytest.mark.parametrize("reps", [2, 3, 8])
def test_kmhg_devices_query_matches_oracle(gpu, test_lib, monkeypatch, reps, replica):
    from kmer_hasher_amd import make_kmer_hash, seq_kmer_pos, synth
    monkeypatch.setenv("KMHG_DEVICES", _devices_list(gpu, reps))
    if replica == "copy":
        monkeypatch.setenv("KMHG_TEST_REPLICA", "1")
    monkeypatch.setenv("KMHG_SLICE_POISON", "1")
    A = synth.add_n_runs(synth.iid(400_000, 71), 0.0005, 72, max_run=40)
    A[-32] = ord("N")                          # end-drop case in the last part
    B = synth.derived(A, 73)
    rr = synth.add_n_runs(synth.repeat_rich(300_000, 74, n_gap_every=50_000), 0.001, 75)
    for idx_seq, k, queries in ((A, 31, (A, B)), (rr, 21, (rr,)), (A, 17, (B,))):
        s = idx_seq.tobytes()
        oi = O.OracleIndex(s, k)
        ptr = make_kmer_hash(s, k)
        for qs in queries:
            qb = qs.tobytes()
            for kq in (k, k - 2):
                got = seq_kmer_pos(ptr, qb, kq).reshape(-1)
                assert np.array_equal(got, oi.query(qb, kq)), (reps, k, kq)
        ptr.free()
    # tiny queries: parts with no windows at all
    ptr = make_kmer_hash("ACGTACGTTT", 3)
    oi = O.OracleIndex("ACGTACGTTT", 3)
    for q in ("ACGTA", "ACGT", "TTTACG"):
        assert np.array_equal(seq_kmer_pos(ptr, q, 3).reshape(-1), oi.query(q, 3)), q
    ptr.free()


def test_kmhg_devices_device_readers(gpu, test_lib, monkeypatch):
    """A multi-device query's rows read on the device: kmhg_query_rows_device (gathered once on
    the index's device) and kmhg_query_copy_device (peer copies of the parts)."""
    import torch
    from kmer_hasher_amd import _lib, make_kmer_hash, synth
    monkeypatch.setenv("KMHG_DEVICES", _devices_list(gpu, 3))
    monkeypatch.setenv("KMHG_TEST_REPLICA", "1")
    s = synth.iid(200_000, 81).tobytes()
    oi = O.OracleIndex(s, 25)
    want = oi.query(s, 25)
    ptr = make_kmer_hash(s, 25)
    L = _lib.lib()
    q = C.c_void_p()
    h = C.c_int64()
    _lib.check(L.kmhg_query_run(ptr.handle, s, len(s), 25, C.byref(q), C.byref(h)))
    assert 2 * h.value == want.size
    dst = torch.empty(2 * h.value, dtype=torch.int32, device="cuda")
    _lib.check(L.kmhg_query_copy_device(q, C.c_void_p(dst.data_ptr()), None))
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy(), want)
    d = C.c_void_p()
    _lib.check(L.kmhg_query_rows_device(q, C.byref(d)))     # gathers the parts on the index's device
    assert d.value
    got = torch.empty_like(dst)
    # copy_device now reads the gathered buffer (the single-buffer path)
    _lib.check(L.kmhg_query_copy_device(q, C.c_void_p(got.data_ptr()), None))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want)
    _lib.check(L.kmhg_query_free(q))
    ptr.free()


def test_kmhg_devices_rejects_bad_list(gpu, monkeypatch):
    from kmer_hasher_amd import make_kmer_hash, seq_kmer_pos
    from kmer_hasher_amd.api import KmerHashError
    ptr = make_kmer_hash("ACGTACGTACGT", 4)
    for bad in ("0,x", "0,,1", "999"):
        monkeypatch.setenv("KMHG_DEVICES", bad)
        with pytest.raises((KmerHashError, RuntimeError), match="KMHG_DEVICES"):
            seq_kmer_pos(ptr, "ACGTACGT", 4)
    ptr.free()

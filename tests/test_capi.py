"""C-ABI library: loads, exports every symbol include/kmhgpu.h declares, and validates
arguments with the reference's error messages before touching a device (CPU-safe)."""
import ctypes as C
import subprocess

import numpy as np

import pytest

from kmer_hasher_amd import _lib, api


def test_library_loads_and_exports_header_symbols():
    L = _lib.lib()
    declared = _lib.header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib._PROTOS), "ctypes prototypes out of sync with the header"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(declared) <= exported


def test_product_library_reads_no_test_only_knob():
    """Fault injection and the A/B-only switches exist only in libkmhgpu_test.so (built from the
    same objects with the orchestrator compiled -DKMHG_TEST_BUILD): the product library does not
    even hold their names; the test build exports the same C-ABI."""
    import os
    test_lib = os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmhgpu_test.so")
    prod = open(os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmhgpu.so"), "rb").read()
    test = open(test_lib, "rb").read()
    for knob in (b"KMHG_TEST_DISORDER", b"KMHG_COUNT_BID", b"KMHG_RK_CAP", b"KMHG_D2H\0"):
        assert knob not in prod, knob
        assert knob in test, knob
    out = subprocess.run(["nm", "-D", "--defined-only", test_lib], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(_lib.header_symbols()) <= exported


def test_product_library_reads_only_four_knobs():
    """No environment variable can switch the product library's build or query path (VERDICT
    round 5, item 7): the only KMHG_ names it holds are its four product knobs; the path
    selectors live in the test build."""
    import re
    prod = open(_lib.LIB_PATH, "rb").read()
    names = set(re.findall(rb"KMHG_[A-Z0-9_]+", prod))
    assert names == {b"KMHG_TIMING", b"KMHG_DEVICES", b"KMHG_ROW_ORDER", b"KMHG_D2H_THREADS"}, names
    test = open(_lib.TEST_LIB_PATH, "rb").read()
    for knob in (b"KMHG_BUILD", b"KMHG_MAXR", b"KMHG_PACK8", b"KMHG_NB_ROUND", b"KMHG_DS_U8",
                 b"KMHG_QUERY_DIAG", b"KMHG_COUNT_TABLE", b"KMHG_SLICE_POISON"):
        assert knob in test, knob


def test_lib_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob     # the .hip_fatbin holds a gfx950 object
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob


@pytest.mark.parametrize("k", [0, -1, 33])
def test_build_rejects_k(k):
    out = C.c_void_p()
    rc = _lib.lib().kmhg_build(b"ACGTACGTACGT" * 4, 48, k, 0, C.byref(out))
    assert rc == _lib.KMHG_EINVAL
    assert _lib.lib().kmhg_last_error() == b"k must be a positive integer less than 1+MAX_K"


def test_build_rejects_short_sequence():
    out = C.c_void_p()
    rc = _lib.lib().kmhg_build(b"ACGTA", 5, 5, 0, C.byref(out))
    assert rc == _lib.KMHG_EINVAL
    assert _lib.lib().kmhg_last_error() == b"the length of the sequence must be at least k"
    # a NUL ends the sequence like a C string does (R strings never hold one)
    rc = _lib.lib().kmhg_build(b"ACG\0TACGT", 9, 4, 0, C.byref(out))
    assert rc == _lib.KMHG_EINVAL


def test_python_api_validation_messages():
    with pytest.raises(api.KmerHashError, match="the length of the sequence must be at least k"):
        api.make_kmer_hash("ACGT", 4)
    with pytest.raises(api.KmerHashError, match="k must be a positive integer less than 1"):
        api.make_kmer_hash("ACGTACGT", 40)
    with pytest.raises(api.KmerHashError, match="seq_r should be a character vector"):
        api.make_kmer_hash([], 4)
    with pytest.raises(api.KmerHashError, match="ptr_r should be an external pointer"):
        api.kmer_pos("not a pointer", 15)
    with pytest.raises(api.KmerHashError, match="ptr_r should be an external pointer"):
        api.seq_kmer_pos(None, "ACGT", 3)
    bad = api.ExtPtr(0, tag="kmer_tree_250930")
    with pytest.raises(api.KmerHashError, match="External pointer has incorrect tag"):
        api.kmer_pos(bad, 15)


def test_timing_report_is_json_without_device():
    import json
    buf = C.create_string_buffer(4096)
    assert _lib.lib().kmhg_timing_report(buf, len(buf)) == 0
    assert isinstance(json.loads(buf.value.decode()), dict)


def _khash_order_product(keys: np.ndarray) -> np.ndarray:
    keys = np.ascontiguousarray(keys, np.uint64)
    out = np.empty(len(keys), np.uint32)
    assert _lib.lib().kmhg_khash_order(keys.ctypes.data, len(keys), out.ctypes.data) == 0
    return out.astype(np.int64)


def test_khash_row_order_replay_matches_oracle(golden, testfa):
    """The product's host replay of khash 0.2.8 (row order of kmer.pos in KMHG_ORDER_KHASH mode)
    against the oracle's replay, which test_oracle_golden pins to the reference's raw digests --
    and directly against those digests."""
    from kmh_canon import sha
    from oracle import oracle as O
    from synth_inputs import sequence
    for r in golden[0]["records"]:
        if r["U"] > 300_000:
            continue
        oi = O.OracleIndex(sequence(r["name"], testfa), r["k"])
        order = _khash_order_product(oi.keys)
        assert np.array_equal(order, oi.khash_order()), (r["name"], r["k"])
        assert sha(oi.counts[order]) == r["raw_sha"]["count"]
    rng = np.random.default_rng(5)
    for U in (0, 1, 3, 4, 5, 100, 5000):             # resize boundaries included
        keys = np.unique(rng.integers(0, 2**62, U, dtype=np.uint64))
        rng.shuffle(keys)
        want = np.empty(len(keys), np.int64)
        assert O._orc().orc_khash_order(np.ascontiguousarray(keys), len(keys), want) == len(keys)
        assert np.array_equal(_khash_order_product(keys), want)

"""BASELINE.json configs at FULL size against digests of the reference's own output.

tests/golden/fullsize.json (tests/golden/make_fullsize_golden.py) holds, for configs 2-4, the
sha256 of what the compiled reference core (oracle/_ref: src/kmer_pos.c + src/kmer_util.c +
klib) returns, in its khash row order, and for config 5 the digest of the clean-room oracle's
query rows (the reference needs ~65 GB of host memory there).  The HIP path is run through the
device C-ABI (kmhg_build_device, kmhg_set_row_order(KMHG_ORDER_KHASH), kmhg_positions_fill_device,
kmhg_query_run_device) on the same seeded inputs and must reproduce every digest byte for byte.
"""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fullsize():
    with open(os.path.join(HERE, "golden", "fullsize.json")) as f:
        return json.load(f)


def _sha_dev(t) -> str:
    """sha256 of a device tensor's bytes, copied to the host in 256 MiB slices."""
    import torch
    h = hashlib.sha256()
    flat = t.reshape(-1).view(torch.uint8) if t.numel() else t.reshape(-1)
    for part in flat.split(1 << 28):
        h.update(memoryview(part.cpu().numpy()))
    return h.hexdigest()


def _build_khash(seq_np, k):
    import torch
    from kmer_hasher_amd import _lib, device as D
    seq = torch.from_numpy(seq_np).cuda()
    idx = D.DeviceIndex.build(seq, k)
    _lib.check(_lib.lib().kmhg_set_row_order(idx.handle, 1))       # KMHG_ORDER_KHASH
    return seq, idx


def _check_index(idx, r):
    inf = idx.info()
    assert (inf["n_kmers"], inf["n_positions"], inf["n_pairs"], inf["max_count"]) == \
        (r["U"], r["N"], r["P"], r["max_n"])
    if "kmer_count" in r:
        assert inf["kmer_count"] == r["kmer_count"]


def _check_positions(idx, r, opt):
    res = idx.positions(opt)
    for f in ("count", "pos", "pair.pos", "kmer"):
        if res[f] is not None and f in r["raw_sha"]:
            if f == "kmer":
                ks = res[f].cpu().numpy().copy()      # (U, k+1): k chars + NUL
                ks[:, -1] = ord("\n")                 # kmh_canon.sha joins strings by "\n"
                got = hashlib.sha256(ks.reshape(-1)[:-1].tobytes()).hexdigest()
            else:
                got = _sha_dev(res[f])
            assert got == r["raw_sha"][f], f
    del res


def _check_query(idx, seq, r, k):
    """The rows on the device and, as an R session receives them, in a host matrix
    (kmhg_query_fill: diagonal runs over PCIe, expanded by host threads)."""
    import ctypes
    import numpy as np
    from kmer_hasher_amd import _lib
    q = idx.query(seq, k)
    want = r["query"][str(k)]
    assert q.n_rows == want["H"]
    rows = q.rows()
    host = np.empty(2 * q.n_rows, np.int32)
    _lib.check(_lib.lib().kmhg_query_fill(q._h, ctypes.c_void_p(host.ctypes.data)))
    q.free()
    assert _sha_dev(rows) == want["sha"]
    assert hashlib.sha256(host.view(np.uint8)).hexdigest() == want["sha"]


def test_config2_10mbp_k31_reference_digests(gpu, fullsize):
    from kmer_hasher_amd import synth
    r = fullsize["config2"]
    seq, idx = _build_khash(synth.iid(r["L"], 1), r["k"])
    _check_index(idx, r)
    _check_positions(idx, r, 1 | 2 | 8)
    _check_query(idx, seq, r, 31)
    idx.free()


def test_config3_100mbp_k21_reference_digests(gpu, fullsize):
    """configs[2] at full size: 100 Mbp iid, k=21, build + kmer.pos + self seq.kmer.pos."""
    from kmer_hasher_amd import synth
    r = fullsize["config3"]
    seq, idx = _build_khash(synth.iid(r["L"], 2), r["k"])
    _check_index(idx, r)
    _check_positions(idx, r, 2 | 8)
    _check_query(idx, seq, r, 21)
    idx.free()


def test_config4_40mbp_pairs_reference_digests(gpu, fullsize):
    """configs[3] at full size: 40 Mbp repeat-rich, k=31, kmer.pos pos + pair.pos + count
    (P = 685,613,382 pair rows, 8.2 GB)."""
    from kmer_hasher_amd import synth
    r = fullsize["config4"]
    assert 5e8 <= r["P"] <= 1.5e9
    seq, idx = _build_khash(synth.config4(r["L"], 3), r["k"])
    _check_index(idx, r)
    _check_positions(idx, r, 2 | 4 | 8)
    # the pair rows as an R session receives them (kmhg_positions_fill: written by host threads
    # from the position lists)
    import ctypes
    import numpy as np
    from kmer_hasher_amd import _lib
    host = np.empty(3 * r["P"], np.int32)
    _lib.check(_lib.lib().kmhg_positions_fill(idx.handle, 4, None, None,
                                              ctypes.c_void_p(host.ctypes.data), None))
    assert hashlib.sha256(host.view(np.uint8)).hexdigest() == r["raw_sha"]["pair.pos"]
    del host
    idx.free()


def test_config5_500mbp_cross_query_digest(gpu, fullsize):
    """configs[4] on one GPU at full size: index(A = 500 Mbp iid), query B = derived(A)."""
    import torch
    from kmer_hasher_amd import device as D, synth
    r = fullsize["config5"]
    A = synth.iid(r["L"], 4)
    B = synth.derived(A, 5)
    a = torch.from_numpy(A).cuda()
    del A
    idx = D.DeviceIndex.build(a, r["k"])
    _check_index(idx, r)
    del a
    b = torch.from_numpy(B).cuda()
    del B
    _check_query(idx, b, r, r["k"])
    idx.free()

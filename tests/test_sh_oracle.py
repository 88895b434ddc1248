"""Read counting (count.kmers.fq.sh.rp / seq.kmer.depth.sh / kmer.spec.sh.n), CPU side: the
oracle against the reference's golden vectors, the oracle against the compiled reference on
fuzzed FASTX files (when oracle/_ref is built), and the product library's host FASTX reader
(kmhg_fastx_read: no GPU call) against the oracle's kseq restatement."""
import ctypes as C
import os

import numpy as np
import pytest

import sh_inputs as I
from kmh_canon import sha
from oracle import oracle as O

GOLD = I.load_golden()


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    return I.materialise(str(tmp_path_factory.mktemp("sh")))


def oracle_case(case, files):
    o = O.OracleSH(case["k"], case["source_n"])
    for f, pb, mq, mr, src in case["calls"]:
        o.add_fastq(files[f], mq, mr if mr >= 0 else 2**62, src)
    return o


def test_qll_table_pinned():
    assert sha(O.qll_table()) == GOLD["qll_sha"]


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: c["name"])
def test_oracle_matches_reference(case, inputs):
    files, genome = inputs
    o = oracle_case(case, files)
    keys, M = o.arrays()
    assert len(keys) == case["U"]
    assert sha(keys) == case["keys_sha"]
    assert sha(M) == case["counts_sha"]
    if "keys" in case:
        assert keys.tolist() == case["keys"]
    strings = I.depth_strings(genome, case["k"])
    for d in case["depth"]:
        assert sha(o.depth(strings[d["string"]], case["k"])) == d["sha"]
    for sp in case["spectra"]:
        got = o.spectrum(sp["max_count"], sp["comb"], sp["comb_inner"], sp["source_min"])
        assert sha(got) == sp["sha"]


@pytest.mark.skipif(not O.ref_sh_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("seed", [3, 4, 5])
def test_oracle_fuzz_vs_reference(seed, tmp_path):
    p = str(tmp_path / "r.fq")
    open(p, "wb").write(I.random_fastx(300, seed))
    for k, mq in [(4, 0), (11, 18), (25, 7)]:
        r = O.RefSH().add_fastq(p, k, min(8, 2 * k), mq, 2**62, 2, 1)
        o = O.OracleSH(k, 2).add_fastq(p, mq, 2**62, 1)
        rk, rm = r.arrays()
        ok, om = o.arrays()
        assert np.array_equal(rk, ok) and np.array_equal(rm, om)
        s = open(p, "rb").read()[:500].replace(b"\n", b"N")
        if len(s) >= k:
            assert np.array_equal(r.depth(s, k), o.depth(s, k))


def _host_reads(path, max_reads, k):
    from kmer_hasher_amd import _lib
    L = _lib.lib()
    h = C.c_void_p()
    _lib.check(L.kmhg_fastx_read(path.encode(), max_reads, k, C.byref(h)))
    try:
        nrec, nr, nb = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check(L.kmhg_reads_info(h, C.byref(nrec), C.byref(nr), C.byref(nb)))
        seq = np.zeros(nb.value + 1, np.uint8)
        qual = np.zeros(nb.value + 1, np.uint8)
        off = np.zeros(nr.value + 1, np.int64)
        hq = np.zeros(nr.value + 1, np.uint8)
        _lib.check(L.kmhg_reads_copy(h, seq.ctypes.data, qual.ctypes.data, off.ctypes.data,
                                     hq.ctypes.data))
    finally:
        L.kmhg_reads_free(h)
    return nrec.value, [(bytes(seq[off[i]:off[i + 1]]),
                         None if not hq[i] else bytes(qual[off[i]:off[i + 1]]))
                        for i in range(nr.value)]


@pytest.mark.parametrize("name", I.REF_FILES + ["tricky.fq", "random.fq", "sim.fq"])
@pytest.mark.parametrize("k,max_reads", [(5, -1), (21, 7), (31, -1)])
def test_host_reader_matches_kseq(name, k, max_reads, inputs):
    pytest.importorskip("torch")
    files, _ = inputs
    if not os.path.exists(os.path.join(os.path.dirname(O.__file__), "..", "kmer_hasher_amd",
                                       "libkmhgpu.so")):
        pytest.skip("libkmhgpu.so not built")
    nrec, reads = _host_reads(files[name], max_reads, k)
    recs = list(O.fastx_records(O.read_fastx(files[name])))
    if max_reads >= 0:
        recs = recs[:max_reads]
    assert nrec == len(recs)
    assert reads == [(s, q) for s, q in recs if len(s) > k]

"""Host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; VERDICT round 2
item 8).  tools/asan/host_check is built from the very sources the product and the
checker compile -- kmhg_fastx.h (the FASTA/FASTQ reader that parses untrusted files), kmhg_khash.h
(the khash row-order replay), oracle/kmer_oracle.c and oracle/sh_oracle.c -- with
-fsanitize=address,undefined -fno-sanitize-recover=all, so any out-of-bounds access, leak or UB
aborts the run.  Its outputs are also compared with the unsanitized Python/C oracle, on the
reference's own FASTQ fixtures and on fuzzed files."""
import gzip
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
EXE = os.path.join(ROOT, "tools", "asan", "host_check")
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def exe():
    # flock: pytest-xdist workers each run this fixture; one make at a time
    r = subprocess.run(["flock", os.path.join(ROOT, "tools", "asan", ".build.lock"),
                        "make", "-s", "-C", os.path.join(ROOT, "tools", "asan")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return EXE


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, (args, r.returncode, r.stderr[-3000:])
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    return r.stdout.split("\n")


def fnv(b: bytes) -> str:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def wsum(a: np.ndarray) -> str:
    """host_check's order-sensitive digest: sum x_i (i * 0x9E3779B97F4A7C15 + 1) mod 2^64."""
    x = a.astype(np.int64).view(np.uint64) if a.dtype == np.int64 else \
        (a.astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
         if a.dtype == np.int32 else a.astype(np.uint64))
    w = np.arange(x.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)
    with np.errstate(over="ignore"):
        return f"{int((x * w).sum(dtype=np.uint64)):016x}"


def expect_records(data: bytes, limit: int):
    out = []
    for i, (s, q) in enumerate(O.fastx_records(data)):
        if i >= limit:
            break
        out.append(f"R {len(s)} {0 if q is None else 1} {fnv(s)} {fnv(q or b'')}")
    return out


def fuzz_files(tmp_path):
    rng = np.random.default_rng(2024)
    base = open(os.path.join(GOLD, "test_10.fastq"), "rb").read()
    files = []
    specials = [b"\n", b"\r", b"@", b"+", b">", b" ", b"\t", b"N", b"\r\n"]
    for i in range(40):
        b = bytearray(base)
        for _ in range(int(rng.integers(1, 12))):
            p = int(rng.integers(0, len(b) + 1))
            op = rng.integers(0, 4)
            if op == 0 and len(b):
                del b[p:p + int(rng.integers(1, 40))]
            elif op == 1:
                b[p:p] = specials[int(rng.integers(0, len(specials)))]
            elif op == 2:
                b = b[:p]
            else:
                b[p:p] = bytes(rng.integers(0, 256, int(rng.integers(1, 30))).astype(np.uint8))
        data = bytes(b)
        path = str(tmp_path / (f"fz{i}.fq" + (".gz" if i % 3 == 0 else "")))
        with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
            f.write(data)
        files.append((path, data))
    for name, data in (("empty.fq", b""), ("only_header.fq", b"@r1"), ("fasta_crlf.fa",
                       b">a x\r\nACGT\r\nNNAC\r\n>b\r\n\r\nTT\r\n"), ("plus_eof.fq", b"@a\nAC\n+")):
        path = str(tmp_path / name)
        open(path, "wb").write(data)
        files.append((path, data))
    return files


def test_fastx_reader_fixtures_and_fuzz(exe, tmp_path):
    cases = [(os.path.join(GOLD, f), None) for f in ("test.fastq.gz", "test_10.fastq",
                                                      "repeat_40.fq")]
    cases += fuzz_files(tmp_path)
    for path, data in cases:
        if data is None:
            data = O.read_fastx(path)
        for limit in (10**9, 3):
            got = [l for l in run(exe, "fastx", path, limit) if l.startswith("R ")]
            assert got == expect_records(data, limit), (path, limit)


@pytest.mark.parametrize("n", [0, 1, 3, 4, 100, 3079, 3080, 250_000])
def test_khash_replay(exe, n):
    out = run(exe, "khash", n, 11 + n)
    assert out[0].startswith("ok"), out


def test_oracle_index_and_query(exe, tmp_path, testfa):
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b"ACGTacgtNnRYKM-.", np.uint8)
    p = np.array([4, 4, 4, 4, 1, 1, 1, 1, .3, .1, .1, .1, .1, .1, .05, .05])
    seqs = [testfa.encode(), b"ACGTNACG", b"G" * 40, b"A" * 3]
    seqs += [alphabet[rng.choice(alphabet.size, int(rng.integers(2, 5000)), p=p / p.sum())]
             .tobytes() for _ in range(6)]
    for i, s in enumerate(seqs):
        path = str(tmp_path / f"s{i}.txt")
        open(path, "wb").write(s)
        for k in (1, 5, 15, 31, 32):
            if len(s) <= k or (i == 0 and k < 15):      # test.fa at k < 15: ~1e9 query rows
                continue
            got = run(exe, "index", path, k)[0].split()
            oi = O.OracleIndex(s, k)
            kq = min(k, 31)
            rows = oi.query(s, kq) if len(s) > kq else np.empty(0, np.int32)
            want = [oi.U, oi.N, oi.P, oi.max_n, rows.size // 2,
                    wsum(rows) if len(s) > kq else "0" * 16]
            assert got == [str(x) for x in want], (i, k)


def test_read_kmers(exe):
    for f in ("test.fastq.gz", "test_10.fastq", "repeat_40.fq"):
        path = os.path.join(GOLD, f)
        for k, q in ((21, 10), (31, 0), (11, 30)):
            got = run(exe, "reads", path, k, q)[0].split()
            parts = [O.read_kmers(s, qual, k, q) for s, qual in
                     O.fastx_records(O.read_fastx(path)) if len(s) > k]
            km = np.concatenate(parts) if parts else np.empty(0, np.uint64)
            assert got == [str(km.size), wsum(km)], (f, k, q)

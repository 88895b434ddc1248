"""Seeded synthetic sequences for the parity tests and bench.py.

All generators are deterministic functions of their arguments (counter-based splitmix64),
return ``numpy.uint8`` arrays of ASCII bases, and never touch the network or the reference.

  iid(L, seed)                       uniform ACGT, 2 bits per base from splitmix64
  add_n_runs(seq, frac, seed)        N-runs of length 1..100 covering ~frac of the bases
  add_lowercase(seq, frac, seed)     flips ~frac of the bases to lower case
  add_ambiguity(seq, frac, seed)     sprinkles IUPAC codes / '-' / '.' (encoded, not skipped)
  repeat_rich(L, seed)               tandem arrays + interspersed families + N gaps
  config4(L, seed)                   config 4's sequence (repeat_rich tuned into the P band)
  derived(A, seed)                   config 5's B: SNVs, inversions, translocations, N-runs
"""
from __future__ import annotations

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_BASES = np.frombuffer(b"ACGT", np.uint8)


def splitmix64(idx: np.ndarray, seed: int) -> np.ndarray:
    """Counter-based splitmix64: value i = mix(seed + (i+1)*gamma)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _rng(seed: int, salt: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, salt]))


def iid(L: int, seed: int = 1, chunk: int = 1 << 24) -> np.ndarray:
    """L uniform bases; 32 bases per 64-bit splitmix64 draw (2 bits each, MSB first)."""
    out = np.empty(L, np.uint8)
    nwords = (L + 31) // 32
    shifts = np.arange(62, -2, -2, dtype=np.uint64)
    for w0 in range(0, nwords, chunk):
        w1 = min(nwords, w0 + chunk)
        words = splitmix64(np.arange(w0, w1, dtype=np.uint64), seed)
        codes = ((words[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.uint8).reshape(-1)
        b0 = w0 * 32
        n = min(L - b0, codes.size)
        out[b0:b0 + n] = _BASES[codes[:n]]
    return out


def add_n_runs(seq: np.ndarray, frac: float = 0.001, seed: int = 7, max_run: int = 100):
    s = seq.copy()
    L = s.size
    r = _rng(seed, 1)
    n_runs = max(1, int(L * frac / ((1 + max_run) / 2)))
    starts = r.integers(0, L, n_runs)
    lens = r.integers(1, max_run + 1, n_runs)
    for a, b in zip(starts, lens):
        s[a:a + b] = ord("N")
    return s


def add_lowercase(seq: np.ndarray, frac: float = 0.1, seed: int = 11):
    s = seq.copy()
    m = _rng(seed, 2).random(s.size) < frac
    s[m] = s[m] | 0x20
    return s


def add_ambiguity(seq: np.ndarray, frac: float = 0.01, seed: int = 13):
    s = seq.copy()
    codes = np.frombuffer(b"RYKMSWBDHV-.nN", np.uint8)
    r = _rng(seed, 3)
    m = r.random(s.size) < frac
    s[m] = codes[r.integers(0, codes.size, int(m.sum()))]
    return s


def repeat_rich(L: int = 40_000_000, seed: int = 3, tandem_frac: float = 0.05,
                family_frac: float = 0.40, n_gap_every: int = 2_000_000) -> np.ndarray:
    """Config 4: iid background + ~5% tandem arrays (period 2-200) + ~40%
    interspersed families (consensus 300-6,000 bp, 5-500 copies, 0-15% substitutions) +
    100-N scaffold gaps.  Pair count P = sum C(n,2) lands in the 0.5e9-1.5e9 band at 40 Mbp, k=31."""
    r = _rng(seed, 4)
    s = iid(L, seed)
    # interspersed families
    target = int(L * family_frac)
    placed = 0
    while placed < target:
        clen = int(r.integers(300, 6001))
        copies = int(r.integers(5, 501))
        div = float(r.uniform(0.0, 0.15))
        cons = _BASES[r.integers(0, 4, clen)]
        for _ in range(copies):
            if placed >= target:
                break
            c = cons.copy()
            m = r.random(clen) < div
            c[m] = _BASES[r.integers(0, 4, int(m.sum()))]
            a = int(r.integers(0, L - clen))
            s[a:a + clen] = c
            placed += clen
    # tandem arrays
    target = int(L * tandem_frac)
    placed = 0
    while placed < target:
        per = int(r.integers(2, 201))
        alen = int(r.integers(500, 20001))
        unit = _BASES[r.integers(0, 4, per)]
        arr = np.resize(unit, alen)
        m = r.random(alen) < 0.01
        arr[m] = _BASES[r.integers(0, 4, int(m.sum()))]
        a = int(r.integers(0, L - alen))
        s[a:a + alen] = arr
        placed += alen
    for g in range(n_gap_every, L - 100, n_gap_every):
        s[g:g + 100] = ord("N")
    return s


def config4(L: int = 40_000_000, seed: int = 3) -> np.ndarray:
    """BASELINE.json configs[3]: the repeat-rich sequence with the family share raised to 50 %,
    which puts the 40 Mbp, k=31, seed-3 pair count at P = 685,613,382 (max n 14,097), inside
    SURVEY.md §8(d)'s band P in [0.5e9, 1.5e9] (the 40 % default gives 4.75e8)."""
    return repeat_rich(L, seed, family_frac=0.5)


def derived(A: np.ndarray, seed: int = 5, snv: float = 0.01, n_rearr: int = 20,
            n_frac: float = 0.0001) -> np.ndarray:
    """Config 5's query B: A with 1% SNVs, n_rearr inversions/translocations (1-5 Mbp, scaled
    down for short A) and ~0.01% N-runs."""
    r = _rng(seed, 5)
    B = A.copy()
    L = B.size
    m = r.random(L) < snv
    B[m] = _BASES[r.integers(0, 4, int(m.sum()))]
    comp = np.zeros(256, np.uint8)
    for a, b in zip(b"ACGTacgtN", b"TGCAtgcaN"):
        comp[a] = b
    maxlen = max(2, min(5_000_000, L // 50))
    minlen = max(1, min(1_000_000, maxlen // 2))
    for _ in range(n_rearr):
        ln = int(r.integers(minlen, maxlen + 1))
        a = int(r.integers(0, L - ln))
        if r.random() < 0.5:     # inversion (reverse complement in place)
            B[a:a + ln] = comp[B[a:a + ln][::-1]]
        else:                    # translocation: swap with another segment
            b = int(r.integers(0, L - ln))
            tmp = B[a:a + ln].copy()
            B[a:a + ln] = B[b:b + ln]
            B[b:b + ln] = tmp
    if n_frac > 0:
        B = add_n_runs(B, n_frac, seed + 1)
    return B


def reads(genome: np.ndarray, n_reads: int, read_len: int = 150, seed: int = 31,
          err: float = 0.005, n_frac: float = 0.0005, rc_frac: float = 0.5):
    """Short reads sampled from ``genome`` for count.kmers.fq.sh.rp (SURVEY.md §8 f next-4).

    Returns (seq, qual), each (n_reads, read_len) uint8: random start, reverse-complemented with
    probability rc_frac, substitutions at rate err (their qualities drawn low), N calls at rate
    n_frac (quality '#'), and Illumina-like phred+33 qualities ('#'..'J') that decay along the
    read, so the reference's quality filter accepts, rejects and restarts windows."""
    rng = _rng(seed, 17)
    L = len(genome)
    start = rng.integers(0, L - read_len, n_reads)
    idx = start[:, None] + np.arange(read_len)[None, :]
    s = genome[idx].copy()
    flip = rng.random(n_reads) < rc_frac
    comp = np.zeros(256, np.uint8)
    comp[list(b"ACGTNacgtn")] = list(b"TGCANtgcan")
    s[flip] = comp[s[flip][:, ::-1]]
    # qualities: mean decays from Q38 to Q25 along the read, noise +-8, clipped to [2, 41]
    mean = np.linspace(38, 25, read_len)[None, :]
    q = np.clip(np.rint(mean + rng.normal(0, 5, (n_reads, read_len))), 2, 41).astype(np.uint8)
    e = rng.random((n_reads, read_len)) < err
    s[e] = _BASES[rng.integers(0, 4, int(e.sum()))]
    q[e] = rng.integers(2, 15, int(e.sum())).astype(np.uint8)
    nm = rng.random((n_reads, read_len)) < n_frac
    s[nm] = ord("N")
    q[nm] = 2
    return s, (q + 33).astype(np.uint8)


def fastq_bytes(seq: np.ndarray, qual: np.ndarray, prefix: str = "r") -> bytes:
    """4-line FASTQ text of equal-length reads (seq, qual as returned by reads())."""
    n, rl = seq.shape
    names = [f"@{prefix}{i}\n".encode() for i in range(n)]
    body = np.empty((n, 2 * rl + 4), np.uint8)
    body[:, :rl] = seq
    body[:, rl] = 10
    body[:, rl + 1] = ord("+")
    body[:, rl + 2] = 10
    body[:, rl + 3:2 * rl + 3] = qual
    body[:, 2 * rl + 3] = 10
    return b"".join(h + r.tobytes() for h, r in zip(names, body))

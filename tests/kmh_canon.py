"""Canonical forms shared by the golden-vector generator and the parity tests.

The reference's kmer.pos rows follow khash bucket order (reference src/kmer_hash.c:1096-1124),
which is an artefact of its hash table.  Parity is defined on the canonical relabelling
"distinct k-mers ranked by their first position" (SURVEY.md §8c); the GPU engine emits that
order natively, and the khash order itself is pinned separately (orc_khash_order).
"""
import hashlib

import numpy as np


def sha(a) -> str:
    if isinstance(a, (list, tuple)):
        a = "\n".join(a).encode()
    elif isinstance(a, np.ndarray):
        a = np.ascontiguousarray(a).tobytes()
    return hashlib.sha256(a).hexdigest()


def canon_from_raw(raw: dict):
    """raw = kmer_positions(opt=15) output in khash order -> canonical dict + the permutation.

    rank[i_raw-1] = canonical 0-based id.  Positions inside a key are ascending in the
    reference, so a key's first row carries its first position."""
    pos = raw["pos"].reshape(-1, 2)
    cnt = raw["count"]
    U = len(cnt)
    starts = np.zeros(U + 1, np.int64)
    np.cumsum(cnt, out=starts[1:])
    first = pos[starts[:-1], 1] if U else np.empty(0, np.int32)
    order = np.argsort(first, kind="stable")          # canonical id -> raw id (0-based)
    rank = np.empty(U, np.int64)
    rank[order] = np.arange(U)
    out = {}
    out["count"] = cnt[order].astype(np.int32)
    if raw.get("kmer") is not None:
        out["kmer"] = [raw["kmer"][j] for j in order]
    # pos rows grouped by canonical id
    segs = [pos[starts[j]:starts[j + 1], 1] for j in order]
    p = np.concatenate(segs) if segs else np.empty(0, np.int32)
    i = np.repeat(np.arange(1, U + 1, dtype=np.int32), out["count"])
    out["pos"] = np.stack([i, p.astype(np.int32)], 1).reshape(-1)
    if raw.get("pair.pos") is not None:
        pr = raw["pair.pos"].reshape(-1, 3)
        pcnt = cnt.astype(np.int64) * (cnt.astype(np.int64) - 1) // 2
        pst = np.zeros(U + 1, np.int64)
        np.cumsum(pcnt, out=pst[1:])
        if U and pst[-1]:
            idx = np.concatenate([np.arange(pst[j], pst[j + 1]) for j in order])
            q = pr[idx].copy()
            q[:, 0] = np.repeat(np.arange(1, U + 1, dtype=np.int32), pcnt[order])
        else:
            q = np.empty((0, 3), np.int32)
        out["pair.pos"] = q.reshape(-1).astype(np.int32)
    return out, order


class _MemoOracle:
    """An oracle index whose derived outputs are computed once per test session: the parity
    tests run the same inputs through several kernel variants (streams x ranks x radix caps), and
    the CPU oracle -- not the GPU -- dominated their time."""

    def __init__(self, oi):
        self._oi = oi
        self._memo = {}
        self.U, self.N, self.P, self.max_n = oi.U, oi.N, oi.P, oi.max_n
        self.counts = oi.counts

    def _get(self, name, fn):
        if name not in self._memo:
            self._memo[name] = fn()
        return self._memo[name]

    def pos_rows(self):
        return self._get("pos", self._oi.pos_rows)

    def pair_rows(self):
        return self._get("pairs", self._oi.pair_rows)

    def kmer_strings(self):
        return self._get("kmer", self._oi.kmer_strings)

    def query(self, seq, kq):
        qb = seq.encode("latin-1") if isinstance(seq, str) else bytes(seq)
        return self._get(("q", hashlib.sha1(qb).digest(), kq), lambda: self._oi.query(seq, kq))


_ORACLES: dict = {}


def oracle_index(s, k: int, cap: int = 24):
    """OracleIndex(s, k) (oracle/oracle.py), memoised per (sequence, k) for the session."""
    from oracle import oracle as O
    b = s.encode("latin-1") if isinstance(s, str) else bytes(s)
    key = (hashlib.sha1(b).digest(), len(b), k)
    hit = _ORACLES.pop(key, None)
    if hit is None:
        hit = _MemoOracle(O.OracleIndex(s, k))
    _ORACLES[key] = hit                           # most recently used last
    while len(_ORACLES) > cap:
        _ORACLES.pop(next(iter(_ORACLES)))
    return hit

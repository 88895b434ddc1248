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

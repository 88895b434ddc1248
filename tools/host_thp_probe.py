"""Where a fresh host result matrix's time goes, with and without transparent huge pages (THP):
the R API fills a matrix R has just allocated (plain malloc, 4-KB pages unless someone asks for
huge pages) and the previous result is freed by R's collector.  numpy asks for huge pages on
its large arrays itself (madvise(MADV_HUGEPAGE)), so this probe turns that off to stand in for R,
and compares kmhg_query_fill into such an array with and without the library's own hint
(`--no-lib-hint`: the test build with KMHG_D2H_HUGE=0).
    python tools/host_thp_probe.py [calls] [--no-lib-hint]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def _thp_state() -> dict:
    out = {}
    for f in ("enabled", "defrag"):
        try:
            out[f] = open(f"/sys/kernel/mm/transparent_hugepage/{f}").read().strip()
        except OSError as e:
            out[f] = f"unreadable: {e}"
    return out


def _anon_huge_kb() -> int:
    for line in open("/proc/self/smaps_rollup"):
        if line.startswith("AnonHugePages:"):
            return int(line.split()[1])
    return -1


def main():
    import contextlib
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    calls = int(args[0]) if args else 10
    no_hint = "--no-lib-hint" in sys.argv
    if no_hint:
        os.environ["KMHG_D2H_HUGE"] = "0"
    import torch
    assert torch.cuda.is_available()
    from kmer_hasher_amd import _lib
    with (_lib.using_test_build() if no_hint else contextlib.nullcontext()):
        run(calls, no_hint)


def run(calls: int, no_hint: bool):
    try:
        from numpy._core.multiarray import _set_madvise_hugepage
    except ImportError:
        from numpy.core.multiarray import _set_madvise_hugepage
    from kmer_hasher_amd import _lib, api, synth
    seq = synth.iid(10_000_000, 1).tobytes()
    k = 31
    ptr = api.make_kmer_hash(seq, k)
    L = _lib.lib()
    b = api._as_seq_bytes(seq, "x")
    q, h = C.c_void_p(), C.c_int64()
    _lib.check(L.kmhg_query_run(ptr.handle, b, len(b), k, C.byref(q), C.byref(h)))
    H = h.value
    res = {"thp": _thp_state(), "rows": H, "calls": calls, "library_hint": not no_hint}
    for numpy_hint in (True, False):
        _set_madvise_hugepage(numpy_hint)
        fill = rel = 0.0
        huge = []
        prev = np.empty(2 * H, np.int32)
        _lib.check(L.kmhg_query_fill(q, prev.ctypes.data))
        for _ in range(calls):
            rows = np.empty(2 * H, np.int32)
            t0 = time.perf_counter()
            _lib.check(L.kmhg_query_fill(q, rows.ctypes.data))
            t1 = time.perf_counter()
            huge.append(_anon_huge_kb())
            del prev
            t2 = time.perf_counter()
            prev = rows
            fill += t1 - t0
            rel += t2 - t1
        del prev
        res["numpy_hugepage_hint" if numpy_hint else "plain_malloc"] = {
            "fill_ms": round(fill / calls * 1e3, 3), "release_ms": round(rel / calls * 1e3, 3),
            "anon_huge_kb_after_fill": max(huge)}
    L.kmhg_query_free(q)
    ptr.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

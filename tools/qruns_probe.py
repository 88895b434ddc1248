"""A sharded-query sender's range, two ways, on config 5 (500 Mbp index, its derived query,
k = 31): (a) the range query's rows, then encoded as runs (kmhg_query_run_device_range +
kmhg_rows_runs, the path before kmhg_query_run_device_range_runs), (b) the runs made from the
window records without writing rows (kmhg_query_run_device_range_runs).  Each timed from launch to
the runs being ready on the device, min over reps.
    python tools/qruns_probe.py [ranks] [reps]      # the sender's range = the last 1/ranks"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import torch
    assert torch.cuda.is_available()
    from kmer_hasher_amd import synth
    from kmer_hasher_amd.device import DeviceIndex, rows_to_runs
    k, L = 31, 500_000_000
    A = synth.iid(L, 4)
    ta = torch.from_numpy(A).cuda()
    tb = torch.from_numpy(synth.derived(A, 5)).cuda()
    del A
    idx = DeviceIndex.build(ta, k)
    idx.info()
    nw = tb.numel() - k + 1
    w0, w1 = nw - nw // ranks, nw
    res = {"ranks": ranks, "windows": w1 - w0}

    def rows_then_encode():
        rows = idx.query_range(tb, k, w0, w1).rows_view()
        runs = rows_to_runs(rows)
        return rows.shape[0], runs

    def runs_direct():
        kind, t, h = idx.query_range_runs(tb, k, w0, w1)
        return h, (t if kind == "runs" else None)

    for name, fn in (("rows_then_encode", rows_then_encode), ("runs_direct", runs_direct)):
        h, runs = fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h, runs = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = {"ms": round(min(ts) * 1e3, 3), "rows": h,
                     "runs": None if runs is None else int(runs.shape[0])}
        del runs
    a, b = res["rows_then_encode"], res["runs_direct"]
    res["same_counts"] = a["rows"] == b["rows"]
    idx.free()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

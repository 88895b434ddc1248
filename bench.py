"""bench.py -- the headline benchmark of BASELINE.json on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

metric: "Mbp/s indexed (make.kmer.hash k=31) at 1/2/4/8 GPUs; seq.kmer.pos query Mbp/s".
A step is one make.kmer.hash build (kmhg_build_device: radix partition of the windows by hash
bucket, per-bucket LDS tables, totals to a pinned record) of one synthetic sequence already
resident in HBM, and the index is freed again.  kmhg_build_device is asynchronous, so the timed
steps pipeline host enqueue with device execution; `synchronous` reports the same steps with the
host waiting for every build (the R API's make.kmer.hash semantics).  Config 2 (default, BASELINE.json configs[1]): 10 Mbp iid ACGT, k = 31.  The
seq.kmer.pos self-query of the same sequence is timed the same way and reported in `query`;
`counts` times count.kmers of it, `reads` count.kmers.fq.sh.rp of 400 K simulated 150-bp reads
sampled from it (packed in HBM) and `depth` seq.kmer.depth.sh of it against that suffix hash
(SURVEY.md §8 f next-4), each with the reference's own core timed beside it.

N > 1: one rank per GPU.  Launched by torch.distributed.run (WORLD_SIZE must equal --gpus), or
as `python bench.py --gpus N`, which starts the N ranks itself (spawn_ranks) before touching the
GPU.  value = N independent make.kmer.hash builds, every rank indexing its own L-base sequence
(`parallelism: replicas{N}`, no data-path collective, weak scaling): N x L Mbp over the
max-over-ranks time per step.  Two side records carry the sharded paths of SURVEY.md §8e:
`sharded_query` -- north_star's seq.kmer.pos of config 5 (index(A) built on rank 0 and broadcast
once, B's slices scattered from rank 0, range queries, rows gathered to rank 0; phases, and the
rows delivered into a node-shared host matrix as `to_host`) -- and `sharded_build`, the
owner-computes build of ONE N x L sequence (src/kmer_reader.c:28-39's partition) with the
assembly that makes it queryable.

`roofline` prices the dominant build kernel from per-kernel HIP events recorded on the stream
the kernels run on; `traffic` comes from profiles/pmc_<config>.json (rocprofv3 --pmc passes made
by tools/profile.sh) when present.  `cpu_baseline` times the reference's own C core
(oracle/_ref/libkmh_ref.so, 1 thread) on rank 0 over a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    2: dict(workload="configs[1]: synthetic 10 Mbp iid ACGT (splitmix64 seed 1+rank), k=31, "
                     "make.kmer.hash index build; self seq.kmer.pos query timed alongside",
            L=10_000_000, k=31),
    3: dict(workload="configs[2]: synthetic 100 Mbp iid ACGT (splitmix64 seed 2+rank), k=21, "
                     "index build + seq.kmer.pos self-query", L=100_000_000, k=21),
    4: dict(workload="configs[3]: synthetic 40 Mbp repeat-rich (synth.config4 seed 3: "
                     "repeat_rich with 50 % families, P = 6.86e8 in SURVEY §8(d)'s band), k=31, "
                     "kmer.pos(opt.flag=14: pos + pair.pos + count) readout into HBM",
            L=40_000_000, k=31),
    5: dict(workload="configs[4]: two synthetic 500 Mbp sequences (A iid seed 4; B = A + 1% SNV "
                     "+ 20 inversions/translocations + N-runs), k=31, seq.kmer.pos(B vs index(A)) "
                     "with B's windows sharded over the ranks, index broadcast once over RCCL, "
                     "rows gathered to rank 0", L=500_000_000, k=31),
}


# HIP-event labels (kmhg_timing_*) -> the kernel names rocprofv3 reports (template instances in
# full, and the variant a label launches: e.g. k_v2_hist0 runs k_v2_hist0p<true>)
PMC_PREFIX = {"k_v2_scatter_seq": ("k_v2_scatter<true", "k_v2_scatter<false, true"),
              "k_v2_scatter": ("k_v2_scatter<false, false",),
              "k_v2_hist0": ("k_v2_hist0p<", "k_v2_hist0("),
              "k_v2_hist": ("k_v2_histp<", "k_v2_hist<"),
              "k_scan_u32": ("k_scan_lb_u32",),
              "k_v2_bounds": ("k_v2_bounds_lo", "k_v2_bounds"),
              "k_v2_bucket_wg": ("k_v2_bucket_wg<false",),
              "k_query_probe": ("k_query_probe<",),
              "k_read_pairs": ("k_read_pairs",), "k_read_pos": ("k_read_pos",),
              "k_read_keys": ("k_read_keys",)}


def pmc_traffic(pmc: dict, kernel: str):
    """HBM bytes per launch of `kernel` from a profiles/pmc_*.json summary."""
    if kernel in pmc and isinstance(pmc[kernel], dict):
        return pmc[kernel].get("hbm_bytes_per_launch")
    for pre in PMC_PREFIX.get(kernel, ()):
        for name, v in pmc.items():
            if isinstance(v, dict) and (name.startswith(pre) or name + "(" == pre):
                return v.get("hbm_bytes_per_launch")
    return None


BID_MAX_WINDOWS = 12 << 20   # kmhg_engine.cpp build_device_v2: bucket-id streams up to here


def bid_streams(Nw: int) -> bool:
    """Whether a position build of Nw windows runs bucket-id radix streams (the engine's rule;
    only the test build lets KMHG_BUILD_BID force it)."""
    return Nw <= BID_MAX_WINDOWS


def algorithmic_bytes(kernel: str, L: int, Nw: int, U: int, N: int, H: int = 0) -> int | None:
    """Minimal bytes each kernel must move (DESIGN.md "Roofline accounting").  Bucket-id builds
    (bid_streams): V_hist0 writes a 4-B id per window, the first pass reads the ids and writes
    (id, pos), the last pass reads them and writes positions, the bucket kernel reads positions
    and cuts the keys from the code words (0.25 B per window once)."""
    bid = bid_streams(Nw)
    if kernel == "k_v2_hist0" and bid:
        return L + 4 * Nw
    if kernel == "k_v2_scatter_seq":    # read L chars; write (key 8 B, pos 4 B) per valid window
        return 4 * Nw + 8 * N if bid else L + 12 * N
    if kernel == "k_v2_scatter":        # one radix pass: read + write 12 B per window
        return 12 * N if bid else 24 * N
    if kernel in ("k_v2_bucket", "k_v2_bucket_wg", "k_v2_bucket_sort"):   # read 12 B/window; one 16-B slot per distinct key; 4 B per
        rd = 4 * N + Nw // 4 if bid else 12 * N
        return rd + 16 * U + 4 * (N - U)   # position of a repeated key (>= N - U of them)
    if kernel == "k_build_insert":      # read L chars; key+count per distinct key; slot id/window
        return L + 12 * U + 4 * Nw
    if kernel == "k_build_compact":     # key+count read, key+count+offset written per key
        return 12 * U + 16 * U
    if kernel == "k_build_scatter":     # slot id read + position write per window
        return 8 * N
    if kernel == "k_query_probe":       # read L chars; one 16-B slot probe + 4-B record per window
        return L + 20 * Nw
    if kernel == "k_query_emit":        # 4-B window record read + 8-B row write (positions of keys
        return 4 * Nw + 8 * H             # seen once are inline in the record)
    return None


def survey_bytes(kind: str, L: int = 0, U: int = 0, N: int = 0, Nq: int = 0, H: int = 0,
                 P: int = 0, opt: int = 0) -> int:
    """SURVEY.md §8(d) / BASELINE.md §3 algorithmic bytes of one unit of work (one build, one
    query, one readout): the per-unit figures times the units one launch processes.
      build    B = L + 12 U + 4 N           (read chars; key + count/offset per distinct k-mer;
                                             4 B per position)
      query    B = L_q + 12 N_q + 12 H      (read chars; 8-B key + 4-B offset per window; 4 B
                                             position read + 8 B (i, j) row written per hit)
      readout  B = 4U + 4N + 8N[opt&2] + 12P[opt&4] + 4U[opt&8]"""
    if kind == "build":
        return L + 12 * U + 4 * N
    if kind == "query":
        return L + 12 * Nq + 12 * H
    if kind == "readout":
        return (4 * U + 4 * N + (8 * N if opt & 2 else 0) + (12 * P if opt & 4 else 0)
                + (4 * U if opt & 8 else 0))
    raise ValueError(kind)


# HIP-event labels that cover several kernels (one LAUNCH of two kernels), by PMC kernel name
PMC_GROUP = {"k_query_emit": ("k_query_emit", "k_query_emit1"),
             "k_scan_tiles_u64": ("k_scan_tiles_u64", "k_block_sum_u64", "k_block_scan_u64")}


def pmc_step_traffic(pmc: dict, kernels) -> int | None:
    """Summed PMC HBM bytes of one step's kernels (per-launch averages x launches per step)."""
    if not pmc:
        return None
    tot, seen = 0, False
    for name, launches in kernels.items():
        for part in PMC_GROUP.get(name, (name,)):
            t = pmc_traffic(pmc, part)
            if t is not None:
                tot += t * launches
                seen = True
    return tot if seen else None


def roofline(B: int, dom: str, dom_ms: float, step_ms: float, pmc: dict,
             model_bytes: int | None = None, step_kernels: dict | None = None,
             device_ms: float | None = None) -> dict:
    """The contract's roofline object for the dominant kernel of one unit of work:
    achieved = B (SURVEY.md §8(d) bytes of the unit) / the dominant kernel's HIP-event average;
    frac_of_step = B / the whole step's wall time per unit; traffic = PMC HBM bytes per launch
    of the dominant kernel (profiles/pmc_config<c>.json); traffic_step = the summed PMC bytes of
    every kernel of the step; traffic_frac = traffic_step / the step's summed kernel time
    (device_ms) / peak -- the bytes the kernels really moved, so that work avoided (frac well
    above traffic_frac) and HBM efficiency are told apart.  kernel_model prices the dominant
    kernel by the bytes it alone must move (secondary)."""
    ach = B / (dom_ms * 1e-3) / 1e9
    traffic = pmc_traffic(pmc, dom)
    out = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
           "algorithmic_bytes": B, "avg_ms": round(dom_ms, 5),
           "frac_of_step": round(B / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "bytes_source": "SURVEY.md §8(d)"}
    if traffic:
        out["traffic_gbs"] = round(traffic / (dom_ms * 1e-3) / 1e9, 2)
    if step_kernels:
        ts = pmc_step_traffic(pmc, step_kernels)
        if ts:
            out["traffic_step"] = ts
            out["traffic_step_over_B"] = round(ts / B, 3)
            if device_ms:
                out["traffic_frac"] = round(ts / (device_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                out["device_ms"] = round(device_ms, 5)
    if model_bytes:
        ma = model_bytes / (dom_ms * 1e-3) / 1e9
        out["kernel_model"] = {"algorithmic_bytes": model_bytes, "achieved": round(ma, 2),
                               "frac": round(ma / HBM_PEAK_GBS, 4),
                               "note": "bytes the dominant kernel alone must move (bench.py "
                                       "algorithmic_bytes)"}
    return out


def host_info() -> dict:
    """nproc / CPU model of the host the CPU baseline runs on."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model}


def query_roofline(qper: dict, L: int, Nw: int, H: int, pmc: dict, step_ms: float,
                   launches: dict | None = None) -> dict | None:
    """Roofline of the query: SURVEY.md §8(d)'s query bytes over the summed HIP-event averages of
    the query's kernels (probe, scan, emit); the dominant kernel's own time, PMC traffic and
    kernel_model ride along."""
    if not qper:
        return None
    dom = max(qper, key=qper.get)
    B = survey_bytes("query", L=L, Nq=Nw, H=H)
    # (no kernel_model: the diagonal path avoids most of the probe's modelled bytes -- a self dot
    # plot's probe moved 50 MB against a 210 MB model -- so a model-bytes "frac" would report work
    # avoided as bandwidth; traffic_frac below prices the bytes really moved)
    out = roofline(B, dom, qper[dom], step_ms, pmc, None, launches or {n: 1 for n in qper},
                   device_ms=sum(qper.values()))
    # §8(d)'s query bytes belong to the probe and the emit together (round 4: with the emit at
    # ~5 TB/s the probe alone is the larger kernel, and B over the probe's time alone exceeded
    # the peak), so `achieved` prices them over the query's kernels together
    dev_ms = sum(qper.values())
    ach = B / (dev_ms * 1e-3) / 1e9
    out.update({"kernel": "+".join(sorted(qper)), "dominant_kernel": dom,
                "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 4),
                "avg_ms": round(dev_ms, 5), "dominant_ms": round(qper[dom], 5)})
    if out.get("traffic"):
        out["traffic_gbs"] = round(out["traffic"] / (qper[dom] * 1e-3) / 1e9, 2)
    out["note"] = ("achieved = SURVEY.md §8(d)'s query bytes over the summed HIP-event times of "
                   "the query's kernels (probe, scan, emit); traffic / traffic_gbs are the "
                   "dominant kernel's PMC bytes, traffic_frac the PMC bytes of every query kernel "
                   "over their summed time.  A self dot plot resolves most windows on the "
                   "diagonal against the index's code words, so the probe moves fewer bytes than "
                   "12 per window: frac above traffic_frac is work avoided, not bandwidth")
    return out


def host_boundary(seq_bytes: bytes, k: int, calls: int = 10) -> dict:
    """The R-API rate: make.kmer.hash / seq.kmer.pos through the host-pointer C-ABI entries
    (kmhg_build: pageable host sequence -> H2D -> build -> synchronize; kmhg_query_run +
    kmhg_query_fill: H2D -> query -> rows D2H into host memory), i.e. PCIe-inclusive.  Reported
    beside `value`, never as it."""
    from kmer_hasher_amd import api
    api.make_kmer_hash(seq_bytes, k).free()            # first call: pool, code objects
    t0 = time.perf_counter()
    for _ in range(calls):
        api.make_kmer_hash(seq_bytes, k).free()
    t_b = (time.perf_counter() - t0) / calls
    ptr = api.make_kmer_hash(seq_bytes, k)
    rows = api.seq_kmer_pos(ptr, seq_bytes, k)
    t0 = time.perf_counter()
    for _ in range(calls):
        rows = api.seq_kmer_pos(ptr, seq_bytes, k)
    t_q = (time.perf_counter() - t0) / calls
    # the query's legs: kmhg_query_run (sequence H2D + the device query, synchronous), then
    # kmhg_query_fill into a fresh array (R's allocMatrix: its pages are faulted in by the copy)
    # and into an array already touched (the DMA + copy alone)
    import ctypes as C
    import numpy as np
    from kmer_hasher_amd import _lib
    L = _lib.lib()
    t_run = t_fresh = t_warm = t_rel = 0.0
    warm = np.ones(2 * rows.shape[0], np.int32)
    for _ in range(calls):
        q, h = C.c_void_p(), C.c_int64()
        t0 = time.perf_counter()
        _lib.check(L.kmhg_query_run(ptr.handle, seq_bytes, len(seq_bytes), k, C.byref(q),
                                    C.byref(h)))
        t1 = time.perf_counter()
        fresh = np.empty(2 * h.value, np.int32)
        _lib.check(L.kmhg_query_fill(q, fresh.ctypes.data))
        t2 = time.perf_counter()
        _lib.check(L.kmhg_query_fill(q, warm.ctypes.data))
        t3 = time.perf_counter()
        L.kmhg_query_free(q)
        t_run += t1 - t0
        t_fresh += t2 - t1
        t_warm += t3 - t2
        t4 = time.perf_counter()
        del fresh                         # the host returns the result's pages (munmap)
        t_rel += time.perf_counter() - t4
    ptr.free()
    mbp = len(seq_bytes) / 1e6
    return {"build": {"value": round(mbp / t_b, 2), "unit": "Mbp/s", "ms": round(t_b * 1e3, 3)},
            "query": {"value": round(mbp / t_q, 2), "unit": "Mbp/s", "ms": round(t_q * 1e3, 3),
                      "rows": int(rows.shape[0]),
                      "legs_ms": {"h2d_and_device_query": round(t_run / calls * 1e3, 3),
                                  "rows_to_fresh_array": round(t_fresh / calls * 1e3, 3),
                                  "rows_to_touched_array": round(t_warm / calls * 1e3, 3),
                                  "page_faults": round((t_fresh - t_warm) / calls * 1e3, 3),
                                  "result_release": round(t_rel / calls * 1e3, 3),
                                  "note": "fresh = a new array whose pages the copy faults in "
                                          "(as R's allocMatrix); touched = the same copy into "
                                          "resident pages (DMA + host copy only); "
                                          "result_release = freeing the previous call's 2 x H "
                                          "int32 result (the host unmapping its pages: R's GC "
                                          "pays the same for its matrix), part of `ms` because "
                                          "each call's result replaces the last"}},
            "calls": calls,
            "note": "PCIe-inclusive: host sequence in (pageable), host rows out, synchronous "
                    "per call (the R API); not `value`"}


class _pinned_one_core:
    """Pin this process to one of its allowed CPUs for a CPU-baseline leg (taskset -c, as
    BASELINE.md §3 asks), restoring the previous affinity afterwards."""

    def __enter__(self):
        try:
            self.prev = os.sched_getaffinity(0)
            os.sched_setaffinity(0, {min(self.prev)})
        except (AttributeError, OSError):
            self.prev = None
        return self

    def __exit__(self, *exc):
        if self.prev:
            os.sched_setaffinity(0, self.prev)


def cpu_baseline(seq_bytes: bytes, k: int, sample_bp: int = 10_000_000, reps_max: int = 3,
                 budget_s: float = 20.0) -> dict | None:
    """Reference C core (compiled from the reference's own sources into oracle/_ref) timed on
    the host, single-threaded and pinned to one core, on a prefix sample of the workload: build
    (seq_to_hash) and self query (seq_kmer_positions) timed separately, teardown (clear_kmer_h,
    the finaliser) on its own line."""
    try:
        from oracle import oracle as O
        if not O.ref_available():
            return None
        sample = seq_bytes[: min(len(seq_bytes), sample_bp)]
        t_build, t_query, t_free, reps, n = 0.0, 0.0, 0.0, 0, 0
        t_start = time.perf_counter()
        with _pinned_one_core():
            while time.perf_counter() - t_start < budget_s / 2 or reps == 0:
                t0 = time.perf_counter()
                r = O.RefIndex(sample, k)
                t1 = time.perf_counter()
                q = r.query(sample, k)
                t2 = time.perf_counter()
                n = q.size // 2
                del q
                t3 = time.perf_counter()
                r.close()
                t_free += time.perf_counter() - t3
                t_build += t1 - t0
                t_query += t2 - t1
                reps += 1
                if reps >= reps_max:
                    break
        mbp = len(sample) / 1e6
        whole = len(sample) == len(seq_bytes)
        return {"value": round(mbp * reps / t_build, 3), "unit": "Mbp/s", "cores": 1,
                "kind": "reference",
                "sample": (f"the whole {mbp:.1f} Mbp sequence" if whole else
                           f"{mbp:.1f} Mbp prefix of the same sequence") +
                          f", k={k}, {reps} build(s) of src/kmer_pos.c seq_to_hash + "
                          "seq_kmer_positions via oracle/_ref (gcc -O2, 1 thread pinned)",
                "build_s": round(t_build / reps, 3),
                "query_value": round(mbp * reps / t_query, 3), "query_s": round(t_query / reps, 3),
                "query_rows": n, "teardown_s": round(t_free / reps, 3), "host": host_info()}
    except Exception as e:  # the baseline is reported, never required
        return {"value": None, "unit": "Mbp/s", "cores": 1, "kind": "reference",
                "sample": f"unavailable: {e}"}


def cpu_counts_baseline(seq_bytes: bytes, k: int, sample_bp: int = 3_000_000) -> dict:
    """count_kmers (src/kmer_hash.c:548-591: seq_to_counts over the reference's khash core,
    oracle/_ref) on a bounded prefix of the same sequence, 1 thread."""
    try:
        from oracle import oracle as O
        sample = seq_bytes[:sample_bp]
        t0 = time.perf_counter()
        r = O.RefIndex.counts([sample], k, 0, 2)
        t = time.perf_counter() - t0
        r.close()
        return {"value": round(len(sample) / 1e6 / t, 3), "unit": "Mbp/s", "cores": 1,
                "kind": "reference",
                "sample": f"{len(sample) / 1e6:.1f} Mbp prefix, k={k}, count_kmers(source 0 of 2) "
                          "restated over the compiled khash core (oracle/_ref, gcc -O2)"}
    except Exception as e:  # reported, never required
        return {"value": None, "unit": "Mbp/s", "cores": 1, "kind": "reference",
                "sample": f"unavailable: {e}"}


# the reference's own usage (test.R:146): count.kmers.fq.sh.rp(fq, c(31, 28, 10, 47, -1, 200, 2, 0))
READS_N, READS_LEN, READS_MINQ, READS_CPU = 400_000, 150, 10, 40_000


def reads_algorithmic_bytes(kernel: str, n_bases: int, n_reads: int, words: int) -> int | None:
    """Minimum bytes of the read-counting iterator (one walk): every base and quality read once
    (2 B/base), its read's offset (8 B) and output offset (4 B), and 8 B written per accepted
    k-mer (`words`, the k-mer occurrences counted; the EMPTY_KEY padding of rejected windows is
    not counted)."""
    if kernel == "k_read_kmers_emit":
        return 2 * n_bases + 12 * n_reads + 8 * words
    return None


def counts_algorithmic_bytes(kernel: str, L: int, U: int, S: int, nslots: int = 0) -> int | None:
    """Minimum bytes of the count.kmers kernels (first batch into a new pointer): C_walk reads
    every slot of the adopted table (16 B) and, per key, writes its row (key 8 B, S counts,
    row_slot 4 B, order key 8 B), slot_row (4 B) and the slot's count fields (8 B)."""
    if kernel in ("k_count_walk", "k_count_walk_b"):
        return 16 * nslots + U * (8 + 4 * S + 4 + 8 + 4 + 8)
    return None


def depth_algorithmic_bytes(kernel: str, L: int, S: int) -> int | None:
    """k_depth_probe: every base read once and one 16-B slot probe per window, S int32 out per
    base."""
    if kernel == "k_depth_probe":
        return L + 16 * L + 4 * S * L
    return None


def _leg_roofline(per: dict, kernel: str, ab) -> dict:
    ach = ab / (per[kernel] * 1e-3) / 1e9 if ab else None
    return {"bound": "hbm", "kernel": kernel, "achieved": round(ach, 2) if ach else None,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None, "algorithmic_bytes": ab,
            "avg_ms": round(per[kernel], 5)}


def cpu_reads_baseline(fq: bytes, seq_bytes: bytes, k: int, depth_bp: int = 2_000_000):
    """count_kmers_fastq_sh_rp (src/kmer_hash.c:810-857, 1 reader thread) and seq_kmer_counts
    (src/kmer_reader.c:155-193) of the reference's own counting core (oracle/_ref) on a bounded
    sample: the first READS_CPU reads written as FASTQ, and a depth_bp prefix."""
    try:
        import tempfile
        from oracle import oracle as O
        with tempfile.NamedTemporaryFile(suffix=".fq") as f:
            f.write(fq)
            f.flush()
            r = O.RefSH()
            t0 = time.perf_counter()
            r.add_fastq(f.name, k, 28, READS_MINQ, 2**62, 2, 0)
            t = time.perf_counter() - t0
        bases = READS_CPU * READS_LEN
        rb = {"value": round(bases / 1e6 / t, 3), "unit": "Mbp/s", "cores": 1,
              "kind": "reference",
              "sample": f"{READS_CPU} reads x {READS_LEN} bp ({bases / 1e6:.1f} Mbp) from a FASTQ "
                        "file, count_kmers_fastq_sh_rp core (kmer_reader_read, 1 thread, "
                        "oracle/_ref gcc -O2)"}
        s = seq_bytes[:depth_bp]
        t0 = time.perf_counter()
        r.depth(s, k)
        t = time.perf_counter() - t0
        r.close()
        db = {"value": round(len(s) / 1e6 / t, 3), "unit": "Mbp/s", "cores": 1,
              "kind": "reference",
              "sample": f"{len(s) / 1e6:.1f} Mbp prefix, seq_kmer_counts against the suffix hash "
                        "of the sample reads (oracle/_ref)"}
        return rb, db
    except Exception as e:  # reported, never required
        na = {"value": None, "unit": "Mbp/s", "cores": 1, "kind": "reference",
              "sample": f"unavailable: {e}"}
        return na, dict(na)


_JSON_OUT = sys.stdout        # the result line's stream (main() keeps the process's real stdout)


def _claim_stdout() -> None:
    """Stdout carries the one JSON line and nothing else: from here on, what anything else prints
    there (RCCL's version banner at process-group init, runtime notices) goes to stderr."""
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def check_world(gpus: int, world_env: str | None) -> None:
    """A launcher's WORLD_SIZE must equal --gpus: n_gpus in the line is the ranks that ran."""
    if world_env is not None and int(world_env) != gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world_env} but --gpus {gpus}: launch one rank per "
                         "GPU (--nproc-per-node N) with --gpus N")


def rank_command(gpus: int, argv: list[str], port: int) -> list[str]:
    """The torch.distributed.run command that starts `gpus` ranks of this script (one process
    per GPU, rendezvous on 127.0.0.1) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def spawn_ranks(gpus: int, argv: list[str] | None = None) -> int:
    """Run the N ranks as a child process group and return its exit status.  The parent has not
    initialised the GPU (no torch import), so nothing here replaces a process that holds it; the
    ranks' stdout is this process's stdout (rank 0 prints the one JSON line)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    sys.stdout.flush()
    return subprocess.call(rank_command(gpus, sys.argv[1:] if argv is None else argv, port),
                           env=env)


def launch_check(args) -> None:
    """--launch-check: the rank launch and world check alone (tests/test_bench_launch.py), over
    gloo on the CPU: every rank joins the group and asserts its size, rank 0 prints one line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")
        t = torch.ones(1)
        dist.all_reduce(t)
        world = int(t.item())
    if int(os.environ.get("RANK", "0")) == 0:
        _emit({"metric": "launch-check", "n_gpus": world, "pid_parent": os.getppid()})
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-reads", action="store_true",
                    help="skip the read-counting / depth legs (count.kmers.fq.sh.rp)")
    ap.add_argument("--profile", action="store_true",
                    help="short run for rocprofv3 (no CPU leg, no JSON extras)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 process group (nccl = RCCL; gloo only to rehearse the N > 1 "
                         "code on one GPU)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 rehearsal on a one-GPU box: every rank on cuda:0 (with gloo)")
    ap.add_argument("--dist", action="store_true",
                    help="take the N > 1 code path (process group over --backend, owner-computes "
                         "build, assembly) even at world size 1: the RCCL rehearsal on a one-GPU "
                         "box (python -m torch.distributed.run --nproc-per-node 1 bench.py --dist)")
    ap.add_argument("--no-large", action="store_true",
                    help="skip the out-of-cache side record (500 Mbp build + cross query)")
    ap.add_argument("--only-large", action="store_true",
                    help="run the out-of-cache record alone (profiling), printed as its own line")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU test of the rank launch: gloo process group, no GPU, one line")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without a launcher: start the N ranks here, before this
        # process touches the GPU (it never does: it only waits for its child)
        raise SystemExit(spawn_ranks(args.gpus))
    check_world(args.gpus, os.environ.get("WORLD_SIZE"))
    _claim_stdout()
    if args.launch_check:
        return launch_check(args)
    # the side legs (query, counts, reads, depth) run for at least 50 timed calls: 20 calls of a
    # 0.1-0.5 ms leg are a few ms of wall time, where one host hiccup shows as a 2x swing
    leg_steps = max(args.steps, 50)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1 or args.dist
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.rehearse:
            local = 0
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from kmer_hasher_amd import _lib
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth

    cfg = CONFIGS[args.config]
    L, k = cfg["L"], cfg["k"]
    if args.only_large:
        rec = bench_large(args, dev)
        if rank == 0:
            _emit({"metric": "out-of-cache build + cross query (config 5 workload, one GPU)",
                   **rec})
        return
    if args.config in (4, 5):
        (bench_readout if args.config == 4 else bench_sharded_query)(args, cfg, dev, world, rank)
        if distributed:
            dist.barrier()
            dist.destroy_process_group()
        return
    seed = (1 if args.config == 2 else 2) + rank
    host_seq = synth.iid(L, seed)
    seq = torch.from_numpy(host_seq).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def barrier():
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    def build_step(wait=False):
        # kmhg_build_device is asynchronous: back-to-back steps pipeline the host's enqueue of
        # step i+1 with the device's execution of step i; every step runs the whole build
        idx = D.DeviceIndex.build(seq, k, stream)
        info = idx.info() if wait else None        # info() waits for the build
        idx.free()
        if info is not None:
            check_build(info)
        return info

    progress("build steps")
    # ---------------- build: W untimed warmups, 2 steps with events around every kernel (find the
    # dominant one), then exactly K timed steps with events around the dominant kernel only, so
    # the per-kernel events add no dead time to the rest of the timed region
    for _ in range(args.warmup):
        info = build_step(wait=True)
    # the same steps with a wait after each (the synchronous make.kmer.hash of the R API)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        info = build_step(wait=True)
    barrier()
    t_sync = time.perf_counter() - t0
    D.timing_enable(True)
    D.timing_select(None)
    D.timing_reset()
    n_id = 2
    for _ in range(n_id):
        info = build_step(wait=True)
    wt = D.timing_report()
    all_kernels = {n: v[1] / v[0] for n, v in wt.items() if v[0]}
    per_step = {n: v[1] / n_id for n, v in wt.items() if v[0]}
    dom = max(per_step, key=per_step.get)
    D.timing_select(dom)
    D.timing_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        build_step()
    barrier()
    t_build = time.perf_counter() - t0
    info = build_step(wait=True)                   # totals of one more (waited) build
    ktimes = D.timing_report()
    D.timing_enable(False)
    D.timing_select(None)

    # ---------------- N > 1: the headline is the owner-computes build of ONE genome of N x L
    # bases: rank 0 holds it and broadcasts it, every rank builds the k-mers of
    # its bucket range (kmhg_build_device_part); assembling the whole index on every rank is timed
    # once, apart.  The replicas above (every rank its own L bases) become a side record.
    sharded = None
    if distributed:
        sharded = _side_record("sharded build", bench_sharded_build, args, k, L, dev, world,
                               rank, seed)

    progress("self query")
    # ---------------- query: self seq.kmer.pos against one resident index.  The first query of an
    # index also derives the diagonal path's unique-window bits and slot tags (k_diag_valid /
    # k_diag_prep, kept with the index): timed on its own as first_call_ms.
    idx = D.DeviceIndex.build(seq, k, stream)
    idx.info()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = idx.query(seq, k, stream)
    H = q.n_rows
    q.free()
    torch.cuda.synchronize()
    t_query_first = time.perf_counter() - t0
    # ... and the first query of a second index, once the process has loaded those kernels:
    # what every later index's first seq.kmer.pos costs (the R user's query-once case)
    idx2 = D.DeviceIndex.build(seq, k, stream)
    idx2.info()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = idx2.query(seq, k, stream)
    q.free()
    torch.cuda.synchronize()
    t_query_first2 = time.perf_counter() - t0
    idx2.free()
    for _ in range(max(1, args.warmup)):
        q = idx.query(seq, k, stream)
        H = q.n_rows
        q.free()
    D.timing_enable(True)
    D.timing_reset()
    for _ in range(2):
        q = idx.query(seq, k, stream)
        q.free()
    qt = D.timing_report()
    qper = {n: v[1] / v[0] for n, v in qt.items() if v[0]}
    D.timing_enable(False)
    barrier()
    t0 = time.perf_counter()
    for _ in range(leg_steps):
        q = idx.query(seq, k, stream)
        q.free()
    barrier()
    t_query = time.perf_counter() - t0
    # the same index queried with an unrelated sequence of the same length (seed + 100): almost
    # every window misses, so the diagonal path's anchors predict nothing and every window
    # probes the table -- the path's worst case, reported beside the self dot plot
    H_other, t_other, oper = 0, 0.0, {}
    if not args.profile:        # (the profile's per-kernel PMC averages stay self-query only)
        other = torch.from_numpy(synth.iid(L, seed + 100)).to(dev)
        n_other = leg_steps         # >= 50 calls, like the other legs (0.2 ms each)
        q = idx.query(other, k, stream)
        q.free()
        D.timing_enable(True)
        D.timing_reset()
        for _ in range(2):
            idx.query(other, k, stream).free()
        oper = {n: v[1] / v[0] for n, v in D.timing_report().items() if v[0]}
        D.timing_enable(False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(n_other):
            q = idx.query(other, k, stream)
            H_other = q.n_rows
            q.free()
        barrier()
        t_other = (time.perf_counter() - t0) / n_other
        del other
    # teardown (the finaliser, src/kmer_hash.c:56-66; the reference's takes 2.56 s at 10 Mbp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx.free()
    torch.cuda.synchronize()
    t_free = time.perf_counter() - t0

    progress("counts / reads / depth legs")
    # ---------------- count.kmers (SURVEY.md §8 f next-4) of the same sequence: one call per step
    # into a new counts pointer (k, source 0 of 2)
    cper, t_count, cU, cslots, t_order, order_k = {}, 0.0, 0, 0, 0.0, {}
    if not args.profile:
        for _ in range(max(1, args.warmup)):
            D.DeviceIndex.count(seq, k, 0, 2, stream=stream).free()
        D.timing_enable(True)
        D.timing_reset()
        for _ in range(2):
            c = D.DeviceIndex.count(seq, k, 0, 2, stream=stream)
            ci = c.info()
            cU, cslots = ci["n_kmers"], ci["table_slots"]
            c.free()
        ct = D.timing_report()
        cper = {n: v[1] / 2 for n, v in ct.items() if v[0]}
        D.timing_enable(False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(leg_steps):
            D.DeviceIndex.count(seq, k, 0, 2, stream=stream).free()
        barrier()
        t_count = time.perf_counter() - t0
        # the rows' first-insertion order is restored once, when a readout first asks for rows
        # (ensure_row_order): timed here on its own (kmhg_counts_export with no output copies)
        c = D.DeviceIndex.count(seq, k, 0, 2, stream=stream)
        torch.cuda.synchronize()
        D.timing_enable(True)
        D.timing_reset()
        t0 = time.perf_counter()
        _lib.check(_lib.lib().kmhg_counts_export(c.handle, None, None))
        t_order = time.perf_counter() - t0
        order_k = {n: v[1] for n, v in D.timing_report().items() if v[0]}
        D.timing_enable(False)
        c.free()

    # ---------------- count.kmers.fq.sh.rp over reads sampled from the same sequence (packed reads
    # resident in HBM, one new suffix hash per step), then seq.kmer.depth.sh of the sequence
    # against it (SURVEY.md §8 f next-4)
    rper, dper, t_reads, t_depth, rU, n_bases, sample_fq = {}, {}, 0.0, 0.0, 0, 0, None
    t_reads_first = 0.0
    r_words = 0
    if not args.profile and not args.no_reads:
        rs, rq = synth.reads(host_seq, READS_N, READS_LEN, 51 + rank)
        reads = D.DeviceReads.from_arrays(rs, rq, dev)
        n_bases = READS_N * READS_LEN
        if rank == 0 and not args.no_cpu:
            sample_fq = synth.fastq_bytes(rs[:READS_CPU], rq[:READS_CPU])
        del rs, rq
        prm = (k, 28, READS_MINQ, 47, -1, 200, 2, 0)
        # the first call of the process (one-time allocations and uploads included): the batch
        # chooses its bucket spread from its own HLL estimate, so no earlier call is needed
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.DeviceIndex.count_reads(reads, prm, stream=stream).free()
        torch.cuda.synchronize()
        t_reads_first = time.perf_counter() - t0
        for _ in range(max(1, args.warmup)):
            D.DeviceIndex.count_reads(reads, prm, stream=stream).free()
        D.timing_enable(True)
        D.timing_reset()
        for _ in range(2):
            c = D.DeviceIndex.count_reads(reads, prm, stream=stream)
            rU = c.info()["n_kmers"]
            c.free()
        rper = {n: v[1] / 2 for n, v in D.timing_report().items() if v[0]}
        D.timing_enable(False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(leg_steps):
            D.DeviceIndex.count_reads(reads, prm, stream=stream).free()
        barrier()
        t_reads = time.perf_counter() - t0
        sh = D.DeviceIndex.count_reads(reads, prm, stream=stream)
        dout = torch.empty((L, 2), dtype=torch.int32, device=dev)
        for _ in range(max(1, args.warmup)):
            sh.depth(seq, k, dout, stream=stream)
        D.timing_enable(True)
        D.timing_reset()
        for _ in range(2):
            sh.depth(seq, k, dout, stream=stream)
        dper = {n: v[1] / 2 for n, v in D.timing_report().items() if v[0]}
        D.timing_enable(False)
        barrier()
        t0 = time.perf_counter()
        for _ in range(leg_steps):
            sh.depth(seq, k, dout, stream=stream)
        barrier()
        t_depth = time.perf_counter() - t0
        import ctypes as _C
        import numpy as np
        from kmer_hasher_amd import _lib
        _inf = sh.info()
        _M = np.zeros(_inf["n_kmers"] * _inf["sources"], np.int32)
        _lib.check(_lib.lib().kmhg_counts_export(sh.handle, None, _C.c_void_p(_M.ctypes.data)))
        r_words = int(_M.astype(np.int64).sum())      # k-mer occurrences counted per step
        sh.free()
        del reads, dout

    tb = torch.tensor([t_build, t_query, t_sync, t_count, t_reads, t_depth], dtype=torch.float64,
                      device=dev)
    if distributed:
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
    progress("sharded records")
    # north_star's sharded seq.kmer.pos (config 5: index broadcast once, B scattered, range
    # queries, rows gathered) on every N > 1 line; at N = 1 `large.query` is its one-GPU point
    sq = None
    if distributed and not args.profile and not args.no_large:
        sq = _side_record("sharded query", lambda *a: sharded_query_record(*a)[0], args, dev,
                          world, rank, max(1, min(args.steps, 10)))
    progress("out-of-cache record")
    # the out-of-cache side record (one GPU only: the driver's N = 1 line; the 8-GPU scaling runs
    # skip it)
    large = None
    if world == 1 and not args.dist and not args.profile and not args.no_large \
            and args.config == 2:
        large = bench_large(args, dev)
    t_build, t_query, t_sync, t_count, t_reads, t_depth = tb.tolist()

    if rank == 0:
        Nw = L - k + 1
        U, N = info["n_kmers"], info["n_positions"]
        mbp_total = L * world / 1e6
        value = mbp_total * args.steps / t_build
        qvalue = mbp_total * leg_steps / t_query
        # dominant build kernel (largest time per step in the warm-up) and its roofline from
        # the HIP events recorded around it in the timed steps
        per = all_kernels
        tot = per_step
        dom_ms = ktimes[dom][1] / ktimes[dom][0] if ktimes.get(dom, [0])[0] else per[dom]
        pmc = {}
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{args.config}.json")
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
            except Exception:
                pmc = {}
        step_ms = t_build / args.steps * 1e3
        launches = {n: v[0] / n_id for n, v in wt.items() if v[0]}
        B = survey_bytes("build", L=L, U=U, N=N)
        out = {
            "metric": "Mbp/s indexed (make.kmer.hash k=31) at 1/2/4/8 GPUs; "
                      "seq.kmer.pos query Mbp/s",
            "value": round(value, 2),
            "unit": "Mbp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_build / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": cfg["workload"], "seq_len": L, "k": k,
                       "distinct_kmers": U, "positions": N, "parallelism": f"replicas{world}"},
            "roofline": roofline(B, dom, dom_ms, step_ms, pmc,
                                 algorithmic_bytes(dom, L, Nw, U, N), launches,
                                 device_ms=sum(per_step.values())),
            "synchronous": {"value": round(mbp_total * args.steps / t_sync, 2), "unit": "Mbp/s",
                            "ms_per_step": round(t_sync / args.steps * 1e3, 4),
                            "note": "same steps, host waits for each build (R-API semantics)"},
            "query": {"value": round(qvalue, 2), "unit": "Mbp/s", "rows": H,
                      "ms_per_step": round(t_query / leg_steps * 1e3, 4),
                      "first_call_ms": round(t_query_first * 1e3, 3),
                      "first_query_new_index_ms": round(t_query_first2 * 1e3, 3),
                      "kernels_ms": {n: round(v, 5) for n, v in qper.items()},
                      "roofline": query_roofline(qper, L, Nw, H, pmc,
                                                 t_query / leg_steps * 1e3),
                      "unrelated": {"value": round(L * world / 1e6 / t_other, 2) if t_other
                                    else None, "unit": "Mbp/s",
                                    "ms_per_step": round(t_other * 1e3, 4), "rows": H_other,
                                    "steps": leg_steps,
                                    "kernels_ms": {n: round(v, 5) for n, v in oper.items()},
                                    "roofline": query_roofline(
                                        oper, L, Nw, H_other, _load_pmc("unrelated"),
                                        t_other * 1e3) if oper else None,
                                    "note": "index queried with an unrelated iid sequence "
                                            "(seed + 100): every window probes the table (the "
                                            "general lookup); PMC from "
                                            "profiles/pmc_configunrelated.json"},
                      "note": "self dot plot (the bench sequence against its own index): the "
                              "diagonal path's best case; first_call_ms is the first query of "
                              "the process (the index's one-time diagonal-path preparation -- "
                              "window bits; the slot tags come with the build -- and the first "
                              "launch of those kernels), first_query_new_index_ms the first "
                              "query of a second index"},
            "kernels_ms": {n: round(v, 5) for n, v in per.items()},
            "kernel_ms_per_step": round(sum(tot.values()), 5),
            "teardown_ms": round(t_free * 1e3, 4),
        }
        if t_count:
            out["counts"] = {
                "value": round(mbp_total * leg_steps / t_count, 2), "unit": "Mbp/s",
                "ms_per_step": round(t_count / leg_steps * 1e3, 4), "distinct_kmers": cU,
                "kernels_ms_per_step": {n: round(v, 5) for n, v in cper.items()},
                "first_readout_row_order": {
                    "ms": round(t_order * 1e3, 4),
                    "kernels_ms": {n: round(v, 5) for n, v in order_k.items()},
                    "note": "once per counts pointer (and again after a later batch), when a "
                            "readout first asks for rows: the rows' first-insertion order derived "
                            "from their order keys (k_rows_place / k_rows_order)"},
                "note": "count.kmers(seq, c(k, 0, 2)) into a new pointer per step: partitioned "
                        "build of the batch, whose table the new pointer adopts, its rows "
                        "written in slot order with their insertion-order keys (k_count_walk); "
                        "first_readout_row_order is the one-time ordering a readout triggers"}
            cdom = max((n for n in cper if n.startswith("k_count_")), key=cper.get, default=None)
            if cdom:
                out["counts"]["roofline"] = _leg_roofline(
                    cper, cdom, counts_algorithmic_bytes(cdom, L, cU, 2, cslots))
        if t_reads:
            dom_r = "k_read_kmers_emit"      # the row's own kernel (the batch build is the index's)
            ab_r = reads_algorithmic_bytes(dom_r, n_bases, READS_N, r_words)
            out["reads"] = {
                "value": round(n_bases * world / 1e6 * leg_steps / t_reads, 2), "unit": "Mbp/s",
                "ms_per_step": round(t_reads / leg_steps * 1e3, 4), "reads": READS_N,
                "read_len": READS_LEN, "k": k, "min_q": READS_MINQ, "distinct_kmers": rU,
                "kmer_words": r_words,
                "first_call": {"value": round(n_bases / 1e6 / t_reads_first, 2), "unit": "Mbp/s",
                               "ms": round(t_reads_first * 1e3, 3),
                               "note": "the process's first count.kmers.fq.sh.rp call, one-time "
                                       "allocations included"},
                "kernels_ms_per_step": {n: round(v, 5) for n, v in rper.items()},
                "roofline": {"bound": "hbm", "kernel": dom_r,
                             "achieved": round(ab_r / (rper[dom_r] * 1e-3) / 1e9, 2)
                             if ab_r else None,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ab_r / (rper[dom_r] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                             if ab_r else None, "algorithmic_bytes": ab_r},
                "note": "count.kmers.fq.sh.rp(c(k, 28, min_q, 47, -1, 200, 2, 0)) of reads sampled "
                        "from the bench sequence (synth.reads: 150 bp, decaying phred, 0.5% "
                        "substitutions), packed in HBM, a new suffix hash per step"}
            out["depth"] = {
                "value": round(L * world / 1e6 * leg_steps / t_depth, 2), "unit": "Mbp/s",
                "ms_per_step": round(t_depth / leg_steps * 1e3, 4),
                "kernels_ms_per_step": {n: round(v, 5) for n, v in dper.items()},
                "note": "seq.kmer.depth.sh of the bench sequence against that suffix hash"}
            if "k_depth_probe" in dper:
                out["depth"]["roofline"] = _leg_roofline(
                    dper, "k_depth_probe", depth_algorithmic_bytes("k_depth_probe", L, 2))
        out["build_path"] = {"build": info["build"], "fallback": info["fallback"],
                             "note": "kmhg_info of the waited builds: 2 = partitioned, lane-order "
                                     "ranks; 3 = ballot ranks (the device failed the LDS "
                                     "lane-order self-check); 1 = global-atomic; fallback = 1 "
                                     "would mean a rebuild (the run fails instead)"}
        out["config"]["parallelism"] = "single" if world == 1 and not distributed \
            else f"replicas{world}"
        if distributed:
            out["config"]["workload"] = (
                f"configs[{args.config - 1}] sharded by sequence: every rank indexes its own "
                f"synthetic {L / 1e6:.0f} Mbp iid ACGT sequence (splitmix64 seed "
                f"{seed - rank} + rank), k={k}, make.kmer.hash; n_gpus independent indices, no "
                "data-path collective (weak scaling); the owner-computes build of ONE "
                "n_gpus x L sequence is the sharded_build record")
        if sharded:
            # the owner-computes build of one genome as a side record: its part
            # step, and the rate at which the parts become an index every rank can query
            out["sharded_build"] = sharded
        if sq:
            out["sharded_query"] = sq
        if large:
            out["large"] = large
        if not args.profile:
            out["host_boundary"] = host_boundary(host_seq.tobytes(), k)
        if not args.no_cpu and not args.profile:
            # config 3: the whole 100 Mbp (≈ 60 s of CPU: the verdict's full-size baseline)
            out["cpu_baseline"] = cpu_baseline(
                host_seq.tobytes(), k, sample_bp=L if args.config == 3 else 10_000_000,
                reps_max=1 if args.config == 3 else 3)
            if t_count:
                out["counts"]["cpu_baseline"] = cpu_counts_baseline(host_seq.tobytes(), k)
            if t_reads and sample_fq is not None:
                rb, db = cpu_reads_baseline(sample_fq, host_seq.tobytes(), k)
                out["reads"]["cpu_baseline"] = rb
                out["depth"]["cpu_baseline"] = db
        for leg in ("query", "counts", "reads", "depth"):
            if leg in out:
                out[leg]["steps"] = leg_steps
        print(json.dumps(out), file=_JSON_OUT, flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def _side_record(name: str, fn, *a):
    """An N > 1 side record whose failure must not cost the line its headline: an exception that
    every rank raises alike (an API or argument error) is recorded as the record's `error` and
    the ranks carry on; the headline `value` was measured before it."""
    import torch.distributed as dist
    try:
        return fn(*a)
    except Exception as e:                         # noqa: BLE001 -- reported in the line
        progress(f"{name} failed: {type(e).__name__}: {e}")
        if dist.is_initialized():
            dist.barrier()
        return {"error": f"{type(e).__name__}: {e}"[:500]}


def check_build(info: dict) -> None:
    """A waited build must not have fallen back to the global-atomic rebuild (kmhg_info.fallback:
    a bucket's LDS table overflowed or its stream failed the order check): the timed steps would
    not include that rebuild, so the run fails instead of reporting them."""
    if info.get("fallback"):
        raise SystemExit(f"bench: a build fell back to the global-atomic rebuild ({info}); "
                         "the timed steps would not measure what an R user gets")


def bench_sharded_build(args, k, L, dev, world, rank, seed):
    """Owner-computes make.kmer.hash of one (world x L)-base sequence over the ranks: a step is
    every rank's part build (kmhg_build_device_part), max over ranks.  Returns rank 0's record
    (value, ms_per_step and the roofline of rank 0's dominant part-build kernel included)."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd import synth
    big = torch.from_numpy(synth.iid(L * world, 1000 + seed - rank)).to(dev) if rank == 0 else None
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    seq_all = kd.broadcast_sequence(big, 0, dev, codec=kd.HipSeqCodec())   # packed, as C1
    torch.cuda.synchronize()
    t_bc = time.perf_counter() - t0
    for _ in range(max(1, args.warmup)):
        D.DeviceIndex.build_part(seq_all, k, rank, world).wait().free()
    # kernel times of rank 0's part build (dominant kernel -> roofline)
    D.timing_enable(True)
    D.timing_select(None)
    D.timing_reset()
    for _ in range(2):
        D.DeviceIndex.build_part(seq_all, k, rank, world).wait().free()
    wt = D.timing_report()
    per_step = {n: v[1] / 2 for n, v in wt.items() if v[0]}
    per_launch = {n: v[1] / v[0] for n, v in wt.items() if v[0]}
    D.timing_enable(False)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D.DeviceIndex.build_part(seq_all, k, rank, world).free()
    torch.cuda.synchronize()
    dist.barrier()
    t_part = time.perf_counter() - t0
    part = D.DeviceIndex.build_part(seq_all, k, rank, world)
    inf = kd.part_info_all(part, dev)
    # the parts -> the whole index on every rank (all-gather over the backend): once untimed (the
    # pools' first allocations), then timed over a few assemblies
    kd.assemble_parts(part, dev).free()
    n_asm = 3
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n_asm):
        idx = kd.assemble_parts(part, dev)
        if i + 1 < n_asm:
            idx.free()
    torch.cuda.synchronize()
    t_asm = (time.perf_counter() - t0) / n_asm
    _ai = idx.info()
    U, Npos, slots = _ai["n_kmers"], _ai["n_positions"], _ai["table_slots"]
    idx.free()
    part.free()
    tt = torch.tensor([t_part, t_bc, t_asm], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t_part, t_bc, t_asm = tt.tolist()
    if rank != 0:
        return None
    Ltot = L * world
    step_ms = t_part / args.steps * 1e3
    dom = max(per_step, key=per_step.get)
    # rank 0's share of SURVEY.md §8(d)'s build bytes: every rank reads the whole sequence, and
    # writes its ~1/world of the keys and positions
    B = Ltot + (12 * U + 4 * Npos) // world
    # bytes each rank receives in the assembly: the other parts' slots and positions
    in_bytes = (world - 1) * (slots * D.SLOT_BYTES + 4 * Npos) // world
    return {"value": round(Ltot / 1e6 * args.steps / t_part, 2), "unit": "Mbp/s",
            "ms_per_step": round(step_ms, 4), "seq_len": Ltot, "k": k,
            "value_queryable": round(Ltot / 1e6 / (step_ms * 1e-3 + t_asm), 2),
            "value_queryable_note": "n_gpus x L / (part-build step + one assembly over the "
                                    "process group's backend): the rate at which the parts "
                                    "become an index every rank can query (the reference's "
                                    ".Call returns a usable index, src/kmer_hash.c:506-540)",
            "distinct_kmers": U, "positions": Npos, "rank0_part_kmers": inf["n_kmers"],
            "sequence_broadcast_ms": round(t_bc * 1e3, 3),
            "assemble_ms": round(t_asm * 1e3, 3), "assemble_calls": n_asm,
            "assemble_bytes_in_per_rank": in_bytes,
            "backend": dist.get_backend(),
            "rank0_kernels_ms_per_step": {n: round(v, 5) for n, v in per_step.items()},
            "roofline": dict(roofline(B, dom, per_launch[dom], step_ms, {}), note=(
                "rank 0's dominant part-build kernel; algorithmic_bytes = the whole sequence "
                "(every rank reads it) + 1/n_gpus of SURVEY.md §8(d)'s key and position bytes")),
            "note": "owner-computes build of ONE sequence of n_gpus x seq_len bases: each rank "
                    "walks every window and builds the k-mers of its bucket range "
                    "(kmhg_build_device_part); the parts together are the whole index, "
                    "assembling it on every rank (all-gather) is timed as assemble_ms (mean of "
                    "assemble_calls); the sequence broadcast (once per genome) as "
                    "sequence_broadcast_ms"}


def _emit(out):
    print(json.dumps(out), file=_JSON_OUT, flush=True)


_T_START = time.perf_counter()


def progress(msg: str) -> None:
    """One progress line on stderr (rank-tagged): long phases of a run stay visibly alive."""
    r = os.environ.get("RANK", "0")
    print(f"[bench r{r} +{time.perf_counter() - _T_START:.1f}s] {msg}", file=sys.stderr,
          flush=True)


LARGE_L, LARGE_K = 500_000_000, 31


def bench_large(args, dev) -> dict:
    """Out-of-cache side record of the default line: config 5's workload on one
    GPU -- make.kmer.hash of A (500 Mbp iid, k = 31: a 12 GB table and 2 GB of positions, far
    beyond the 256 MiB Infinity Cache; the reference loop src/kmer_pos.c:66-98) timed like the
    headline (warmups, then K asynchronous builds bracketed by synchronize), and B's cross
    seq.kmer.pos against that index (src/kmer_pos.c:110-136; B = A + 1 % SNVs + 20
    inversions / translocations + N-runs), K timed queries.  Each carries its roofline (SURVEY.md
    §8(d) bytes, frac_of_step, PMC traffic from profiles/pmc_large.json); the reference's own
    whole-size CPU numbers (profiles/rd4e_ref_config5.json) are cited beside them."""
    import torch
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth
    L, k = LARGE_L, LARGE_K
    t_gen = time.perf_counter()
    A = synth.iid(L, 4)
    B = synth.derived(A, 5)
    ta = torch.from_numpy(A).to(dev)
    tb = torch.from_numpy(B).to(dev)
    del A, B
    t_gen = time.perf_counter() - t_gen
    stream = torch.cuda.current_stream()
    pmc = _load_pmc("large")
    steps = max(1, args.steps)
    # ---- build
    for _ in range(max(1, min(args.warmup, 2))):
        check_build(D.DeviceIndex.build(ta, k, stream).info())
    D.timing_enable(True)
    D.timing_select(None)
    D.timing_reset()
    bi = D.DeviceIndex.build(ta, k, stream)
    binfo = bi.info()
    bi.free()
    wt = D.timing_report()
    D.timing_enable(False)
    bper = {n: v[1] for n, v in wt.items() if v[0]}
    blaunch = {n: v[0] for n, v in wt.items() if v[0]}
    check_build(binfo)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        D.DeviceIndex.build(ta, k, stream).free()
    torch.cuda.synchronize()
    tb_ms = (time.perf_counter() - t0) / steps * 1e3
    U, N = binfo["n_kmers"], binfo["n_positions"]
    bdom = max(bper, key=bper.get)
    build_rec = {
        "value": round(L / 1e6 / (tb_ms * 1e-3), 2), "unit": "Mbp/s", "ms_per_step": round(tb_ms, 4),
        "steps": steps, "distinct_kmers": U, "positions": N,
        "kernels_ms_per_step": {n: round(v, 4) for n, v in bper.items()},
        "kernel_ms_sum": round(sum(bper.values()), 4),
        "roofline": roofline(survey_bytes("build", L=L, U=U, N=N), bdom,
                             bper[bdom] / blaunch[bdom], tb_ms, pmc, None, blaunch,
                             device_ms=sum(bper.values())),
        "build_path": {"build": binfo["build"], "fallback": binfo["fallback"]}}
    # ---- B's cross query against index(A)
    idx = D.DeviceIndex.build(ta, k, stream)
    idx.info()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    q = idx.query(tb, k, stream)
    H = q.n_rows
    q.free()
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t0
    for _ in range(max(1, min(args.warmup, 2))):
        idx.query(tb, k, stream).free()
    D.timing_enable(True)
    D.timing_reset()
    for _ in range(2):
        idx.query(tb, k, stream).free()
    qt = D.timing_report()
    D.timing_enable(False)
    qper = {n: v[1] / 2 for n, v in qt.items() if v[0]}
    qlaunch = {n: v[0] / 2 for n, v in qt.items() if v[0]}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx.query(tb, k, stream).free()
    torch.cuda.synchronize()
    tq_ms = (time.perf_counter() - t0) / steps * 1e3
    # the same query with its rows delivered into a fresh pageable host matrix, as an R session
    # receives them (kmhg_query_fill's path: diagonal runs over PCIe, expanded by host threads;
    # the N = 1 point of sharded_query.to_host).  The matrix's release (R's collector) is not
    # timed.
    n_host = max(1, min(steps, 5))
    th = 0.0
    for i in range(n_host + 1):
        hostm = torch.empty((H, 2), dtype=torch.int32)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        q = idx.query(tb, k, stream)
        D.rows_to_host(q.rows_view(), hostm, stream)
        q.free()
        if i:
            th += time.perf_counter() - t0
        del hostm
    th_ms = th / n_host * 1e3
    idx.free()
    # the first query of a second index, once the process's pools hold query-sized blocks: what
    # every later make.kmer.hash + seq.kmer.pos pair of an R session pays (the diagonal path's
    # preparation: V_diag_valid after a build that wrote the tags), with its kernels
    idx = D.DeviceIndex.build(ta, k, stream)
    idx.info()
    del ta
    torch.cuda.synchronize()
    D.timing_enable(True)
    D.timing_reset()
    t0 = time.perf_counter()
    idx.query(tb, k, stream).free()
    torch.cuda.synchronize()
    t_first2 = time.perf_counter() - t0
    fk = {n: round(v[1], 4) for n, v in D.timing_report().items() if v[0]}
    D.timing_enable(False)
    # the general lookup beyond the cache: index(A) queried by an independent i.i.d. 500 Mbp
    # sequence (seed 6), so every window misses and probes the 12 GB table through its slot
    # tags (the reference's kh_get per window, src/kmer_pos.c:55-60, 126-132)
    del tb
    tc = torch.from_numpy(synth.iid(L, 6)).to(dev)
    idx.query(tc, k, stream).free()
    D.timing_enable(True)
    D.timing_reset()
    for _ in range(2):
        idx.query(tc, k, stream).free()
    ut = D.timing_report()
    D.timing_enable(False)
    uper = {n: v[1] / 2 for n, v in ut.items() if v[0]}
    ulaunch = {n: v[0] / 2 for n, v in ut.items() if v[0]}
    n_u = max(1, min(steps, 10))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_u):
        q = idx.query(tc, k, stream)
        H_u = q.n_rows
        q.free()
    torch.cuda.synchronize()
    tu_ms = (time.perf_counter() - t0) / n_u * 1e3
    del tc
    idx.free()
    Nw = L - k + 1
    unrel_rec = {
        "value": round(L / 1e6 / (tu_ms * 1e-3), 2), "unit": "Mbp/s", "ms_per_step": round(tu_ms, 4),
        "steps": n_u, "rows": H_u,
        "kernels_ms_per_step": {n: round(v, 5) for n, v in uper.items()},
        "roofline": query_roofline(uper, L, Nw, H_u, _load_pmc("largeunrel"), tu_ms, ulaunch),
        "note": "index(A) queried by an independent i.i.d. 500 Mbp sequence (splitmix64 seed 6): "
                "every window misses and probes the 12 GB table through its slot tags (one random "
                "16-B tag group per window, the table only at a matching tag); PMC from "
                "profiles/pmc_configlargeunrel.json (tools/query_unrelated.py --L 500000000)"}
    query_rec = {
        "value": round(L / 1e6 / (tq_ms * 1e-3), 2), "unit": "Mbp/s", "ms_per_step": round(tq_ms, 4),
        "steps": steps, "rows": H, "first_query_ms": round(t_first * 1e3, 3),
        "first_query_new_index_ms": round(t_first2 * 1e3, 3),
        "first_query_new_index_kernels_ms": fk,
        "first_query_note": "first_query_ms: the first query of the process at this size (its "
                            "query buffers' first allocation included); "
                            "first_query_new_index_ms: the first query of a second index (the "
                            "per-index preparation an R session's build-and-query pays)",
        "kernels_ms_per_step": {n: round(v, 5) for n, v in qper.items()},
        "roofline": query_roofline(qper, L, Nw, H, pmc, tq_ms, qlaunch),
        "to_host": {"value": round(L / 1e6 / (th_ms * 1e-3), 2), "unit": "Mbp/s",
                    "ms_per_step": round(th_ms, 3), "steps": n_host,
                    "note": "the query with its rows delivered into a fresh pageable host "
                            "matrix as kmhg_query_fill does for R (diagonal runs over the one "
                            "PCIe link, expanded by host threads; the matrix's release not "
                            "timed): the N = 1 point of sharded_query.to_host"}}
    ref = _whole_size_config5()
    return {"workload": "configs[4] on one GPU: synthetic A = 500 Mbp iid ACGT (splitmix64 seed "
                        "4), B = A + 1% SNV + 20 inversions/translocations + N-runs (seed 5), "
                        "k=31; make.kmer.hash(A) and seq.kmer.pos(index(A), B), inputs resident "
                        "in HBM",
            "seq_len": L, "k": k, "build": build_rec, "query": query_rec, "unrelated": unrel_rec,
            "generate_s": round(t_gen, 2),
            "cpu_baseline": {"value": ref["build_value"] if ref else None, "unit": "Mbp/s",
                             "cores": ref["cores"] if ref else 1, "kind": "reference",
                             "sample": "the whole 500 Mbp A / B through the compiled reference "
                                       "(oracle/_ref) on a GPU box's host, 1 thread, recorded "
                                       "once (tools/ref_config5.py); cited, not re-run",
                             "whole_size_reference": ref},
            "note": "out-of-cache side record: the build's table is 12 GB and every radix "
                    "stream 6 GB, so its bytes go to HBM (configs[1]'s 240 MB table sits in the "
                    "Infinity Cache)"}


def bench_readout(args, cfg, dev, world, rank):
    """Config 4: kmer.pos pair.pos off-diagonals of a repeat-rich 40 Mbp index, per rank."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth
    L, k = cfg["L"], cfg["k"]
    host = synth.config4(L, 3 + rank)
    seq = torch.from_numpy(host).to(dev)
    t0 = time.perf_counter()
    idx = D.DeviceIndex.build(seq, k)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    info = idx.info()
    opt = 14
    # the first kmer.pos call also builds the readout order (k_read_first + k_read_order, cached
    # on the index): timed on its own, outside the steps
    D.timing_enable(True)
    D.timing_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = idx.positions(opt)
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t0
    del res
    kt_first = D.timing_report()
    D.timing_enable(False)
    for _ in range(args.warmup):
        res = idx.positions(opt)
        del res
    D.timing_enable(True)
    D.timing_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = idx.positions(opt)
        del res
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    kt = D.timing_report()
    D.timing_enable(False)
    # the same readout into fresh host matrices, as the R API's kmer.pos returns it
    # (kmhg_positions_fill: pos rows and counts copied, pair rows written by host threads from
    # the position lists); the matrices' release is not timed
    host_ms = None
    if not args.profile:
        import ctypes as _C
        import numpy as np
        from kmer_hasher_amd import _lib
        P_, N_, U_ = info["n_pairs"], info["n_positions"], info["n_kmers"]
        th = []
        for _ in range(3):
            bufs = [np.empty(2 * N_, np.int32), np.empty(3 * P_, np.int32), np.empty(U_, np.int32)]
            t0 = time.perf_counter()
            _lib.check(_lib.lib().kmhg_positions_fill(
                idx.handle, opt, None, *[_C.c_void_p(b.ctypes.data) if b.size else None
                                         for b in bufs]))
            th.append(time.perf_counter() - t0)
            del bufs
        host_ms = min(th) * 1e3
    tt = torch.tensor([t], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = tt.item()
    if rank == 0:
        P, N, U = info["n_pairs"], info["n_positions"], info["n_kmers"]
        per = {n: v[1] / v[0] for n, v in kt.items() if v[0]}
        launches = {n: v[0] / args.steps for n, v in kt.items() if v[0]}
        dom = max(per, key=per.get)
        ab = {"k_read_pairs": 12 * P + 8 * P, "k_read_pos": 8 * N + 4 * N}.get(dom)
        pmc = _load_pmc(4)
        B = survey_bytes("readout", U=U, N=N, P=P, opt=opt)
        cpu = None
        if not args.no_cpu and not args.profile:
            cpu = cpu_readout_baseline(host.tobytes(), k, opt)
        _emit({"metric": "kmer.pos pair.pos rows/s (config 4)", "value": round(P * world * args.steps / t / 1e9, 4),
               "unit": "G pair rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(t / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "i32", "data": "synthetic",
               "config": {"workload": cfg["workload"], "seq_len": L, "k": k, "distinct_kmers": U,
                          "positions": N, "pairs": P, "max_count": info["max_count"],
                          "build_s": round(t_build, 4),
                          "first_call_ms": round(t_first * 1e3, 3),
                          "first_call_prepare_ms": {n: round(v[1] / v[0], 4) for n, v in kt_first.items()
                                                    if v[0] and n in ("k_read_first", "k_read_order")}},
               "roofline": roofline(B, dom, per[dom], t / args.steps * 1e3, pmc, ab, launches),
               "cpu_baseline": cpu,
               "host": None if host_ms is None else {
                   "ms": round(host_ms, 3), "value": round(P / (host_ms * 1e-3) / 1e9, 4),
                   "unit": "G pair rows/s",
                   "note": "kmer.pos(opt 14) into fresh host matrices (kmhg_positions_fill, the R "
                           "API: pos rows and counts copied D2H, pair rows written by host "
                           "threads from the position lists), best of 3; PCIe- and host-memory-"
                           "inclusive, never `value`"},
               "kernels_ms": {n: round(v, 4) for n, v in per.items()}})
    idx.free()


def _load_pmc(config: int) -> dict:
    path = os.path.join(ROOT, "profiles", f"pmc_config{config}.json")
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return {}


def cpu_readout_baseline(seq_bytes: bytes, k: int, opt: int) -> dict:
    """kmer_positions(opt) of the compiled reference (oracle/_ref: the bucket walk of
    src/kmer_hash.c:1096-1124 restated over the reference's khash core) on the whole config-4
    index, 1 thread pinned: build and readout timed separately, teardown on its own line."""
    try:
        from oracle import oracle as O
        with _pinned_one_core():
            t0 = time.perf_counter()
            r = O.RefIndex(seq_bytes, k)
            t_build = time.perf_counter() - t0
            t_read, npos, npair = r.time_positions(opt)
            t0 = time.perf_counter()
            r.close()
            t_free = time.perf_counter() - t0
        return {"value": round(npair / t_read / 1e9, 5), "unit": "G pair rows/s", "cores": 1,
                "kind": "reference",
                "sample": f"the whole {len(seq_bytes) / 1e6:.0f} Mbp config-4 sequence, k={k}: "
                          f"kmer_positions(opt={opt}) into flat arrays (the R matrices' data), "
                          "oracle/_ref gcc -O2, 1 thread pinned",
                "readout_s": round(t_read, 3), "build_s": round(t_build, 3),
                "build_value": round(len(seq_bytes) / 1e6 / t_build, 3),
                "build_unit": "Mbp/s", "teardown_s": round(t_free, 3), "pos_rows": npos,
                "pair_rows": npair, "host": host_info()}
    except Exception as e:  # reported, never required
        return {"value": None, "unit": "G pair rows/s", "cores": 1, "kind": "reference",
                "sample": f"unavailable: {e}"}


def sharded_query_record(args, dev, world, rank, steps: int, timing_kernels: bool = False):
    """config 5's seq.kmer.pos sharded over the ranks (BASELINE.json north_star):
    B (500 Mbp) queried against index(A) (500 Mbp iid, k = 31), the reference loop
    src/kmer_pos.c:110-136 behind src/kmer_hash.c:1151-1172.

    index(A) is built on rank 0 and its image (table + positions + code block) broadcast once
    (timed, outside the steps).  A step is one seq.kmer.pos of B as the R session issues it: B
    sits on rank 0; C1 scatters to every rank the slice of B its window range reads; each rank
    runs the HIP range query; the rows are gathered into ONE device buffer on rank 0 in rank
    order (= the reference's row order; `value`).  `to_host` times the same step with the rows
    delivered instead into one host matrix shared by the node's ranks, each rank copying its own
    rows over its own PCIe link (dist.deliver_rows_host), and `c1_broadcast` the C1 phase as a
    broadcast of the whole B.  Phases are timed in separate synchronized steps, max over ranks.
    Returns rank 0's record (None elsewhere) and the kernel times of the timed steps."""
    import torch
    import torch.distributed as dist
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import dist as kd
    from kmer_hasher_amd import synth
    L, k = LARGE_L, LARGE_K
    tb, ta, index, t_build = None, None, None, 0.0
    if rank == 0:
        A = synth.iid(L, 4)
        tb = torch.from_numpy(synth.derived(A, 5)).to(dev)
        ta = torch.from_numpy(A).to(dev)
        del A
        D.DeviceIndex.build(ta, k).wait().free()       # the pool's first allocations, untimed
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        index = D.DeviceIndex.build(ta, k)
        index.wait()
        t_build = time.perf_counter() - t0
    t_bcast = 0.0
    # every collective of the path runs whenever a process group exists (the RCCL world-1
    # rehearsal, `--dist`, included); without one (`--config 5` at N = 1) the step is the plain
    # query
    use_pg = dist.is_available() and dist.is_initialized()
    if use_pg:
        # once untimed (the receivers' first allocations), then timed
        rep = kd.broadcast_index(index, dev)
        if rank:
            rep.free()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        index = kd.broadcast_index(index, dev)
        dist.barrier()
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - t0
    info = index.info()
    eng = kd.HipQueryEngine(index)
    # the scatter's receive buffer (non-root ranks), reused across steps
    seq_buf = torch.empty(L + 16, dtype=torch.uint8, device=dev) if rank else None
    sink = kd.HostRowSink(0) if use_pg else None
    host1 = None                                  # no process group: a pinned host matrix

    def step(timings=None, to_host=False, c1="scatter"):
        nonlocal host1
        if use_pg:
            return kd.sharded_query(eng, tb, k, dst=0, src=0, timings=timings, c1=c1,
                                    sink=sink if to_host else None, seq_buf=seq_buf)
        t0 = time.perf_counter()
        r = eng.query_range(tb, k, 0, tb.numel() - k + 1)
        if timings is not None:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        if to_host:
            if host1 is None or host1.shape[0] < r.shape[0]:
                host1 = torch.empty((r.shape[0], 2), dtype=torch.int32, pin_memory=True)
            D.rows_to_host(r, host1[:r.shape[0]])
            r = host1[:r.shape[0]]
        if timings is not None:
            t2 = time.perf_counter()
            for n_, dt in (("broadcast", 0.0), ("query", t1 - t0), ("gather", t2 - t1)):
                timings[n_] = timings.get(n_, 0.0) + dt
        return r

    def timed(n, **kw):
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        H = 0
        for _ in range(n):
            rows = step(**kw)
            H = rows.shape[0] if rows is not None else 0
            del rows
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, H

    def phases(n=2, **kw):
        ph = {}
        for _ in range(n):
            rows = step(ph, **kw)
            del rows
        return [ph.get(p, 0.0) / n for p in ("broadcast", "query", "gather")]

    progress(f"sharded query: index built {t_build:.3f} s, broadcast {t_bcast:.3f} s")
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rows = step()                  # first query: the index's diagonal-path preparation
        torch.cuda.synchronize()
        t_first = time.perf_counter() - t0
        del rows
        for _ in range(max(1, min(args.warmup, 3))):
            rows = step()
            del rows
        ph_dev = phases()
        if timing_kernels:
            D.timing_enable(True)
            D.timing_reset()
        t_dev, H = timed(steps)
        kt = D.timing_report() if timing_kernels else {}
        if timing_kernels:
            D.timing_enable(False)
        # the gather's wire format: rank 0's own range as diagonal runs (dist.HipRunCodec; the
        # other ranks' rows travel the same way), untimed
        w_r0 = kd.shard_ranges(L - k + 1, world)[0]
        loc = eng.query_range(tb, k, *w_r0) if rank == 0 else None
        runs0 = eng.codec.encode(loc) if loc is not None else None
        runs_fmt = None if loc is None else {
            "rows": int(loc.shape[0]), "runs": None if runs0 is None else int(runs0.shape[0])}
        del loc, runs0
        progress("sharded query: rows to the host matrix")
        # rows into the host matrix (what an R session receives): first delivery (the shared
        # buffer's creation and registration) untimed
        n_host = max(1, min(steps, 5))
        host_skip = None
        try:
            rows = step(to_host=True)
            del rows
            ph_host = phases(to_host=True)
            t_host, H_host = timed(n_host, to_host=True)
        except RuntimeError as e:     # no room for the shared host matrix (every rank raises)
            host_skip = str(e)
            ph_host, t_host, H_host = [0.0, 0.0, 0.0], 0.0, H
        ph_bc = phases(c1="broadcast") if use_pg else [0.0, 0.0, 0.0]
    finally:
        if sink is not None:
            sink.close()
    vals = [t_dev, t_host] + ph_dev + ph_host + ph_bc
    tt = torch.tensor(vals, dtype=torch.float64, device=dev)
    if use_pg:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t_dev, t_host, *ph = tt.tolist()
    ph_dev, ph_host, ph_bc = ph[0:3], ph[3:6], ph[6:9]
    index.free()
    # ---- the owner-routed alternative (no index broadcast, no replica): A broadcast, every rank
    # builds the k-mers it owns (dist.owner_build), B queried over the resident parts
    # (dist.owner_query: B broadcast, owned windows probed, rows merged on rank 0)
    own = None
    if use_pg:
        progress("sharded query: owner-routed parts")
        part, _ = kd.owner_build(ta, k, dev, src=0)      # untimed: first allocations
        kd.part_info_all(part, dev)
        part.free()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        part, _ = kd.owner_build(ta, k, dev, src=0)
        kd.part_info_all(part, dev)
        dist.barrier()
        torch.cuda.synchronize()
        t_obuild = time.perf_counter() - t0
        oeng = kd.HipPartEngine(part)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rows = kd.owner_query(oeng, tb, k, dst=0, src=0)
        torch.cuda.synchronize()
        t_ofirst = time.perf_counter() - t0
        H_own = rows.shape[0] if rows is not None else 0
        del rows
        oph = {}
        for _ in range(2):
            rows = kd.owner_query(oeng, tb, k, dst=0, src=0, timings=oph)
            del rows
        n_own = max(1, min(steps, 5))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_own):
            rows = kd.owner_query(oeng, tb, k, dst=0, src=0)
            del rows
        dist.barrier()
        torch.cuda.synchronize()
        t_own = time.perf_counter() - t0
        part.free()
        to = torch.tensor([t_obuild, t_ofirst, t_own] +
                          [oph.get(p, 0.0) / 2 for p in ("broadcast", "query", "gather", "merge")],
                          dtype=torch.float64, device=dev)
        dist.all_reduce(to, op=dist.ReduceOp.MAX)
        own = to.tolist() + [H_own, n_own]
    if rank != 0:
        return None, kt
    assert H_host == H, (H_host, H)
    if own is not None and int(own[7]) != H:
        raise SystemExit(f"bench: the owner-routed query returned {int(own[7])} rows, the "
                         f"replicated one {H}")

    def ms(x):
        return round(x * 1e3, 3)

    rec = {"value": round(L / 1e6 * steps / t_dev, 2), "unit": "Mbp/s",
           "ms_per_step": round(t_dev / steps * 1e3, 3), "steps": steps, "n_gpus": world,
           "scaling": "strong", "seq_len": L, "k": k, "rows": H,
           "distinct_kmers": info["n_kmers"],
           "index_build_s": round(t_build, 4), "index_broadcast_s": round(t_bcast, 4),
           "first_query_ms": ms(t_first),
           "phases_ms": {"query_scatter": ms(ph_dev[0]), "range_query": ms(ph_dev[1]),
                         "row_gather": ms(ph_dev[2]),
                         "note": "separate synchronized steps, max over ranks"},
           "to_host": {"skipped": host_skip} if host_skip else {
                       "value": round(L / 1e6 * n_host / t_host, 2), "unit": "Mbp/s",
                       "ms_per_step": round(t_host / n_host * 1e3, 3), "steps": n_host,
                       "phases_ms": {"query_scatter": ms(ph_host[0]),
                                     "range_query": ms(ph_host[1]),
                                     "rows_to_host": ms(ph_host[2])},
                       "note": "the same step with the rows delivered into one host matrix "
                               "(the R matrix's data): every rank delivers its own rows into "
                               "a node-shared, HIP-registered buffer at its row offset "
                               "(dist.deliver_rows_host: diagonal runs over the rank's PCIe "
                               "link, expanded by host threads, kmhg_rows_to_host); without a "
                               "process group the one GPU's rows into a pinned host matrix"},
           "roofline": sharded_roofline(survey_bytes("query", L=L, Nq=L - k + 1, H=H),
                                        t_dev / steps, ph_dev[1], world),
           "gather_format": dict(runs_fmt, bytes_ratio=round(
               8 * runs_fmt["rows"] / (12 * runs_fmt["runs"]), 1) if runs_fmt["runs"] else None,
               note="the rows cross xGMI as diagonal runs (12 B per run of rows (i, j), (i + 1, "
                    "j + 1), ...; dist.gather_rows + HipRunCodec: kmhg_rows_runs on the "
                    "senders, kmhg_runs_expand on rank 0); counted on rank 0's own window "
                    "range") if runs_fmt else None,
           "c1_broadcast_ms": ms(ph_bc[0]) if use_pg else None,
           "owner_routed": None if own is None else {
               "value": round(L / 1e6 * own[8] / own[2], 2), "unit": "Mbp/s",
               "ms_per_step": round(own[2] / own[8] * 1e3, 3), "steps": own[8],
               "rows": own[7], "part_build_ms": ms(own[0]), "first_query_ms": ms(own[1]),
               "phases_ms": {"query_broadcast": ms(own[3]), "part_query": ms(own[4]),
                             "row_gather": ms(own[5]), "merge": ms(own[6])},
               "build_and_query_once_ms": {
                   "owner_routed": ms(own[0] + own[1]),
                   "replicated": ms(t_build + t_bcast + t_first),
                   "note": "make.kmer.hash(A) then one seq.kmer.pos(B), as an R session issues "
                           "them: owner-computes parts (A broadcast, every rank builds the "
                           "k-mers it owns) + one owner-routed query, against rank 0's build + "
                           "the index image broadcast + the first sharded query"},
               "note": "no assembly, no index broadcast: every rank holds its part (1/n_gpus "
                       "of the index); a query step broadcasts B, every rank probes the "
                       "windows whose k-mer it owns (kmhg_query_run_device_part), the rows and "
                       "per-tile offsets go to rank 0, which interleaves them by window "
                       "(kmhg_merge_part_rows)"},
           "c1_broadcast_note": "C1 as a broadcast of the whole B (one separate step), against "
                                "query_scatter's slices",
           "backend": dist.get_backend() if use_pg else None,
           "note": "index(A) built on rank 0, its image broadcast once (index_broadcast_s); a "
                   "step scatters B's slices from rank 0, runs every rank's window range on "
                   "the HIP engine and gathers the rows into one device buffer on rank 0 in "
                   "rank order (the reference's row order), sent as diagonal runs"}
    return rec, kt


def sharded_roofline(B: int, step_s: float, query_s: float, world: int) -> dict:
    """The sharded query against the node's HBM roofline: SURVEY.md §8(d)'s query bytes of the
    whole job over the step (C1 + range queries + rows gathered) and over the range-query phase
    alone, per GPU (the job's bytes / n_gpus), against one GPU's 8 TB/s."""
    per_gpu = B / world
    ach = per_gpu / step_s / 1e9 if step_s else None
    achq = per_gpu / query_s / 1e9 if query_s else None
    return {"bound": "hbm", "algorithmic_bytes": B, "bytes_per_gpu": int(per_gpu),
            "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
            "range_query_achieved": round(achq, 2) if achq else None,
            "range_query_frac": round(achq / HBM_PEAK_GBS, 4) if achq else None,
            "bytes_source": "SURVEY.md §8(d) query bytes (L_q + 12 N_q + 12 H) of the whole job, "
                            "split evenly over the GPUs; frac over the whole step, "
                            "range_query_frac over the range-query phase alone"}


def bench_sharded_query(args, cfg, dev, world, rank):
    """Config 5 as its own line (`--config 5`): sharded_query_record's step is the headline,
    with the roofline of the per-rank range query, the reference on a bounded prefix beside it
    and the 500 Mbp index build (rank 0) as a side record."""
    import torch
    from kmer_hasher_amd import device as D
    from kmer_hasher_amd import synth
    L, k = cfg["L"], cfg["k"]
    rec, kt = sharded_query_record(args, dev, world, rank, args.steps, timing_kernels=True)
    # the 500 Mbp index build itself (make.kmer.hash of A), rank 0: per-kernel times of one
    # build, then BUILD5_STEPS timed builds (each waited for and freed)
    build_rec = None
    cpu_sample = None
    if rank == 0 and not args.profile:
        A = synth.iid(L, 4)
        if not args.no_cpu:
            cpu_sample = (A[:CONFIG5_CPU_BP].tobytes(),
                          synth.derived(A, 5)[:CONFIG5_CPU_BP].tobytes())
        ta = torch.from_numpy(A).to(dev)
        del A
        D.DeviceIndex.build(ta, k).wait().free()
        D.timing_enable(True)
        D.timing_select(None)
        D.timing_reset()
        D.DeviceIndex.build(ta, k).wait().free()
        _bt = D.timing_report()
        bper = {n: v[1] for n, v in _bt.items() if v[0]}
        blaunch = {n: v[0] for n, v in _bt.items() if v[0]}
        D.timing_enable(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(BUILD5_STEPS):
            bi = D.DeviceIndex.build(ta, k)
            binfo = bi.info()
            bi.free()
            check_build(binfo)
        torch.cuda.synchronize()
        tb5 = (time.perf_counter() - t0) / BUILD5_STEPS
        del ta
        bdom = max(bper, key=bper.get)
        build_rec = {"value": round(L / 1e6 / tb5, 2), "unit": "Mbp/s",
                     "ms_per_build": round(tb5 * 1e3, 3), "builds": BUILD5_STEPS,
                     "kernels_ms_per_build": {n: round(v, 4) for n, v in bper.items()},
                     "kernel_ms_sum": round(sum(bper.values()), 4),
                     "roofline": roofline(survey_bytes("build", L=L, U=binfo["n_kmers"],
                                                       N=binfo["n_positions"]),
                                          bdom, bper[bdom] / blaunch[bdom], tb5 * 1e3,
                                          _load_pmc(5), None, blaunch,
                                          device_ms=sum(bper.values())),
                     "build_path": {"build": binfo["build"], "fallback": binfo["fallback"]},
                     "note": "make.kmer.hash of A alone (500 Mbp, k=31), each build waited for "
                             "and freed; kernels_ms from HIP events of one build"}
    if rank == 0:
        per = {n: v[1] / v[0] for n, v in kt.items() if v[0]}
        launches = {n: v[0] / args.steps for n, v in kt.items() if v[0]}
        Nw_rank = (L - k + 1) // world
        H = rec["rows"]
        cpu = cpu_query_baseline(*cpu_sample, k) if cpu_sample else None
        cfg_rec = {kk: rec[kk] for kk in ("rows", "distinct_kmers", "index_build_s",
                                          "index_broadcast_s", "first_query_ms", "phases_ms")}
        _emit({"metric": "seq.kmer.pos query Mbp/s (config 5, sharded)",
               "value": rec["value"], "unit": "Mbp/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": rec["ms_per_step"], "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
               "config": {"workload": cfg["workload"], "seq_len": L, "k": k, **cfg_rec,
                          "parallelism": f"shard{world}"},
               "roofline": query_roofline(per, L // world, Nw_rank, H // world, _load_pmc(5),
                                          rec["ms_per_step"], launches),
               "to_host": rec["to_host"], "c1_broadcast_ms": rec["c1_broadcast_ms"],
               "cpu_baseline": cpu,
               "index_build": build_rec,
               "kernels_ms": {n: round(v, 4) for n, v in per.items()}})


# config 5's CPU baseline: the reference on a prefix of A and of B (the whole 500 Mbp index needs
# ~65 GB and minutes of one core)
CONFIG5_CPU_BP = 20_000_000
BUILD5_STEPS = 3


def _whole_size_config5():
    """The reference itself on the WHOLE 500 Mbp A / B (tools/ref_config5.py, run once on a GPU
    box's host: ~65 GB, 3.5 minutes of one core), recorded in profiles/rd4e_ref_config5.json;
    cited beside the bounded sample, not re-run by every bench."""
    try:
        r = json.load(open(os.path.join(ROOT, "profiles", "rd4e_ref_config5.json")))
        c = r["cpu"]
        return {"query_value": c["query_mbps"], "build_value": c["build_mbps"], "unit": "Mbp/s",
                "cores": c["cores"], "build_s": c["build_s"], "query_s": c["query_s"],
                "teardown_s": c["teardown_s"], "rows": r["query"]["31"]["H"],
                "rows_sha256": r["query"]["31"]["sha"], "host": c.get("host"),
                "source": "profiles/rd4e_ref_config5.json (tools/ref_config5.py)"}
    except Exception:
        return None


def cpu_query_baseline(a: bytes, b: bytes, k: int) -> dict:
    """seq_kmer_positions (src/kmer_pos.c:110-136) of the compiled reference (oracle/_ref): B's
    prefix queried against the index of A's prefix, 1 thread pinned."""
    try:
        from oracle import oracle as O
        with _pinned_one_core():
            t0 = time.perf_counter()
            r = O.RefIndex(a, k)
            t_build = time.perf_counter() - t0
            t0 = time.perf_counter()
            q = r.query(b, k)
            t_q = time.perf_counter() - t0
            n = q.size // 2
            del q
            t0 = time.perf_counter()
            r.close()
            t_free = time.perf_counter() - t0
        return {"value": round(len(b) / 1e6 / t_q, 3), "unit": "Mbp/s", "cores": 1,
                "kind": "reference",
                "sample": f"{len(b) / 1e6:.0f} Mbp prefix of B against the index of the "
                          f"{len(a) / 1e6:.0f} Mbp prefix of A, k={k}, oracle/_ref gcc -O2, "
                          "1 thread pinned",
                "query_s": round(t_q, 3), "query_rows": n, "build_s": round(t_build, 3),
                "teardown_s": round(t_free, 3), "host": host_info(),
                "whole_size_reference": _whole_size_config5()}
    except Exception as e:  # reported, never required
        return {"value": None, "unit": "Mbp/s", "cores": 1, "kind": "reference",
                "sample": f"unavailable: {e}"}


if __name__ == "__main__":
    main()

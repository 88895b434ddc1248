"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py <tag> <config>

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (per-kernel avg duration)
  profiles/<tag>_bench.json         the bench line printed under rocprofv3 --kernel-trace
  profiles/pmc_config<config>.json  per kernel: avg FETCH_SIZE / WRITE_SIZE and the HBM bytes per
                                    launch, corrected per MI355X_MICROARCH.md: FETCH_SIZE is in KiB
                                    and reads 1/2 of the bytes of wide coalesced reads on gfx950,
                                    so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (an upper bound
                                    for narrow/random reads, whose calibration is unmeasured).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return sorted(hits)


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "kmhg::"):
        n = n.replace(pre, "")
    return n.strip()


def counters(d, counter):
    per = defaultdict(list)
    for f in find(os.path.join(d, "**", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            per[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


# kernels whose reads are dominated by random 16-B / 4-B accesses (hash probes), for which the
# calibrated FETCH_SIZE already counts the bytes moved (64 B per read)
RANDOM_READ = {"k_query_probe", "k_query_fused", "k_depth_probe", "k_count_first",
               "k_diag_prep", "k_join_probe", "k_build_insert"}


def main():
    tag, cfg = sys.argv[1], sys.argv[2]
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(base, "ktrace", "**", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    log = os.path.join(base, "ktrace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                open(os.path.join(prof, f"{tag}_bench.json"), "w").write(line)
    fetch = counters(os.path.join(base, "pmc_fetch"), "FETCH_SIZE")
    write = counters(os.path.join(base, "pmc_write"), "WRITE_SIZE")
    out = {"_note": "per-launch averages; FETCH/WRITE_SIZE in KiB as rocprofv3 reports them. "
                    "FETCH_SIZE is 1/2 of the bytes of a wide coalesced streaming read "
                    "(MI355X_MICROARCH.md) but 64 B per random 4-B or 16-B read "
                    "(tools/calib/fetch_calib.hip, profiles/calib/): hbm_bytes_streaming = "
                    "(2*FETCH + WRITE)*1024, hbm_bytes_random = (FETCH + WRITE)*1024, and "
                    "hbm_bytes_per_launch is the one that fits the kernel's reads (random for "
                    + ", ".join(sorted(RANDOM_READ)) + "; streaming otherwise)",
           "_tag": tag}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k), write.get(k)
        hs = int((2 * (f or 0) + (w or 0)) * 1024)
        hr = int(((f or 0) + (w or 0)) * 1024)
        out[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_streaming": hs,
                  "hbm_bytes_random": hr,
                  "hbm_bytes_per_launch": hr if k.split("<")[0] in RANDOM_READ else hs}
    json.dump(out, open(os.path.join(prof, f"pmc_config{cfg}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

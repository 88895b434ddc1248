"""CPU checks of bench.py's roofline accounting (SURVEY.md §8(d) bytes, PMC summaries): the
pieces of the JSON line the GPU runs fill in, driven here with fixed kernel times and a synthetic
PMC summary."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

PMC = {  # per-launch HBM bytes, as tools/pmc_summary.py writes them
    "k_query_probe<true>": {"hbm_bytes_per_launch": 500},
    "k_query_emit1": {"hbm_bytes_per_launch": 1200},
    "k_query_emit": {"hbm_bytes_per_launch": 40},
    "k_scan_tiles_u64": {"hbm_bytes_per_launch": 5},
    "k_v2_bucket_wg<false, true, false>": {"hbm_bytes_per_launch": 3000},
}


def test_survey_bytes_match_section_8d():
    L, U, N, Nq, H = 1000, 900, 990, 990, 990
    assert bench.survey_bytes("build", L=L, U=U, N=N) == L + 12 * U + 4 * N
    assert bench.survey_bytes("query", L=L, Nq=Nq, H=H) == L + 12 * Nq + 12 * H
    assert bench.survey_bytes("readout", U=3, N=5, P=7, opt=2 | 4 | 8) == \
        4 * 3 + 4 * 5 + 8 * 5 + 12 * 7 + 4 * 3
    with pytest.raises(ValueError):
        bench.survey_bytes("nope")


def test_query_roofline_prices_the_query_kernels_together():
    """§8(d)'s query bytes over the summed times of probe + scan + emit, never over one kernel
    (round 4: over the probe alone the fraction exceeded the HBM peak)."""
    L, Nw, H = 10_000_000, 9_999_970, 9_999_970
    qper = {"k_query_probe": 0.035, "k_scan_tiles_u64": 0.006, "k_query_emit": 0.024}
    r = bench.query_roofline(qper, L, Nw, H, PMC, step_ms=0.078)
    B = bench.survey_bytes("query", L=L, Nq=Nw, H=H)
    assert r["algorithmic_bytes"] == B
    assert r["avg_ms"] == pytest.approx(sum(qper.values()), abs=1e-5)
    assert r["achieved"] == pytest.approx(B / (sum(qper.values()) * 1e-3) / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r["dominant_kernel"] == "k_query_probe"
    assert r["kernel"] == "k_query_emit+k_query_probe+k_scan_tiles_u64"
    assert r["traffic"] == 500                   # the dominant kernel's PMC bytes


def test_step_traffic_sums_every_kernel_behind_one_label():
    """One HIP-event label covering two kernels (k_query_emit = k_query_emit1 + k_query_emit)
    sums both PMC entries."""
    t = bench.pmc_step_traffic(PMC, {"k_query_probe": 1, "k_query_emit": 1, "k_scan_tiles_u64": 1})
    assert t == 500 + 1200 + 40 + 5
    assert bench.pmc_step_traffic(PMC, {"k_v2_bucket_wg": 2}) == 6000
    assert bench.pmc_step_traffic({}, {"k_query_probe": 1}) is None
    assert bench.pmc_step_traffic(PMC, {"k_not_profiled": 1}) is None


def test_build_roofline_fields():
    B = bench.survey_bytes("build", L=10_000_000, U=9_999_970, N=9_999_970)
    r = bench.roofline(B, "k_v2_bucket_wg", 0.11, 0.245, PMC, None, {"k_v2_bucket_wg": 1})
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert r["frac"] == pytest.approx(B / 0.11e-3 / 1e9 / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r["frac_of_step"] == pytest.approx(B / 0.245e-3 / 1e9 / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r["traffic"] == 3000 and r["traffic_step"] == 3000
    assert r["traffic_step_over_B"] == pytest.approx(3000 / B, abs=1e-3)


def test_traffic_frac_prices_the_bytes_moved():
    """traffic_frac = the PMC bytes of every kernel of the step over their summed device time /
    peak (round 5): next to §8(d)'s frac, it tells work avoided from HBM efficiency.  The query
    roofline carries no kernel_model (the diagonal path avoids most of the modelled bytes)."""
    B = bench.survey_bytes("build", L=10_000_000, U=9_999_970, N=9_999_970)
    big = {"k_v2_bucket_wg<false, true, false>": {"hbm_bytes_per_launch": 350_000_000}}
    r = bench.roofline(B, "k_v2_bucket_wg", 0.11, 0.245, big, None, {"k_v2_bucket_wg": 1},
                       device_ms=0.25)
    assert r["traffic_frac"] == round(350e6 / 0.25e-3 / 1e9 / bench.HBM_PEAK_GBS, 4)
    assert r["device_ms"] == pytest.approx(0.25)
    assert "traffic_frac" not in bench.roofline(B, "k_v2_bucket_wg", 0.11, 0.245, PMC, None,
                                                {"k_v2_bucket_wg": 1})
    qper = {"k_query_probe": 0.035, "k_scan_tiles_u64": 0.006, "k_query_emit": 0.024}
    qpmc = {k: {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"] * 100_000}
            for k, v in PMC.items()}
    q = bench.query_roofline(qper, 10_000_000, 9_999_970, 9_999_970, qpmc, step_ms=0.078)
    assert "kernel_model" not in q
    assert q["traffic_frac"] == round((500 + 1200 + 40 + 5) * 1e5 / 0.065e-3 / 1e9 / 8000, 4)


def test_stdout_carries_only_the_result_line():
    """After _claim_stdout, output printed by anything else (RCCL prints its version banner to
    stdout at process-group init) lands on stderr; the result line alone on stdout."""
    import subprocess
    code = ("import os, sys, json; sys.path.insert(0, %r); import bench; bench._claim_stdout(); "
            "print('banner'); os.write(1, b'native banner\\n'); "
            "print(json.dumps({'value': 1}), file=bench._JSON_OUT, flush=True)"
            % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 1}']
    assert "banner" in r.stderr and "native banner" in r.stderr


def test_sharded_roofline_splits_the_job_over_the_gpus():
    """The sharded query's roofline: §8(d) query bytes of the whole job, an even share per GPU,
    over the whole step and over the range-query phase."""
    L, k, H = 500_000_000, 31, 376_104_028
    B = bench.survey_bytes("query", L=L, Nq=L - k + 1, H=H)
    r = bench.sharded_roofline(B, step_s=3.6e-3, query_s=0.65e-3, world=8)
    assert r["algorithmic_bytes"] == B and r["bytes_per_gpu"] == B // 8
    assert r["achieved"] == pytest.approx(B / 8 / 3.6e-3 / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / bench.HBM_PEAK_GBS, rel=1e-3)
    assert r["range_query_frac"] > r["frac"]
    assert bench.sharded_roofline(B, 0.0, 0.0, 1)["frac"] is None

"""The bench line's roofline fields follow from the committed profile set.

bench.py prices the dominant kernel from `profiles/r06/final/`: the
rocprofv3 kernel-trace average, the kernel-trace busy time and the PMC
traffic / issue records. These CPU tests read the same files through
bench.py's own helpers and recompute the committed bench line's `kernel_ms`,
`achieved`, `frac`, `kernel_busy_ms_per_step`, `traffic` and `limiter`, so a
profile refresh without a matching bench line (or the reverse) fails here.
"""
import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FINAL = os.path.join(ROOT, "profiles", "r06", "final")


@pytest.fixture(scope="module")
def bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _line(name):
    with open(os.path.join(FINAL, name)) as f:
        return json.loads([x for x in f if x.startswith("{")][-1])


def test_profile_files_present():
    for f in ("kernel_stats_lanes4.csv", "kernel_stats_lanes1.csv", "kernel_busy.json",
              "traffic.json", "issue.json", "bench_default.json", "bench_driver.json"):
        assert os.path.exists(os.path.join(FINAL, f)), f


def test_rocprof_average_matches_csv(bench):
    with open(os.path.join(FINAL, "kernel_stats_lanes4.csv")) as f:
        rows = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(f)}
    ent = [v for k, v in rows.items() if "entropy_kernel" in k]
    assert len(ent) == 1
    assert bench._rocprof_ms(4, "entropy") == pytest.approx(ent[0] / 1e6)


def test_committed_line_reproducible(bench):
    rec = _line("bench_default.json")
    r = rec["roofline"]
    assert r["kernel"] == "entropy" and r["bound"] == "hbm"
    # headline: this run's HIP-event duration (round 5 on); round-4 lines
    # carried the committed rocprof average there
    ms = r["kernel_ms"]
    achieved = r["algorithmic_bytes_per_image"] * r["launch_images"] / (ms / 1e3) / 1e9
    assert r["achieved"] == pytest.approx(achieved, rel=1e-3)
    assert r["frac"] == pytest.approx(achieved / r["peak"], rel=1e-3)
    prof_ms = bench._rocprof_ms(rec["config"]["lanes"], "entropy")
    rocprof = r.get("profile", {}).get("kernel_ms_rocprof", r.get("kernel_ms"))
    assert rocprof == pytest.approx(prof_ms, abs=1e-4)
    assert r["kernel_busy_ms_per_step"] == pytest.approx(
        bench._kernel_busy_ms(rec["config"]["lanes"], "entropy"), abs=1e-5)
    traffic = bench._pmc(bench.PMC_TRAFFIC, "entropy", rec["config"]["per_gpu_batch"])
    assert r["traffic"] == traffic["traffic_bytes"]
    issue = bench._pmc(bench.PMC_ISSUE, "entropy", rec["config"]["per_gpu_batch"])
    # the limiter's HBM share: over this run's kernel_ms since round 6 (the
    # time base of `frac`), over the committed rocprof average before
    base_ms = ms if r.get("limiter_time_base") == "kernel_ms" else prof_ms
    hbm = traffic["traffic_bytes"] / (base_ms / 1e3) / 1e9 / bench.HBM_PEAK_GBS
    assert r["limiter"] == bench._limiter(issue, hbm)
    # lanes=1 figure from the one-lane trace
    assert r["lanes1"]["kernel_ms_rocprof"] == pytest.approx(bench._rocprof_ms(1, "entropy"))


def test_both_queue_settings_recorded():
    rec = _line("bench_default.json")
    q = rec["hw_queue_regimes"]
    assert {q["this_run"]["hw_queues"], q["other"]["hw_queues"]} == {4, 16}
    assert q["this_run"]["value"] == rec["value"]
    assert min(q["this_run"]["value"], q["other"]["value"]) >= 0.95 * max(
        q["this_run"]["value"], q["other"]["value"])


def test_limiter_thresholds(bench):
    base = {"waves": 1024, "lds_conflict_per_lds_inst": 1.0}
    assert bench._limiter(None, None).startswith("unmeasured")
    assert bench._limiter({**base, "valu_share": 0.2, "wait_share": 0.3}, 0.7).startswith("HBM")
    assert bench._limiter({**base, "valu_share": 0.6, "wait_share": 0.3}, 0.1).startswith("VALU")
    assert bench._limiter({**base, "valu_share": 0.3, "wait_share": 0.5}, 0.1).startswith("latency")
    assert bench._limiter({**base, "valu_share": 0.3, "wait_share": 0.3}, 0.1).startswith(
        "instruction issue")

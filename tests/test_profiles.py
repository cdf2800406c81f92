"""The committed measurement evidence (profiles/) is self-consistent: the
bench line's arithmetic, its trace-kernel time against the rocprofv3 kernel
statistics of the same code, and the per-launch HBM traffic against the raw
PMC passes it was reduced from (scripts/pmc_traffic.py).  CPU only."""
import csv
import importlib.util
import json
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PROF = REPO / "profiles" / "r01"


def _bench():
    return json.loads((PROF / "bench_config3.json").read_text())


def test_bench_line_contract_fields():
    d = _bench()
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline"):
        assert key in d, key
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in d["roofline"], key
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in d["cpu_baseline"], key
    assert d["config"]["workload"].startswith("config3")
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["unit"] == "GB/s"


def test_bench_line_arithmetic():
    d = _bench()
    c, r = d["config"], d["roofline"]
    rays = c["width"] * c["rows_per_rank"] * d["n_gpus"]
    assert d["value"] == pytest.approx(rays / (d["ms_per_step"] * 1e-3) / 1e6, rel=2e-3)
    assert r["algo_bytes_per_launch"] == 16 * c["width"] * c["rows_per_rank"]
    assert r["achieved"] == pytest.approx(
        r["algo_bytes_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e9, rel=2e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)


def test_trace_time_agrees_with_rocprof():
    """The bench's packet-attached event time of trace3_kernel and the
    rocprofv3 --kernel-trace --stats average of the same kernel."""
    d = _bench()
    rows = list(csv.DictReader(open(PROF / "kernel_stats_config3.csv")))
    trace = [r for r in rows if "trace3_kernel<0, 0>" in r["Name"]]
    assert len(trace) == 1
    rocprof_ms = float(trace[0]["AverageNs"]) / 1e6
    assert d["roofline"]["kernel_ms"] == pytest.approx(rocprof_ms, rel=0.05)


def test_traffic_matches_pmc_passes():
    spec = importlib.util.spec_from_file_location("pmc_traffic",
                                                  REPO / "scripts" / "pmc_traffic.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    w_kb, _ = mod.per_launch(PROF / "pmc_pass1.csv", "WRITE_SIZE")
    f_kb, _ = mod.per_launch(PROF / "pmc_pass2.csv", "FETCH_SIZE")
    summary = json.loads((REPO / "profiles" / "r01_pmc_config3.json").read_text())
    assert summary["write_bytes_per_launch"] == int(round(w_kb * 1024))
    assert summary["fetch_bytes_per_launch"] == int(round(f_kb * 1024 * 2))
    # the frame is written exactly once; re-reads stay a few percent
    assert summary["write_bytes_per_launch"] == summary["algo_bytes_per_launch"]
    assert summary["hbm_bytes_per_launch"] < 1.05 * summary["algo_bytes_per_launch"]
    assert _bench()["roofline"]["traffic"] == summary["hbm_bytes_per_launch"]


def test_config4_traffic_matches_pmc_passes():
    """Round 4: config 4's per-launch HBM traffic (profiles/r04/pmc_config4.json)
    against the raw trace-kernel rows of its WRITE_SIZE / FETCH_SIZE passes:
    the 1 GiB frame is written once (no wasted re-reads)."""
    spec = importlib.util.spec_from_file_location("pmc_traffic",
                                                  REPO / "scripts" / "pmc_traffic.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    r4 = REPO / "profiles" / "r04"
    w_kb, nw = mod.per_launch(r4 / "pmc_config4_pass1.csv", "WRITE_SIZE")
    f_kb, nf = mod.per_launch(r4 / "pmc_config4_pass2.csv", "FETCH_SIZE")
    s = json.loads((r4 / "pmc_config4.json").read_text())
    assert s["config"] == [8192, 8192, 192, 64, 4, "i32x4"]
    assert s["write_bytes_per_launch"] == int(round(w_kb * 1024))
    assert s["fetch_bytes_per_launch"] == int(round(f_kb * 1024 * 2))
    assert s["algo_bytes_per_launch"] == 8192 * 8192 * 16
    assert s["write_bytes_per_launch"] < 1.001 * s["algo_bytes_per_launch"]
    assert s["hbm_bytes_per_launch"] < 1.05 * s["algo_bytes_per_launch"]

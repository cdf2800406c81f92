"""The committed measurement evidence (profiles/) is self-consistent: the
bench line's arithmetic, its trace-kernel time against the rocprofv3 kernel
statistics of the same code, and the per-launch HBM traffic against the raw
PMC passes it was reduced from (scripts/pmc_traffic.py).  CPU only."""
import csv
import importlib.util
import json
from pathlib import Path

import numpy as np
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
    w_kb, _, _ = mod.per_launch(PROF / "pmc_pass1.csv", "WRITE_SIZE")
    f_kb, _, _ = mod.per_launch(PROF / "pmc_pass2.csv", "FETCH_SIZE")
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
    w_kb, nw, _ = mod.per_launch(r4 / "pmc_config4_pass1.csv", "WRITE_SIZE")
    f_kb, nf, _ = mod.per_launch(r4 / "pmc_config4_pass2.csv", "FETCH_SIZE")
    s = json.loads((r4 / "pmc_config4.json").read_text())
    assert s["config"] == [8192, 8192, 192, 64, 4, "i32x4"]
    assert s["write_bytes_per_launch"] == int(round(w_kb * 1024))
    assert s["fetch_bytes_per_launch"] == int(round(f_kb * 1024 * 2))
    assert s["algo_bytes_per_launch"] == 8192 * 8192 * 16
    assert s["write_bytes_per_launch"] < 1.001 * s["algo_bytes_per_launch"]
    assert s["hbm_bytes_per_launch"] < 1.05 * s["algo_bytes_per_launch"]


def test_config3_final_traffic_matches_pmc_passes():
    """Round 4's final library (raw buffer frame stores): config 3's traffic
    file, which bench.py's `roofline.traffic` reads by default
    (profiles/r04_pmc_config3.json), against the raw trace-kernel rows of its
    WRITE_SIZE / FETCH_SIZE passes: the frame is written exactly once."""
    spec = importlib.util.spec_from_file_location("pmc_traffic",
                                                  REPO / "scripts" / "pmc_traffic.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    r4 = REPO / "profiles" / "r04"
    w_kb, _, _ = mod.per_launch(r4 / "pmc_config3_final_pass1.csv", "WRITE_SIZE")
    f_kb, _, _ = mod.per_launch(r4 / "pmc_config3_final_pass2.csv", "FETCH_SIZE")
    s = json.loads((REPO / "profiles" / "r04_pmc_config3.json").read_text())
    assert s["config"] == [4096, 4096, 256, 64, 3, "i32x4"]
    assert s["write_bytes_per_launch"] == int(round(w_kb * 1024))
    assert s["fetch_bytes_per_launch"] == int(round(f_kb * 1024 * 2))
    assert s["write_bytes_per_launch"] == s["algo_bytes_per_launch"] == 4096 * 4096 * 16
    assert s["hbm_bytes_per_launch"] < 1.05 * s["algo_bytes_per_launch"]


def test_round4_bench_line_app_and_kernel_labels():
    """Round 4's final bench line: host_path.app holds reference scenes 1-3
    at 640x480 in both formats, every frame golden-checked, the first call's
    kernel time within 3x of the warm median; every kernel label names a
    kernel the library has."""
    d = json.loads((REPO / "profiles" / "r04" / "bench_r04h.json").read_text().splitlines()[-1])
    assert d["roofline"]["kernel"] == "trace3_kernel"
    assert d["texture_rgba8"]["roofline"]["kernel"] == "trace3_kernel"
    app = d["host_path"]["app"]
    assert app["resolution"] == "640x480" and set(app["scenes"]) == {"scene1", "scene2", "scene3"}
    for name, scene in app["scenes"].items():
        for fmt in ("i32x4", "rgba8"):
            e = scene[fmt]
            assert e["frame_check"] == "bit-exact", (name, fmt)
            assert e["kernel"] in ("frame_small_kernel", "trace3_kernel")
            assert e["first"]["kernel_ms"] <= 3 * e["warm_median"]["kernel_ms"], (name, fmt)
    assert app["scenes"]["scene1"]["i32x4"]["kernel"] == "frame_small_kernel"
    assert app["scenes"]["scene3"]["i32x4"]["kernel"] == "trace3_kernel"


def test_round4_other_configs_name_the_kernel_that_ran():
    lines = [json.loads(l) for l in
             (REPO / "profiles" / "r04" / "other_configs.jsonl").read_text().splitlines()]
    by_size = {(l["config"]["width"], l["config"]["height"]): l["roofline"]["kernel"]
               for l in lines if "config" in l}
    assert by_size[(512, 512)] == "frame_small_kernel"      # config 1
    assert by_size[(1920, 1080)] == "frame_small_kernel"    # config 2
    assert by_size[(8192, 8192)] == "trace3_kernel"         # config 4


def test_round5_bench_line_traffic_and_rocprof():
    """Round 5's headline kernel (trace_bin_kernel, the no-coarse path): the
    traffic file bench.py reads by default (profiles/r05_pmc_config3.json)
    against the raw rows of its WRITE_SIZE / FETCH_SIZE passes (the most
    launched trace kernel of those runs); the bench line of the same build
    carries that traffic, both frame-level fractions, and a kernel time
    within 5 % of rocprofv3's average over the same command (whose launches
    also include the clock ramp and the in-flight loop)."""
    spec = importlib.util.spec_from_file_location("pmc_traffic",
                                                  REPO / "scripts" / "pmc_traffic.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    r5 = REPO / "profiles" / "r05"
    w_kb, nw, kw = mod.per_launch(r5 / "pmc_config3_pass1.csv", "WRITE_SIZE")
    f_kb, nf, kf = mod.per_launch(r5 / "pmc_config3_pass2.csv", "FETCH_SIZE")
    assert kw == kf == "trace_bin_kernel<0>"
    s = json.loads((REPO / "profiles" / "r05_pmc_config3.json").read_text())
    assert s["kernel"] == "trace_bin_kernel<0>"
    assert s["write_bytes_per_launch"] == int(round(w_kb * 1024))
    assert s["fetch_bytes_per_launch"] == int(round(f_kb * 1024 * 2))
    assert s["write_bytes_per_launch"] < 1.0001 * s["algo_bytes_per_launch"]
    assert s["hbm_bytes_per_launch"] < 1.02 * s["algo_bytes_per_launch"]
    d = json.loads((r5 / "bench_r05f.json").read_text().splitlines()[-1])
    r = d["roofline"]
    assert r["kernel"] == "trace_bin_kernel" and r["traffic"] == s["hbm_bytes_per_launch"]
    assert r["frame_frac"] == pytest.approx(
        r["algo_bytes_per_launch"] / (d["ms_per_step"] * 1e-3) / 1e9 / r["peak"], abs=2e-3)
    t = d["texture_rgba8"]
    assert t["roofline"]["frame_frac"] == pytest.approx(
        t["roofline"]["algo_bytes_per_launch"] / (t["ms_per_step"] * 1e-3) / 1e9 / 8000.0,
        abs=2e-3)
    assert d["frames_in_flight"]["frame_check"] == "bit-exact"
    rows = list(csv.DictReader(open(r5 / "kernel_stats_config3_r05f.csv")))
    tb = [x for x in rows if "trace_bin_kernel<0>" in x["Name"]]
    assert len(tb) == 1
    assert r["kernel_ms"] == pytest.approx(float(tb[0]["AverageNs"]) / 1e6, rel=0.05)


def test_round5_rehearsal_lines_carry_host_frame_scaling():
    """The N = 2 / 4 rehearsal lines (ranks sharing one GPU) carry the
    top-level scaling_host_frame of bit-exact host frames."""
    for n in (2, 4):
        d = json.loads((REPO / "profiles" / "r05" / f"rehearse_n{n}.json").read_text())
        assert d["n_gpus"] == n
        shf = d["scaling_host_frame"]
        for fmt in ("i32x4", "rgba8"):
            assert d["host_frame"][fmt]["frame_check"] == "bit-exact"
            assert shf[fmt] == d["host_frame"][fmt]["scaling"]
        assert "frame_frac" in d["roofline"]


def test_round5_final_bench_line_and_rocprof_launches():
    """The final round-5 line (in-flight window after its own clock ramp):
    its trace-kernel time within 3 % of the median launch of rocprofv3's
    kernel trace of the same command, whose mean is the stats file's
    AverageNs (the ramps' first launches and the in-flight windows pull
    the mean up)."""
    r5 = REPO / "profiles" / "r05"
    d = json.loads((r5 / "bench_r05i.json").read_text().splitlines()[-1])
    assert d["frames_in_flight"]["frame_check"] == "bit-exact"
    assert d["frames_in_flight"]["clock_ramp_steps"] > 0
    assert d["ms_per_step"] == d["frames_in_flight"]["ms_per_step"]
    r = d["roofline"]
    assert r["kernel"] == "trace_bin_kernel"
    assert r["frame_frac"] == pytest.approx(
        r["algo_bytes_per_launch"] / (d["ms_per_step"] * 1e-3) / 1e9 / r["peak"], abs=2e-3)
    la = json.loads((r5 / "rocprof_launches_r05i.json").read_text())
    assert r["kernel_ms"] * 1e3 == pytest.approx(la["median_us"], rel=0.03)
    rows = list(csv.DictReader(open(r5 / "kernel_stats_config3_r05i.csv")))
    tb = [x for x in rows if "trace_bin_kernel<0>" in x["Name"]]
    assert len(tb) == 1 and int(tb[0]["Calls"]) == la["launches"]
    assert float(tb[0]["AverageNs"]) / 1e3 == pytest.approx(la["mean_us"], rel=1e-3)



def test_round6_bench_line_checks_its_frames_against_the_fixture():
    """Round 6's line (profiles/r06/bench_r06a.json, the default command on
    the box): both formats' timed frames equal the committed fixture's hash
    (frame_check_ref), the long in-flight window is on by default (600
    frames, independent of --steps) for both formats, and the int32x4 window
    agrees with it within 5 % (the Texture's 3-slot K = 20 window pays the
    pipeline's fill and drain)."""
    d = json.loads((REPO / "profiles" / "r06" / "bench_r06a.json").read_text().splitlines()[-1])
    g = np.load(REPO / "tests" / "golden" / "config3_4096x4096.npz")
    assert d["frame_check_ref"] == "bit-exact"
    assert d["frame_check_ref_source"]["fnv1a64"] == f"{int(g['fnv1a64']):016x}"
    t = d["texture_rgba8"]
    assert t["frame_check_ref"] == "bit-exact"
    assert t["frame_check_ref_source"]["fnv1a64"] == f"{int(g['fnv1a64_rgba8']):016x}"
    for leg in (d, t):
        s = leg["frames_in_flight"]["sustained"]
        assert s["steps"] == 600
        assert s["vs_window"] == pytest.approx(leg["frames_in_flight"]["ms_per_step"] /
                                               s["ms_per_step"], rel=5e-3)
    assert d["frames_in_flight"]["sustained"]["vs_window"] == pytest.approx(1.0, abs=0.05)


def test_round6_rehearsal_lines_carry_the_scaling_contract():
    """The N = 2 / 4 / 8 rehearsals of round 6 (bench.py starting its own
    ranks, every rank on one GPU, gloo): every assembly bit-exact against the
    one-GPU render AND the committed fixture's hash, and the line's scaling
    keys consistent with its own timings."""
    for n in (2, 4, 8):
        d = json.loads((REPO / "profiles" / "r06" / f"rehearse_n{n}.json").read_text())
        assert d["n_gpus"] == n and "phase_errors" not in d
        for how, a in d["assembly"].items():
            assert a["frame_check"] == "bit-exact" and a["frame_check_ref"] == "bit-exact", how
        assert d["frame_check_ref"] == "bit-exact"
        t1 = d["one_gpu"]["ms_per_step"]
        assert d["scaling_assembled"] == pytest.approx(t1 / d["ms_per_step"], rel=1e-3, abs=1e-4)
        assert d["scaling_weak"] == pytest.approx(n * t1 / d["weak_scaling"]["ms_per_step"],
                                                  rel=1e-3, abs=1e-4)
        assert "scaling_host_frame" in d["scaling_note"]
        for fmt in ("i32x4", "rgba8"):
            assert d["host_frame"][fmt]["frame_check"] == "bit-exact"


@pytest.mark.parametrize("tag", ["r06k_final", "r06m_final", "r06s_final", "r06v_final"])
def test_round6_final_line_agrees_with_rocprof_and_pmc(tag):
    """The final round-6 lines (profiles/r06/bench_<tag>.json): the trace
    kernel's time from its packet events within 5 % of rocprofv3's mean over
    the same command (--sustained 0) and 2 % of its median; the line's
    traffic equals the committed PMC passes (1.011x the frame, no re-reads);
    both formats' frames equal the fixture."""
    r6 = REPO / "profiles" / "r06"
    d = json.loads((r6 / f"bench_{tag}.json").read_text().splitlines()[-1])
    r = d["roofline"]
    assert r["kernel"] == "trace_bin_kernel" and d["frame_check_ref"] == "bit-exact"
    assert d["texture_rgba8"]["frame_check_ref"] == "bit-exact"
    la = json.loads((r6 / f"rocprof_launches_{tag}.json").read_text())
    assert r["kernel_ms"] * 1e3 == pytest.approx(la["mean_us"], rel=0.05)
    assert r["kernel_ms"] * 1e3 == pytest.approx(la["median_us"], rel=0.02)
    rows = list(csv.DictReader(open(r6 / f"kernel_stats_config3_{tag}.csv")))
    tb = [x for x in rows if "trace_bin_kernel<0>" in x["Name"]]
    assert len(tb) == 1 and float(tb[0]["AverageNs"]) / 1e3 == pytest.approx(la["mean_us"], rel=1e-3)
    pmc = json.loads((REPO / "profiles" / "r06_pmc_config3.json").read_text())
    # (the line read the PMC file committed before this run: the previous
    # library's passes, 18 KB of fetch apart)
    assert r["traffic"] == pytest.approx(pmc["hbm_bytes_per_launch"], rel=1e-3)
    assert pmc["hbm_bytes_per_launch"] / pmc["algo_bytes_per_launch"] == pytest.approx(1.011, abs=2e-3)
    assert r["frac"] == pytest.approx(
        r["algo_bytes_per_launch"] / (r["kernel_ms"] * 1e-3) / 1e9 / r["peak"], abs=2e-3)

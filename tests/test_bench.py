"""bench.py's arithmetic and the N>1 frame assembly, on the CPU.

The assembly test runs the same rowbands.assemble_frame the GPU bench uses
(RCCL point-to-point there) over gloo with world sizes 2 and 3, bands of
unequal size and an empty band, and checks the root's frame row for row."""
import importlib.util
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def _bench():
    import __graft_entry__
    __graft_entry__.load_package()
    spec = importlib.util.spec_from_file_location("rt_bench", REPO / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_arithmetic():
    b = _bench()
    # 4096^2 rays in 0.0584 ms
    assert b.mrays_per_s(4096 * 4096, 0.0584) == pytest.approx(16777216 / 58.4, rel=1e-12)
    # every band but the root's reaches the root
    assert b.bytes_to_root(4096, 4096, 1, "i32x4") == 0
    assert b.bytes_to_root(4096, 4096, 8, "i32x4") == 16 * 4096 * 4096 * 7 // 8
    assert b.bytes_to_root(4096, 4096, 8, "rgba8") == 4 * 4096 * 4096 * 7 // 8
    assert b.bytes_to_root(640, 97, 2, "i32x4") == 16 * 640 * (97 - 48)
    # value = the fastest assembly whose frame is bit-exact
    asm = {"rccl_p2p": {"ms_per_step": 0.9, "frame_check": "bit-exact"},
           "xgmi_peer_store": {"ms_per_step": 0.5, "frame_check": "bit-exact"}}
    assert b.pick_value(asm)[0] == "xgmi_peer_store"
    asm["xgmi_peer_store"]["frame_check"] = "MISMATCH"
    assert b.pick_value(asm)[0] == "rccl_p2p"
    asm["rccl_p2p"] = {"ms_per_step": None, "error": "no mapping"}
    assert b.pick_value(asm) == (None, None)  # the line then carries value null
    asm["rccl_p2p"] = {"error": "rank 1: RuntimeError: boom"}  # a failed phase
    assert b.pick_value(asm) == (None, None)


def test_cpu_quota(tmp_path):
    b = _bench()
    assert b.cpu_quota(str(tmp_path)) == (None, None)  # no cgroup files
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert b.cpu_quota(str(tmp_path)) == (None, str(tmp_path / "cpu.max"))
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert b.cpu_quota(str(tmp_path))[0] == 16.0
    (tmp_path / "cpu.max").unlink()
    (tmp_path / "cpu").mkdir()
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    (tmp_path / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert b.cpu_quota(str(tmp_path))[0] is None
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("800000\n")
    assert b.cpu_quota(str(tmp_path))[0] == 8.0


def test_cpu_threads_report(monkeypatch):
    b = _bench()
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n, info = b.cpu_threads(0)
    assert n == min(3, aff)
    assert info["affinity_cpus"] == aff and info["os_cpu_count"] == os.cpu_count()
    monkeypatch.delenv("OMP_NUM_THREADS")
    quota = b.cpu_quota()[0]
    assert b.cpu_threads(0)[0] == (aff if quota is None else min(aff, max(1, int(quota))))
    assert b.cpu_threads(1)[0] == 1
    assert "cgroup_cpu_quota" in b.cpu_threads(0)[1]


def test_bench_parse_defaults():
    b = _bench()
    a = b.parse([])
    assert (a.gpus, a.width, a.height, a.spheres, a.cubes, a.seed, a.format) == \
        (1, 4096, 4096, 256, 64, 3, "i32x4")
    assert b.CONFIG_NAMES[(a.width, a.height, a.spheres, a.cubes)] == "config3"
    c4 = b.CONFIG4
    assert b.CONFIG_NAMES[(c4["width"], c4["height"], c4["spheres"], c4["cubes"])] == "config4"


def _assemble_worker(rank, world, port, height, width, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    import torch
    import torch.distributed as dist

    import __graft_entry__

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        __graft_entry__.load_package()
        from opencl_ray_tracer_amd import rowbands

        rb, re = rowbands.band_rows(height, world, rank) if height >= world else \
            (min(rank, height), min(rank + 1, height))

        def rows(a, b):  # pixel (y, x, c) = 1000 y + 10 x + c, this rank's rows
            y = torch.arange(a, b, dtype=torch.int32).view(-1, 1, 1)
            x = torch.arange(width, dtype=torch.int32).view(1, -1, 1)
            ch = torch.arange(4, dtype=torch.int32).view(1, 1, -1)
            return (1000 * y + 10 * x + ch).contiguous()

        frame = None
        if rank == 0:
            frame = torch.full((height, width, 4), -7, dtype=torch.int32)
            frame[rb:re] = rows(rb, re)  # the root renders its band in place
            band = frame[rb:re]
        else:
            band = rows(rb, re)
        rowbands.assemble_frame(frame, band, height, world, rank)
        if rank == 0:
            np.save(result_path, frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,height", [(2, 97), (3, 100), (3, 7)])
def test_assemble_frame_gloo(tmp_path, world, height):
    import torch.multiprocessing as mp

    width = 33
    out = tmp_path / "frame.npy"
    mp.spawn(_assemble_worker, args=(world, _free_port(), height, width, str(out)),
             nprocs=world, join=True)
    frame = np.load(out)
    y = np.arange(height).reshape(-1, 1, 1)
    x = np.arange(width).reshape(1, -1, 1)
    ch = np.arange(4).reshape(1, 1, -1)
    assert np.array_equal(frame, 1000 * y + 10 * x + ch)


def _empty_band_worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    import torch
    import torch.distributed as dist

    import __graft_entry__

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        __graft_entry__.load_package()
        from opencl_ray_tracer_amd import rowbands

        def render_band(rb, re):
            if re <= rb:
                raise AssertionError("an empty row range must not be rendered")
            return torch.arange(rb, re, dtype=torch.int32).view(-1, 1).repeat(1, 5)

        frame = rowbands.render_distributed(render_band, 2, world, rank)
        if rank == 0:
            np.save(result_path, frame.numpy())
    finally:
        dist.destroy_process_group()


def test_render_distributed_more_ranks_than_rows(tmp_path):
    """height < world: the rank without rows still joins the gather (no hang)."""
    import torch.multiprocessing as mp

    out = tmp_path / "frame.npy"
    mp.spawn(_empty_band_worker, args=(3, _free_port(), str(out)), nprocs=3, join=True)
    assert np.array_equal(np.load(out), np.array([[0] * 5, [1] * 5]))


def test_balanced_bands():
    import __graft_entry__
    __graft_entry__.load_package()
    from opencl_ray_tracer_amd.rowbands import balanced_bands

    # equal costs: equal bands
    b = balanced_bands(4096, [(1e-5, 1e-8)] * 4)
    assert [e - s for s, e in b] == [1024] * 4
    # rank 0 without a link costs 1/20 per row: it takes most rows, and every
    # rank's modelled time is (nearly) equal
    costs = [(1e-5, 1e-8)] + [(1e-5, 2e-7)] * 7
    b = balanced_bands(4096, costs)
    assert b[0][0] == 0 and b[-1][1] == 4096
    assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
    rows = [e - s for s, e in b]
    t = [a + s * n for (a, s), n in zip(costs, rows)]
    assert rows[0] > 3000 and max(t) - min(t) <= 2 * max(s for _, s in costs) + 1e-12
    # a rank whose fixed cost alone exceeds the finish time gets no rows
    b = balanced_bands(100, [(0.0, 1e-6), (1.0, 1e-6)])
    assert [e - s for s, e in b] == [100, 0]
    # ... even when it is rank 0: the leftover rows never go to a dropped rank
    b = balanced_bands(100, [(1.0, 1e-6), (0.0, 1e-6), (0.0, 3e-6)])
    assert b[0] == (0, 0) and sum(e - s for s, e in b) == 100 and b[-1][1] == 100
    # every band well-formed and the rows summing to the height, whatever the costs
    rng = np.random.default_rng(3)
    for _ in range(200):
        n = int(rng.integers(1, 9))
        hgt = int(rng.integers(1, 5000))
        costs = [(float(rng.uniform(0, 1e-4)), float(rng.uniform(1e-9, 1e-6))) for _ in range(n)]
        b = balanced_bands(hgt, costs)
        assert b[0][0] == 0 and b[-1][1] == hgt
        assert all(s <= e for s, e in b) and all(x[1] == y[0] for x, y in zip(b, b[1:]))
    with pytest.raises(ValueError):
        balanced_bands(10, [(0.0, 0.0)])


class _FakeCtx:
    """bench.Ctx's collective plumbing on gloo, without a GPU."""

    def __init__(self, rank, world):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank, self.world = rank, world
        self.distributed = world > 1
        self.coll_dev = torch.device("cpu")
        self.pg = None
        self.renewed = 0

    def renew_group(self):
        import datetime
        self.pg = self.dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=5))
        self.renewed += 1


def _args(b, extra=()):
    return b.parse(["--gpus", "2", *extra])


def _phases_worker(rank, world, port, out_path):
    """Two gloo ranks run the N>1 line's phases with failures forced in
    them: an assembly raising on every rank, one raising on rank 1 only while
    rank 0 waits in a collective of that phase (it times out and joins the
    agreement), an extra phase that fails; rank 0 writes the printed line."""
    import datetime
    import io
    import contextlib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=5))
    try:
        b = _bench()
        c = _FakeCtx(rank, world)
        args = _args(b, ["--fail-assembly", "xgmi_peer_store"])
        state = {"assembly": {}}
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            ph = b.Phases(c, 60.0, lambda: b.multi_line(args, c, state), pg_timeout_s=20.0)

            def ok_assembly():
                dist.barrier()
                return {"ms_per_step": 0.5, "frame_check": "bit-exact"}

            def forced():
                if b.failing(args, c, "xgmi_peer_store"):
                    raise RuntimeError(f"--fail-assembly {args.fail_assembly}")
                return {"ms_per_step": 0.1, "frame_check": "bit-exact"}

            def one_rank():
                if rank == 1:
                    raise RuntimeError("rank 1 only")
                dist.barrier()  # rank 0 blocks here until the gloo timeout
                return {"ms_per_step": 0.05, "frame_check": "bit-exact"}

            def after():
                # a collective on the data-path group after the one-rank
                # failure: it must line up again (the group was renewed)
                import torch
                t = torch.ones(1)
                dist.all_reduce(t, group=c.pg)
                return {"frac": 0.5, "sum": float(t.item())}

            ph.run("rccl_p2p", ok_assembly, state["assembly"])
            ph.run("xgmi_peer_store", forced, state["assembly"])
            ph.run("xgmi_peer_store_balanced", one_rank, state["assembly"])
            ph.run("weak_scaling", lambda: 1 / 0, state)
            ph.run("roofline", after, state)
            # the app's host frame, one format bit-exact, one not
            state["host_frame"] = {}
            ph.run("i32x4", lambda: {"scaling": 1.8, "frame_check": "bit-exact"},
                   state["host_frame"])
            ph.run("rgba8", lambda: {"scaling": 1.5, "frame_check": "MISMATCH"},
                   state["host_frame"])
            ph.emit()
            assert c.renewed == 3
        if rank == 0:
            with open(out_path, "w") as f:
                f.write(buf.getvalue())
        else:
            assert buf.getvalue() == ""  # only rank 0 prints
    finally:
        dist.destroy_process_group()


def test_phases_record_failures_gloo(tmp_path):
    """N>1 bench: an assembly that raises (on every rank, or on one rank while
    the other waits in a collective) is recorded as {"error": ...}, the other
    phases still run, and rank 0 prints ONE line that parses."""
    import json
    import torch.multiprocessing as mp

    b = _bench()
    out = tmp_path / "line.txt"
    mp.spawn(_phases_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    lines = [l for l in out.read_text().splitlines() if l.strip()]
    assert len(lines) == 1
    line = json.loads(lines[0])
    asm = line["assembly"]
    assert "error" in asm["xgmi_peer_store"] and "--fail-assembly" in asm["xgmi_peer_store"]["error"]
    assert "error" in asm["xgmi_peer_store_balanced"]
    assert asm["rccl_p2p"]["frame_check"] == "bit-exact"
    # value from the one assembly that completed bit-exactly
    assert line["ms_per_step"] == 0.5 and line["value"] == pytest.approx(4096 * 4096 / 0.5e-3 / 1e6, rel=1e-3)
    assert "error" in line["weak_scaling"]
    rl = line["roofline"]
    assert (rl["frac"], rl["sum"]) == (0.5, 2.0)
    # the frame level: the assembled frame's bytes over ms_per_step, N x peak
    assert rl["frame_frac"] == pytest.approx(
        16 * 4096 * 4096 / 0.5e-3 / 1e9 / (2 * b.HBM_PEAK_GBS), abs=1e-4)
    # the host frame's scaling beside `value`, bit-exact formats only
    shf = line["scaling_host_frame"]
    assert shf["i32x4"] == 1.8 and shf["rgba8"] is None and "t(N=1)/t(N)" in shf["definition"]
    assert line["phase_errors"] == ["assembly.xgmi_peer_store",
                                    "assembly.xgmi_peer_store_balanced", "weak_scaling"]
    assert line["n_gpus"] == 2 and line["metric"]


_WATCHDOG = r"""
import sys, time
sys.path.insert(0, {repo!r})
sys.argv = ["bench.py"]
import importlib.util
spec = importlib.util.spec_from_file_location("rt_bench", {bench!r})
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
class C:
    rank, world, distributed = 0, 1, False
c = C()
args = b.parse([])
state = {{"assembly": {{"rccl_p2p": {{"ms_per_step": 0.25, "frame_check": "bit-exact"}}}}}}
ph = b.Phases(c, 1.0, lambda: b.multi_line(args, c, state))
ph.run("weak_scaling", lambda: time.sleep(60), state)  # hangs past the deadline
print("not reached")
"""


def test_phase_watchdog_prints_line():
    """A phase that hangs (an RCCL collective that never completes) makes rank
    0 print the line built so far, that phase marked as a timeout, and exit
    with EXIT_HUNG (non-zero) long before the hang ends."""
    import json
    import subprocess
    import time

    code = _WATCHDOG.format(repo=str(REPO), bench=str(REPO / "bench.py"))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=50)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert time.monotonic() - t0 < 40
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout
    line = json.loads(lines[0])
    assert "timeout" in line["weak_scaling"]["error"]
    assert line["ms_per_step"] == 0.25 and line["phase_errors"] == ["weak_scaling"]


_TWO_RANKS = r"""
import datetime, os, sys
sys.path.insert(0, {repo!r})
sys.argv = ["bench.py"]
import importlib.util
spec = importlib.util.spec_from_file_location("rt_bench", {bench!r})
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
import torch, torch.distributed as dist
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
class C:
    world, distributed, pg = 2, True, None
c = C()
c.rank, c.torch, c.dist = rank, torch, dist
args = b.parse(["--gpus", "2"])
state = {{"assembly": {{"rccl_p2p": {{"ms_per_step": 0.25, "frame_check": "bit-exact"}}}}}}
ph = b.Phases(c, 3.0, lambda: b.multi_line(args, c, state), pg_timeout_s=120.0)
def phase():
    if rank == 1:
        raise RuntimeError("rank 1 only")
    dist.barrier()  # never joined by rank 1: would block for the 120 s timeout
ph.run("xgmi_peer_store", phase, state["assembly"])
print("not reached")
"""


def test_phase_hang_every_rank_exits_nonzero(tmp_path):
    """An exception on rank 1 while rank 0 blocks in that phase's data-path
    collective, whose timeout (120 s here) is beyond the phase deadline, so
    it is a hang: rank 0's watchdog prints the line with the phase marked as
    failed and exits with EXIT_HUNG, and rank 1, waiting in the agreement,
    ends with EXIT_HUNG as well -- the launcher sees a failed run, and the
    line that names the phase."""
    import json
    import subprocess
    import time

    code = _TWO_RANKS.format(repo=str(REPO), bench=str(REPO / "bench.py"))
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env, cwd=tmp_path))
    outs = [p.communicate(timeout=100) for p in procs]
    assert time.monotonic() - t0 < 90
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 3, (p.returncode, err[-2000:])
        assert "not reached" not in out
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not [l for l in outs[1][0].splitlines() if l.startswith("{")]
    line = json.loads(lines[0])
    assert "error" in line["assembly"]["xgmi_peer_store"]
    assert line["ms_per_step"] == 0.25 and line["phase_errors"] == ["assembly.xgmi_peer_store"]


_DEFAULTS = r"""
import datetime, os, sys, time
sys.path.insert(0, {repo!r})
sys.argv = ["bench.py"]
import importlib.util
spec = importlib.util.spec_from_file_location("rt_bench", {bench!r})
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
import torch, torch.distributed as dist
rank = int(os.environ["RANK"])
args = b.parse(["--gpus", "2"])  # the default timeouts
pg = datetime.timedelta(seconds=args.pg_timeout)
dist.init_process_group("gloo", timeout=pg)
class C:
    world, distributed, pg = 2, True, None
    def renew_group(self):
        self.pg = dist.new_group(backend="gloo", timeout=pg)
c = C()
c.rank, c.torch, c.dist = rank, torch, dist
state = {{"assembly": {{"rccl_p2p": {{"ms_per_step": 0.25, "frame_check": "bit-exact"}}}}}}
ph = b.Phases(c, args.phase_deadline, lambda: b.multi_line(args, c, state), args.pg_timeout)
t0 = time.monotonic()
def one_rank():
    if rank == 1:
        raise RuntimeError("rank 1 only")
    dist.barrier(group=c.pg)  # unmatched: fails after --pg-timeout
ph.run("xgmi_peer_store", one_rank, state["assembly"])
def later():
    t = torch.ones(1)
    dist.all_reduce(t, group=c.pg)  # the renewed group lines up again
    return {{"ms_per_step": 0.5, "frame_check": "bit-exact", "sum": float(t.item())}}
ph.run("xgmi_peer_store_balanced", later, state["assembly"])
ph.run("roofline", lambda: {{"frac": 0.5, "after_s": round(time.monotonic() - t0, 1)}}, state)
ph.emit()
dist.destroy_process_group()
sys.exit(b.exit_status(state))
"""


def test_one_rank_failure_recovers_at_default_timeouts(tmp_path):
    """at the DEFAULT --pg-timeout / --phase-deadline, a phase
    that fails on one rank while the other blocks in its collective ends by
    the collective's timeout, before the watchdog: the failure is recorded,
    the later phases (xgmi_peer_store_balanced, roofline) still run, and
    every rank exits 0 (every phase completed, the line has a value)."""
    import json
    import subprocess
    import time

    b = _bench()
    a = b.parse(["--gpus", "2"])
    # the collective must give up well before the watchdog would fire
    assert a.pg_timeout + 30 <= a.phase_deadline
    code = _DEFAULTS.format(repo=str(REPO), bench=str(REPO / "bench.py"))
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env, cwd=tmp_path))
    outs = [p.communicate(timeout=a.phase_deadline + 60) for p in procs]
    assert time.monotonic() - t0 < a.phase_deadline  # no watchdog involved
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 0, (p.returncode, err[-2000:])
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert "error" in line["assembly"]["xgmi_peer_store"]  # rank 0 records its timeout
    assert line["assembly"]["xgmi_peer_store_balanced"]["sum"] == 2.0
    assert line["roofline"]["frac"] == 0.5
    assert line["phase_errors"] == ["assembly.xgmi_peer_store"]


def test_exit_status():
    b = _bench()
    ok = {"assembly": {"rccl_p2p": {"ms_per_step": 0.5, "frame_check": "bit-exact"},
                       "xgmi_peer_store": {"error": "rank 1: boom"}}}
    assert b.exit_status(ok) == 0  # a caught exception is a completed phase
    bad = {"assembly": {"rccl_p2p": {"ms_per_step": 0.5, "frame_check": "MISMATCH"}}}
    assert b.exit_status(bad) == b.EXIT_NO_VALUE != 0
    assert b.exit_status({}) == b.EXIT_NO_VALUE


def _launch(args, timeout):
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True,
                          text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_starts_its_own_ranks(world):
    """`python bench.py --gpus N` with no launcher (missing #1):
    bench.py starts N rank processes itself (RANK / WORLD_SIZE / MASTER_* set,
    127.0.0.1, before any GPU call), and exactly one JSON line comes out, from
    rank 0, with n_gpus N, a bit-exact assembly over gloo and the scaling
    contract's keys (scaling_assembled, scaling_weak, scaling_note beside
    scaling_host_frame).  --selftest-cpu: the bands are a known pattern, not
    traced (no GPU here); the GPU rehearsal of the same launcher is in
    tests/test_gpu_configs.py."""
    import json
    p = _launch(["--gpus", str(world), "--selftest-cpu", "--steps", "3", "--warmup", "1",
                 "--width", "40", "--height", "37"], timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    # stdout is the line and nothing else (gloo's "[Gloo] Rank ..." logging
    # and any other fd-1 output go to stderr)
    lines = [s for s in p.stdout.splitlines() if s.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["value"] > 0
    asm = line["assembly"]["rccl_p2p"]
    assert asm["frame_check"] == "bit-exact" and sum(asm["rows_per_rank"]) == 37
    t1, tn, tw = line["one_gpu"]["ms_per_step"], line["ms_per_step"], \
        line["weak_scaling"]["ms_per_step"]
    # (both rounded to 4 decimals in the line)
    assert line["scaling_assembled"] == pytest.approx(t1 / tn, rel=1e-3, abs=1e-4)
    assert line["scaling_weak"] == pytest.approx(world * t1 / tw, rel=1e-3, abs=1e-4)
    assert "scaling_host_frame" in line["scaling_note"]
    assert "scaling_host_frame" in line and "phase_errors" not in line


def test_bench_own_ranks_hang_exit_status():
    """A rank hanging inside a phase under bench.py's own launcher: the ranks'
    watchdogs end the run, rank 0 prints one line naming the phase, and the
    parent exits with status 3 (EXIT_HUNG), never 0."""
    import json
    b = _bench()
    p = _launch(["--gpus", "2", "--selftest-cpu", "--steps", "3", "--warmup", "1", "--width", "40",
                 "--height", "37", "--phase-deadline", "5", "--pg-timeout", "100",
                 "--fail-assembly", "rccl_p2p:1:hang"], timeout=120)
    assert p.returncode == b.EXIT_HUNG == 3, p.stderr[-3000:]
    lines = [s for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert "timeout" in line["assembly"]["rccl_p2p"]["error"]
    assert line["phase_errors"] == ["assembly.rccl_p2p"] and line["value"] is None


def test_frame_check_ref_against_fixture(tmp_path):
    """The bench's frame_check_ref (missing #2): the frame's
    FNV-1a-64 against the committed fixture of exactly that workload (frame
    size and scene arrays), per format; a changed word is a MISMATCH, another
    scene has no fixture (None).  A CPU-side mock of the device frame."""
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    b = _bench()
    w, h = 48, 40
    scene = pkg.Scene.synthetic(w, h, 5, 2, seed=7, k=0.2)
    frame = np.random.default_rng(1).integers(-300, 300, (h, w, 4)).astype(np.int32)
    tex = pkg.pack_rgba8(frame)
    np.savez_compressed(tmp_path / f"mock_{w}x{h}.npz", width=np.int32(w), height=np.int32(h),
                        fnv1a64=np.uint64(pkg.fnv1a64(frame)),
                        fnv1a64_rgba8=np.uint64(pkg.fnv1a64(tex)),
                        **{n: getattr(scene, n) for n in b.SCENE_ARRAYS})
    r = b.frame_check_ref(pkg, frame, scene, w, h, "i32x4", tmp_path)
    assert r["frame_check_ref"] == "bit-exact" and f"mock_{w}x{h}.npz" in r["source"]
    assert b.frame_check_ref(pkg, tex, scene, w, h, "rgba8", tmp_path)["frame_check_ref"] == \
        "bit-exact"
    bad = frame.copy()
    bad[h - 1, w - 1, 2] += 1
    assert b.frame_check_ref(pkg, bad, scene, w, h, "i32x4", tmp_path)["frame_check_ref"] == \
        "MISMATCH"
    other = pkg.Scene.synthetic(w, h, 5, 2, seed=8, k=0.2)
    assert b.frame_check_ref(pkg, frame, other, w, h, "i32x4", tmp_path)["frame_check_ref"] is None
    # the headline workload has its fixture, in both formats
    a = b.parse([])
    k = a.width / 640.0
    c3 = pkg.Scene.synthetic(a.width, a.height, a.spheres, a.cubes, seed=a.seed, k=k)
    for fmt in ("i32x4", "rgba8"):
        want, src = b.reference_hash(c3, a.width, a.height, fmt, a.golden)
        assert want is not None and src == "config3_4096x4096.npz", src


def test_sustained_window_is_a_fixed_frame_count():
    b = _bench()
    a = b.parse([])
    assert a.sustained >= 500  # default on, independent of --steps
    assert b.parse(["--sustained", "0"]).sustained == 0

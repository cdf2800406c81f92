"""Benchmark: Mrays/s of the MI355X ray tracer on BASELINE.json's config.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Workload (BASELINE config 3, the headline): one 4096x4096 frame, 256
spheres + 64 cubes, dense synthetic scene (seed 3, k =
4096/640), int32x4 framebuffer (16 B/ray), scene resident in HBM.

A step at N=1: one pass of the hot path over the frame -- the prep, bin and
trace kernels of librt_hip.so writing the frame to HBM (rt_render_device).

A step at N>1 (strong scaling): the SAME frame split into
N contiguous row bands, one per rank, and the frame assembled on rank 0.  The
clock runs from the barrier before the renders to the assembled frame on rank
0 (max over ranks), so the transfer is inside `value`.  Two assemblies are
measured and the faster is `value` (both are reported, each checked
bit-exactly against a one-GPU render of the whole frame on rank 0):
  rccl_p2p         every rank renders its band locally, then RCCL
                   point-to-point sends land it in rank 0's frame rows
                   (rank 0 renders its own band in place);
  xgmi_peer_store  rank 0's frame is mapped into every rank (IPC handle,
                   rt_shared_open) and each rank's trace kernel stores its
                   band straight into it over xGMI; a one-element RCCL
                   all-reduce after the render tells rank 0 all bands landed.
Also reported at N>1: the render/assembly split, the RGBA8 Texture form of
the same assembly (4 B/ray, the north_star's Texture), BASELINE config 4
(8192^2, 192 + 64, seed 4) with the same assembly, and weak scaling (each
rank renders a 4096x4096 band of a 4096 x 4096N frame, no assembly) as a
secondary key -- never as `value`.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
import __graft_entry__  # noqa: E402

METRIC = "Mrays/sec (primary) at 4096×4096, 1/2/4/8 MI355X; % HBM-write roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured copy
BYTES_PER_RAY = {"i32x4": 16, "rgba8": 4}
# BASELINE.json configs by (width, height, spheres, cubes)
CONFIG_NAMES = {(1920, 1080, 16, 4): "config2", (4096, 4096, 256, 64): "config3",
                (8192, 8192, 192, 64): "config4", (16384, 16384, 4096, 0): "config5"}
CONFIG4 = dict(width=8192, height=8192, spheres=192, cubes=64, seed=4)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--warmup-ms", type=float, default=50.0,
                    help="the untimed warmup also runs until this much wall time of GPU load "
                         "has passed (the clock ramps up over tens of milliseconds)")
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096, help="frame rows (all ranks together)")
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--cubes", type=int, default=64)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--k", type=float, default=None, help="object scale (default width/640)")
    ap.add_argument("--format", choices=sorted(BYTES_PER_RAY), default="i32x4")
    ap.add_argument("--cpu-rows", type=int, default=1,
                    help="CPU baseline samples every Nth row of the frame (1 = the whole "
                         "frame: ~4 s for config 3 on 16 threads)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every CPU this job may use: the "
                         "affinity set, capped by the job's CPU share OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the end-to-end rt_render (host buffers) measurement")
    ap.add_argument("--no-extras", action="store_true",
                    help="time only the headline workload (N=1: no RGBA8 Texture line; "
                         "N>1: no Texture / config 4 / weak-scaling keys)")
    ap.add_argument("--path", choices=("auto", "binned", "generic"), default="auto",
                    help="kernel path: generic = the brute-force per-pixel kernel (every ray "
                         "against every primitive), for the compute-bound comparison")
    ap.add_argument("--trace-mode", type=int, default=0,
                    help="diagnostics ablation: 1 = stores only, 2 = no per-pixel tests")
    ap.add_argument("--pmc", default=str(REPO / "profiles" / "r02_pmc_config3.json"),
                    help="committed PMC summary to read `traffic` from")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank renders on cuda:0 and the "
                         "collectives run over gloo on host copies")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# arithmetic shared by the N=1 and N>1 lines (checked by tests/test_bench.py)
# ---------------------------------------------------------------------------
def mrays_per_s(rays: int, ms: float) -> float:
    return rays / (ms * 1e-3) / 1e6


def bytes_to_root(width: int, height: int, world: int, fmt: str, root: int = 0) -> int:
    """Framebuffer bytes that must reach the root: every band but its own."""
    from opencl_ray_tracer_amd.rowbands import band_rows

    rb, re = band_rows(height, world, root)
    return BYTES_PER_RAY[fmt] * width * (height - (re - rb))


def pick_value(assemblies: dict):
    """The fastest assembly whose frame was bit-exact: (name, entry)."""
    ok = [(v["ms_per_step"], k) for k, v in assemblies.items()
          if v.get("ms_per_step") is not None and v.get("frame_check") == "bit-exact"]
    if not ok:
        raise RuntimeError(f"no assembly produced a bit-exact frame: {assemblies}")
    ms, name = min(ok)
    return name, assemblies[name]


def cpu_threads(requested: int) -> tuple:
    """(threads to use, description).  0 = every CPU this job may run on:
    the affinity set, capped by the job's CPU share where the launcher
    states one (OMP_NUM_THREADS; the GPU box grants 16 CPUs per GPU)."""
    affinity = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    n = affinity
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    if requested > 0:
        n = min(requested, affinity)
    return max(1, n), {"affinity_cpus": affinity, "os_cpu_count": os.cpu_count(),
                       "omp_num_threads": share}


class Ctx:
    """Process / device / collective plumbing of one bench run."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus and self.world == 1 and args.gpus != 1:
            raise SystemExit(f"--gpus {args.gpus} needs torchrun with {args.gpus} ranks")
        self.distributed = self.world > 1
        self.backend = "gloo" if args.rehearse else args.backend
        self.gpu = 0 if args.rehearse else local
        if self.distributed:
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            torch.cuda.set_device(self.gpu)
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.gpu))
            else:
                dist.init_process_group("gloo")
        self.dev = torch.device("cuda", self.gpu)
        # collectives move GPU tensors with RCCL, host copies with gloo
        self.coll_dev = self.dev if self.backend == "nccl" else torch.device("cpu")
        # A real stream object: the legacy default stream's handle is 0, which
        # the C ABI reads as "the context's own stream".
        self.stream = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream)

    def barrier(self):
        if self.distributed:
            self.dist.barrier()

    def clock_ramp(self, step, ms: float) -> int:
        """Untimed: repeat step() (in chunks, synchronised) until `ms` of
        wall time under load has passed, so the timed region runs at the
        GPU's steady clock (back-to-back trace replays start at 62 us and
        settle near 51 us).  Returns the steps run."""
        n, t0 = 0, time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(16):
                step()
            n += 16
            self.sync()
        return n

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def max_over_ranks(self, v: float) -> float:
        if not self.distributed:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.coll_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def timed(self, step, steps: int, events=None) -> float:
        """`steps` calls of step() between barrier + sync; this rank's clock
        stops at its own sync (the trailing barrier's latency is outside it);
        returns the max over ranks of wall ms per step.  `events`: a pair of
        torch.cuda.Event recorded on the stream around the K steps."""
        self.sync()
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        if events:
            events[0].record(self.stream)
        for _ in range(steps):
            step()
        if events:
            events[1].record(self.stream)
        self.sync()
        wall = (time.perf_counter() - t0) * 1e3 / steps
        self.barrier()
        return self.max_over_ranks(wall)


def device_scene(pkg, c: Ctx, width, height, spheres, cubes, seed, k):
    scene = pkg.Scene.synthetic(width, height, spheres, cubes, seed=seed, k=k)
    t = {name: c.torch.from_numpy(np.ascontiguousarray(getattr(scene, name))).to(c.dev)
         for name in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                      "cube_colours")}
    ds = {name: v.data_ptr() for name, v in t.items()}
    ds.update(num_spheres=scene.num_spheres, num_cubes=scene.num_cubes)
    ds["_keep"] = t
    return scene, ds


def frame_tensor(c: Ctx, rows, width, fmt):
    shape = (rows, width, 4) if fmt == "i32x4" else (rows, width)
    return c.torch.empty(shape, dtype=c.torch.int32, device=c.dev)


# ---------------------------------------------------------------------------
# N = 1
# ---------------------------------------------------------------------------
def run_single(args, c: Ctx, pkg):
    torch = c.torch
    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640.0
    scene, ds = device_scene(pkg, c, w, h, args.spheres, args.cubes, args.seed, k)
    rt = pkg.RayTracer(c.gpu)
    rt.set_trace_mode(args.trace_mode)
    out = frame_tensor(c, h, w, args.format)
    # ctypes arguments built once; each step enqueues prep + coarse + trace
    step = rt.bind_render_device(ds, w, h, (0, h), out.data_ptr(), fmt=args.format,
                                 path=args.path, stream=c.stream.cuda_stream)
    for _ in range(args.warmup):
        step()
    ramp_steps = c.clock_ramp(step, args.warmup_ms)
    c.sync()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    # The timed region: K steps, nothing attached to the kernels.
    wall_ms = c.timed(step, args.steps, events=(ev0, ev1))
    event_ms = ev0.elapsed_time(ev1) / args.steps

    # Per-kernel durations: the same K steps again with start/stop HIP events
    # attached to each kernel's own dispatch packet on the launch stream
    # (hipExtLaunchKernelGGL; events from a pool grown in an untimed pass).
    # Not the timed region itself: with the events attached the wall time per
    # step grows by 25-40%, while the kernels' own durations agree with
    # rocprofv3's.
    rt.profile(True)
    for _ in range(args.steps):  # untimed: grows the event pool to K renders
        step()
    c.sync()
    rt.profile_read()
    rt.profile(True)
    prof_wall_ms = c.timed(step, args.steps)
    prof = rt.profile_read()
    rt.profile(False)
    n = max(prof["renders"], 1)
    trace_ms, prep_ms, bin_ms = prof["trace_ms"] / n, prof["prep_ms"] / n, prof["bin_ms"] / n

    rays = w * h
    algo_bytes = BYTES_PER_RAY[args.format] * rays
    achieved = algo_bytes / (trace_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = Path(args.pmc)
    # measured for this workload of the real binned trace kernel only
    if args.path != "generic" and args.trace_mode == 0 and pmc_path.exists():
        try:
            pmc = json.loads(pmc_path.read_text())
            if pmc.get("config") == [w, h, args.spheres, args.cubes, args.seed, args.format]:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    host = None
    if not args.no_host_path:
        # the reference's timer scope (MainState.cpp:
        # 662-894: scene upload, render, blocking readback of the frame),
        # through the synchronous host-buffer entry point rt_render.  Never
        # `value`: it includes the PCIe copy of the whole frame.
        host_buf = np.empty(tuple(out.shape), np.int32 if args.format == "i32x4" else np.uint32)

        def host_runs():
            runs = [rt.render(scene, w, h, fmt=args.format, out=host_buf)[1] for _ in range(4)]
            best = min(runs[1:], key=lambda t: t.total_us)
            return {"total_ms": round(best.total_us / 1e3, 3),
                    "upload_ms": round(best.upload_us / 1e3, 3),
                    "kernel_ms": round(best.kernel_us / 1e3, 3),
                    "download_ms": round(best.download_us / 1e3, 3),
                    "mrays_end_to_end": round(rays / best.total_us, 1)}
        host = {"scope": "rt_render: scene upload + kernels + frame download (PCIe) into a "
                         "reused host buffer", **host_runs()}
        # the same into a page-locked buffer (rt_host_register): direct DMA
        pkg.host_register(host_buf)
        host["registered"] = host_runs()
        pkg.host_unregister(host_buf)
        # the reference's own call passes rayOrigins (MainState.cpp:44-50,
        # uploaded at :841-855): the grid is uploaded, recognised on the
        # device, and the binned path still runs
        ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
        grid = np.stack([xs, ys, np.zeros_like(xs), np.ones_like(xs)], -1)
        del ys, xs
        runs = [rt.render(scene, w, h, fmt=args.format, out=host_buf, ray_origins=grid)[1]
                for _ in range(3)]
        best = min(runs[1:], key=lambda t: t.total_us)
        host["explicit_origins"] = {"total_ms": round(best.total_us / 1e3, 3),
                                    "upload_ms": round(best.upload_us / 1e3, 3),
                                    "kernel_ms": round(best.kernel_us / 1e3, 3),
                                    "download_ms": round(best.download_us / 1e3, 3),
                                    "path": best.path}
        del grid, host_buf
        # north_star's consumer is the Texture (MainState.cpp:1023-1037, packed
        # on the host after the int32x4 readback): packed on the device
        # instead, the download is 4 B per pixel, into a page-locked buffer
        if args.format == "i32x4" and not args.no_extras:
            tex_buf = np.empty((h, w), np.uint32)
            pkg.host_register(tex_buf)
            runs = [rt.render(scene, w, h, fmt="rgba8", out=tex_buf)[1] for _ in range(4)]
            pkg.host_unregister(tex_buf)
            best = min(runs[1:], key=lambda t: t.total_us)
            host["texture_rgba8_registered"] = {
                "total_ms": round(best.total_us / 1e3, 3),
                "upload_ms": round(best.upload_us / 1e3, 3),
                "kernel_ms": round(best.kernel_us / 1e3, 3),
                "download_ms": round(best.download_us / 1e3, 3),
                "mrays_end_to_end": round(rays / best.total_us, 1)}
            del tex_buf

    # Second workload: the same frame in the Texture's RGBA8 packing
    # (MainState.cpp:1023-1037, north_star's Texture), 4 B/ray, with its own
    # roofline.  Timed the same way; never `value`.
    texture = None
    if args.format == "i32x4" and not args.no_extras and args.trace_mode == 0:
        tex = frame_tensor(c, h, w, "rgba8")
        tstep = rt.bind_render_device(ds, w, h, (0, h), tex.data_ptr(), fmt="rgba8",
                                      path=args.path, stream=c.stream.cuda_stream)
        for _ in range(args.warmup):
            tstep()
        t_wall = c.timed(tstep, args.steps)
        rt.profile(True)
        for _ in range(args.steps):
            tstep()
        tp = rt.profile_read()
        rt.profile(False)
        t_trace = tp["trace_ms"] / max(tp["renders"], 1)
        t_bytes = BYTES_PER_RAY["rgba8"] * w * h
        t_ach = t_bytes / (t_trace * 1e-3) / 1e9
        texture = {"format": "rgba8", "ms_per_step": round(t_wall, 4),
                   "value": round(mrays_per_s(w * h, t_wall), 1), "unit": "Mrays/s",
                   "roofline": {"bound": "hbm", "achieved": round(t_ach, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(t_ach / HBM_PEAK_GBS, 4),
                                "kernel": kernel_name(args), "kernel_ms": round(t_trace, 4),
                                "algo_bytes_per_launch": t_bytes,
                                "note": "bound by per-wave test chains, not HBM (DESIGN.md §3, profiles/r02/pmc_mix)"}}
        del tex

    cpu = None if args.no_cpu_baseline else cpu_baseline(args, scene, w, h)
    workload = CONFIG_NAMES.get((w, h, args.spheres, args.cubes), "custom")
    kernel = kernel_name(args)
    rt.close()
    return {
        "metric": METRIC, "value": round(mrays_per_s(rays, wall_ms), 1), "unit": "Mrays/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall_ms, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{workload}: {w}x{h} frame, {args.spheres} spheres + "
                               f"{args.cubes} cubes, dense k={k:.2f}, seed {args.seed}",
                   "width": w, "height": h, "spheres": args.spheres, "cubes": args.cubes,
                   "format": args.format, "parallelism": "1 GPU (the whole frame)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": kernel, "kernel_ms": round(trace_ms, 4),
                     "prep_ms": round(prep_ms, 4), "bin_ms": round(bin_ms, 4),
                     "algo_bytes_per_launch": algo_bytes},
        "event_ms_per_step": round(event_ms, 4),
        "profiled_pass_ms_per_step": round(prof_wall_ms, 4),
        "clock_ramp": {"ms": args.warmup_ms, "untimed_steps": ramp_steps},
        "texture_rgba8": texture,
        "cpu_baseline": cpu,
        "host_path": host,
    }


def kernel_name(args) -> str:
    """The dominant kernel: scenes of at most 512 primitives take
    trace_small_kernel."""
    return ("generic_kernel" if args.path == "generic" else
            "trace_small_kernel" if 0 < args.spheres + 12 * args.cubes <= 512 else
            "trace3_kernel")


def cpu_baseline(args, scene, w, h):
    """The oracle (the serial CPU path restated, oracle/rt_oracle.c) timed on
    this box's host CPUs: all CPUs the job may use, plus one core."""
    sys.path.insert(0, str(REPO / "tests"))
    from oracle_lib import Oracle  # CPU baseline only

    threads, cpus = cpu_threads(args.cpu_threads)
    orc = Oracle()
    sample_rows = list(range(0, h, args.cpu_rows))
    c0 = time.perf_counter()
    orc.trace_rows(scene, w, h, sample_rows, threads=threads)
    c_s = time.perf_counter() - c0
    # SURVEY.md §8d CPU baseline (a): the serial path on one core, on a
    # deterministic row subset (every 32nd row of the same frame)
    serial_rows = list(range(0, h, 32))
    c1 = time.perf_counter()
    orc.trace_rows(scene, w, h, serial_rows, threads=1)
    s_s = time.perf_counter() - c1
    return {"value": round(len(sample_rows) * w / c_s / 1e6, 3), "unit": "Mrays/s",
            "cores": threads, "kind": "port",
            "host_cpus": cpus,
            "sample": (f"the whole {w}x{len(sample_rows)} frame" if args.cpu_rows == 1 else
                       f"{len(sample_rows)} rows (every {args.cpu_rows}th) x {w} px")
                      + f" of the same scene, oracle/rt_oracle.c orc_trace_rows_mt on "
                        f"{threads} threads (one row band per thread), {c_s:.1f} s wall",
            "serial_1core": {"value": round(len(serial_rows) * w / s_s / 1e6, 3),
                             "sample": f"every 32nd row ({len(serial_rows)} rows x {w} px), "
                                       f"1 thread, {s_s:.1f} s wall"}}


# ---------------------------------------------------------------------------
# N > 1: strong scaling of one frame, assembled on rank 0
# ---------------------------------------------------------------------------
class Assembly:
    """One frame (width x height, `fmt`) split into row bands over the ranks
    and assembled on rank 0 by `how` ("rccl_p2p" or "xgmi_peer_store")."""

    def __init__(self, c: Ctx, pkg, rt, ds, width, height, fmt, how, path="auto", bands=None):
        from opencl_ray_tracer_amd import rowbands

        self.c, self.rt, self.how, self.fmt = c, rt, how, fmt
        self.width, self.height = width, height
        self.rowbands = rowbands
        self.bands = bands or [rowbands.band_rows(height, c.world, r) for r in range(c.world)]
        self.rb, self.re = self.bands[c.rank]
        self.root = c.rank == 0
        px_bytes = BYTES_PER_RAY[fmt]
        self.row_bytes = width * px_bytes
        self.error = None
        self.shared = None
        torch = c.torch
        stream = c.stream.cuda_stream
        empty = self.re <= self.rb
        if how == "rccl_p2p":
            self.frame = frame_tensor(c, height, width, fmt) if self.root else None
            self.band = (self.frame[self.rb:self.re] if self.root
                         else frame_tensor(c, self.re - self.rb, width, fmt))
            if c.backend != "nccl":  # rehearsal: gloo moves host copies
                self.host_frame = (torch.empty(self.frame.shape, dtype=torch.int32)
                                   if self.root else None)
            dst = self.band.data_ptr()
        else:
            self.shared = rowbands.SharedFrame(rt, self.row_bytes * height, self.row_bytes,
                                               c.rank, handle_device=c.coll_dev)
            if not self.shared.ok:
                self.error = self.shared.error
                return
            self.signal = torch.zeros(1, dtype=torch.int32, device=c.coll_dev)
            self.frame = None
            if self.root:  # a torch view of the shared frame, for the check
                self.frame = _wrap_device(c, self.shared.ptr, height, width, fmt)
            dst = self.shared.ptr_of_row(self.rb)
        self.render = (None if empty else
                       rt.bind_render_device(ds, width, height, (self.rb, self.re), dst, fmt=fmt,
                                             path=path, stream=stream))

    def render_only(self):
        if self.render:
            self.render()

    def assemble_only(self):
        c = self.c
        if self.how == "rccl_p2p":
            if c.backend == "nccl":
                for q in self.rowbands.assemble_frame(self.frame, self.band, self.height, c.world,
                                                      c.rank, async_op=True, bands=self.bands):
                    q.wait()  # the stream waits; the host does not
            else:
                c.sync()
                hf = self.host_frame
                self.rowbands.assemble_frame(hf, self.band.cpu(), self.height, c.world, c.rank,
                                             bands=self.bands)
                if self.root:  # the other ranks' rows, host -> device
                    for r in range(1, c.world):
                        rb, re = self.bands[r]
                        self.frame[rb:re].copy_(hf[rb:re])
        else:
            # every band landed in rank 0's frame once every rank's render
            # finished: a one-element all-reduce behind the render on each
            # rank's stream (RCCL), or a host barrier after a sync (gloo)
            if c.backend == "nccl":
                c.dist.all_reduce(self.signal, async_op=True).wait()
            else:
                c.sync()
                c.dist.barrier()

    def step(self):
        self.render_only()
        self.assemble_only()

    def check(self, ds) -> str:
        """Rank 0: the assembled frame against a one-GPU render of the whole
        frame (bit-exact or not); broadcast so every rank agrees."""
        c = self.c
        ok = c.torch.ones(1, dtype=c.torch.int32, device=c.coll_dev)
        if self.root:
            c.sync()
            ref = frame_tensor(c, self.height, self.width, self.fmt)
            self.rt.bind_render_device(ds, self.width, self.height, (0, self.height),
                                       ref.data_ptr(), fmt=self.fmt,
                                       stream=c.stream.cuda_stream)()
            c.sync()
            ok.fill_(int(c.torch.equal(ref, self.frame)))
            del ref
        c.dist.broadcast(ok, 0)
        return "bit-exact" if int(ok.item()) else "MISMATCH"

    def close(self):
        if self.shared is not None:
            self.c.sync()
            self.shared.close()


def _wrap_device(c: Ctx, ptr: int, rows, width, fmt):
    """A torch int32 tensor viewing `rows` x `width` pixels at device address
    `ptr` (memory owned by librt_hip.so, e.g. the shared frame)."""
    torch = c.torch
    shape = (rows, width, 4) if fmt == "i32x4" else (rows, width)

    class _Arr:
        __cuda_array_interface__ = {"shape": shape, "typestr": "<i4", "data": (ptr, False),
                                    "version": 2, "strides": None}
    return torch.as_tensor(_Arr(), device=c.dev)


def measure_assembly(args, c, pkg, rt, ds, width, height, fmt, how, split=False, bands=None):
    a = Assembly(c, pkg, rt, ds, width, height, fmt, how, bands=bands)
    if a.error:
        a.close()  # frees what the root allocated; a barrier on every rank
        return {"ms_per_step": None, "error": a.error}
    for _ in range(args.warmup):
        a.step()
    c.sync()
    ms = c.timed(a.step, args.steps)
    rb0, re0 = a.bands[0]
    res = {"ms_per_step": round(ms, 4),
           "mrays": round(mrays_per_s(width * height, ms), 1),
           "bytes_to_root": BYTES_PER_RAY[fmt] * width * (height - (re0 - rb0))}
    if split:
        render_ms = c.timed(a.render_only, args.steps)
        # rccl_p2p: the local render; xgmi_peer_store: the render whose
        # stores go over xGMI into rank 0's frame, without the signal
        res["render_ms"] = round(render_ms, 4)
        if how == "rccl_p2p":
            # the assembly alone (bands already rendered): its link rate
            asm_ms = c.timed(a.assemble_only, args.steps)
            res["assemble_ms"] = round(asm_ms, 4)
            res["assemble_gbs_into_root"] = round(res["bytes_to_root"] / (asm_ms * 1e-3) / 1e9, 1)
    res["frame_check"] = a.check(ds)
    res["rows_per_rank"] = [re - rb for rb, re in a.bands]
    a.close()
    return res


def calibrate_peer_store(args, c, pkg, rt, ds, width, height, fmt):
    """Each rank's cost model t(n) = a + s n for rendering n rows into rank
    0's shared frame (xGMI stores; rank 0's own stores are local), from two
    band sizes rendered by all ranks at once.  Returns [(a_r, s_r)] in
    seconds, rows, identical on every rank."""
    from opencl_ray_tracer_amd import rowbands

    row_bytes = width * BYTES_PER_RAY[fmt]
    shared = rowbands.SharedFrame(rt, row_bytes * height, row_bytes, c.rank,
                                  handle_device=c.coll_dev)
    try:
        if not shared.ok:
            return None
        times = []
        sizes = [max(16, height // c.world), max(16, height // (2 * c.world))]
        for n in sizes:
            rb = c.rank * n
            step = rt.bind_render_device(ds, width, height, (rb, rb + n), shared.ptr_of_row(rb),
                                         fmt=fmt, stream=c.stream.cuda_stream)
            for _ in range(args.warmup):
                step()
            c.sync()
            c.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            c.sync()
            times.append((time.perf_counter() - t0) / args.steps)
            c.barrier()
        (n1, t1), (n2, t2) = zip(sizes, times)
        slope = (t1 - t2) / (n1 - n2)
        if not slope > 0.0:  # noise: the larger band alone, no fixed cost
            slope, fixed = t1 / n1, 0.0
        else:
            fixed = max(0.0, t1 - slope * n1)
        mine = c.torch.tensor([fixed, slope], dtype=c.torch.float64, device=c.coll_dev)
        every = [c.torch.empty_like(mine) for _ in range(c.world)]
        c.dist.all_gather(every, mine)
        return [(float(e[0]), float(e[1])) for e in every]
    finally:
        c.sync()
        shared.close()


def measure_host_frame(args, c: Ctx, pkg, rt, scene, w, h, fmt="i32x4"):
    """The reference's own consumer, a host frame (`pixels`, MainState.cpp:
    215/676, read back at :876-907), filled by N GPUs at once: every rank
    calls rt_render (the executeRayTracerOpenCL replacement: scene upload,
    render, download -- the app's timer scope, :662-894) for its band,
    straight into its rows of ONE page-locked host frame shared by the ranks
    (POSIX shared memory), each over its own GPU's PCIe link.  A step ends
    when every rank's rows are in (barrier).  Checked bit-exactly on rank 0
    against a one-GPU device render."""
    from multiprocessing import resource_tracker, shared_memory

    from opencl_ray_tracer_amd.rowbands import band_rows

    shape = (h, w, 4) if fmt == "i32x4" else (h, w)
    nbytes = BYTES_PER_RAY[fmt] * w * h
    rb, re = band_rows(h, c.world, c.rank)
    shm = frame = None
    name = [None]
    try:
        if c.rank == 0:
            shm = shared_memory.SharedMemory(create=True, size=nbytes)
            name = [shm.name]
        c.dist.broadcast_object_list(name, 0)
        if c.rank != 0:
            shm = shared_memory.SharedMemory(name=name[0])
            resource_tracker.unregister(shm._name, "shared_memory")  # rank 0 unlinks it
        frame = np.ndarray(shape, np.int32 if fmt == "i32x4" else np.uint32, buffer=shm.buf)
        pkg.host_register(frame)
        band = frame[rb:re]

        def step():
            if re > rb:
                rt.render(scene, w, h, rows=(rb, re), fmt=fmt, out=band)
            c.dist.barrier()
        for _ in range(max(1, args.warmup)):
            step()
        ms = c.timed(step, args.steps)
        ok = c.torch.ones(1, dtype=c.torch.int32, device=c.coll_dev)
        if c.rank == 0:
            keep, ds = device_scene_from(c, scene)
            ref = frame_tensor(c, h, w, fmt)
            rt.bind_render_device(ds, w, h, (0, h), ref.data_ptr(), fmt=fmt,
                                  stream=c.stream.cuda_stream)()
            c.sync()
            ok.fill_(int(np.array_equal(ref.cpu().numpy().view(frame.dtype), frame)))
            del ref, keep
        c.dist.broadcast(ok, 0)
        pkg.host_unregister(frame)
        return {"scope": "rt_render per rank (scene upload + render + band download over its "
                         "own PCIe link) into one shared page-locked host frame, then a barrier",
                "format": fmt, "ms_per_step": round(ms, 4),
                "mrays_end_to_end": round(mrays_per_s(w * h, ms), 1),
                "host_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1),
                "frame_check": "bit-exact" if int(ok.item()) else "MISMATCH"}
    finally:
        del frame
        if shm is not None:
            shm.close()
            c.dist.barrier()
            if c.rank == 0:
                shm.unlink()


def device_scene_from(c: Ctx, scene):
    t = {name: c.torch.from_numpy(np.ascontiguousarray(getattr(scene, name))).to(c.dev)
         for name in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                      "cube_colours")}
    ds = {name: v.data_ptr() for name, v in t.items()}
    ds.update(num_spheres=scene.num_spheres, num_cubes=scene.num_cubes)
    return t, ds


def measure_assemblies(args, c, pkg, rt, ds, w, h, fmt, split=False):
    """The frame assembled on rank 0 three ways: equal bands by RCCL
    point-to-point, equal bands by xGMI peer stores, and cost-balanced bands
    by xGMI peer stores.  The equal split makes every other rank wait on its
    link while rank 0's own rows need no transfer, so the balanced split
    sizes the bands by each rank's measured cost (render + stores into rank
    0's frame) for all ranks to finish together (rowbands.balanced_bands).
    Same frame, same end point, each checked bit-exactly."""
    from opencl_ray_tracer_amd import rowbands

    res = {how: measure_assembly(args, c, pkg, rt, ds, w, h, fmt, how, split=split)
           for how in ("rccl_p2p", "xgmi_peer_store")}
    costs = calibrate_peer_store(args, c, pkg, rt, ds, w, h, fmt)
    if costs is not None:
        bal = rowbands.balanced_bands(h, costs)
        res["xgmi_peer_store_balanced"] = measure_assembly(
            args, c, pkg, rt, ds, w, h, fmt, "xgmi_peer_store", split=split, bands=bal)
        res["xgmi_peer_store_balanced"]["cost_model_us"] = [
            {"fixed": round(a * 1e6, 2), "per_row": round(s * 1e6, 4)} for a, s in costs]
    return res


def run_multi(args, c: Ctx, pkg):
    from opencl_ray_tracer_amd import rowbands

    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640.0
    scene, ds = device_scene(pkg, c, w, h, args.spheres, args.cubes, args.seed, k)
    rt = pkg.RayTracer(c.gpu)
    rb, re = rowbands.band_rows(h, c.world, c.rank)
    # untimed: bring every GPU to its steady clock (renders of this rank's band)
    ramp_out = frame_tensor(c, max(re - rb, 1), w, args.format)
    ramp = (rt.bind_render_device(ds, w, h, (rb, re), ramp_out.data_ptr(), fmt=args.format,
                                  stream=c.stream.cuda_stream) if re > rb else (lambda: None))
    ramp_steps = c.clock_ramp(ramp, args.warmup_ms)
    del ramp_out

    assemblies = measure_assemblies(args, c, pkg, rt, ds, w, h, args.format, split=True)
    best, entry = pick_value(assemblies)
    ms = entry["ms_per_step"]

    # the trace kernel on this rank's band, local stores (the roofline of the
    # dominant kernel; rank 0's band)
    band = frame_tensor(c, max(re - rb, 1), w, args.format)
    step = (rt.bind_render_device(ds, w, h, (rb, re), band.data_ptr(), fmt=args.format,
                                  stream=c.stream.cuda_stream) if re > rb else (lambda: None))
    for _ in range(args.warmup):
        step()
    rt.profile(True)
    for _ in range(args.steps):
        step()
    prof = rt.profile_read()
    rt.profile(False)
    n = max(prof["renders"], 1)
    trace_ms = prof["trace_ms"] / n
    band_bytes = BYTES_PER_RAY[args.format] * w * (re - rb)
    achieved = band_bytes / (trace_ms * 1e-3) / 1e9 if trace_ms > 0 else 0.0
    del band

    extras = {}
    if not args.no_extras:
        # the Texture (RGBA8, MainState.cpp:1023-1037) assembled the same way
        extras["texture_rgba8"] = measure_assemblies(args, c, pkg, rt, ds, w, h, "rgba8")
        # BASELINE config 4: 8192^2, 192 + 64, row-tiled with the assembly
        c4 = CONFIG4
        k4 = c4["width"] / 640.0
        _, ds4 = device_scene(pkg, c, c4["width"], c4["height"], c4["spheres"], c4["cubes"],
                              c4["seed"], k4)
        extras["config4"] = {
            "workload": f"config4: {c4['width']}x{c4['height']} frame, {c4['spheres']} spheres + "
                        f"{c4['cubes']} cubes, dense k={k4:.1f}, seed {c4['seed']}, "
                        f"{c.world} row bands (BASELINE names 8 GPUs)",
            **measure_assemblies(args, c, pkg, rt, ds4, c4["width"], c4["height"], "i32x4")}
        del ds4
        # weak scaling (secondary): a 4096 x 4096N frame with N x (256 + 64)
        # primitives of the same density, rank r renders rows [4096 r, 4096 (r+1))
        hw = h * c.world
        _, dsw = device_scene(pkg, c, w, hw, args.spheres * c.world, args.cubes * c.world,
                              args.seed, k)
        outw = frame_tensor(c, h, w, args.format)
        stepw = rt.bind_render_device(dsw, w, hw, (c.rank * h, (c.rank + 1) * h),
                                      outw.data_ptr(), fmt=args.format,
                                      stream=c.stream.cuda_stream)
        for _ in range(args.warmup):
            stepw()
        wms = c.timed(stepw, args.steps)
        extras["weak_scaling"] = {
            "workload": f"{w}x{hw} frame, {args.spheres * c.world} spheres + "
                        f"{args.cubes * c.world} cubes; each rank renders {w}x{h} rows, "
                        f"no assembly",
            "ms_per_step": round(wms, 4), "mrays": round(mrays_per_s(w * hw, wms), 1)}
        del outw, dsw
        # the app's host frame filled by every GPU over its own PCIe link
        extras["host_frame"] = measure_host_frame(args, c, pkg, rt, scene, w, h)

    rt.close()
    workload = CONFIG_NAMES.get((w, h, args.spheres, args.cubes), "custom")
    return {
        "metric": METRIC, "value": round(mrays_per_s(w * h, ms), 1), "unit": "Mrays/s",
        "n_gpus": c.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{workload}: {w}x{h} frame, {args.spheres} spheres + "
                               f"{args.cubes} cubes, dense k={k:.2f}, seed {args.seed}",
                   "width": w, "height": h, "spheres": args.spheres, "cubes": args.cubes,
                   "format": args.format,
                   "parallelism": f"row-bands x{c.world}, frame assembled on rank 0 by {best}"
                                  + (" (rehearsal: shared cuda:0, gloo)" if args.rehearse
                                     else "")},
        "assembly": assemblies,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "trace3_kernel", "kernel_ms": round(trace_ms, 4),
                     "algo_bytes_per_launch": band_bytes,
                     "scope": "rank 0's band, local stores"},
        **extras,
        "clock_ramp": {"ms": args.warmup_ms, "untimed_steps": ramp_steps},
        "cpu_baseline": None,
    }


def main():
    args = parse()
    c = Ctx(args)
    pkg = __graft_entry__.load_package()
    line = run_multi(args, c, pkg) if c.distributed else run_single(args, c, pkg)
    if c.rank == 0:
        print(json.dumps(line), flush=True)
    if c.distributed:
        c.dist.destroy_process_group()


if __name__ == "__main__":
    main()

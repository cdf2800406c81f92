"""Benchmark: Mrays/s of the MI355X ray tracer on BASELINE.json's config.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

A step = one full pass of the hot path over one frame band: the prep, bin
and trace kernels of librt_hip.so on a scene already resident in HBM,
writing the int32x4 framebuffer band to HBM (rt_render_device).

Workload at N=1 is BASELINE config 3: 4096x4096, 256 spheres + 64 cubes,
dense synthetic scene (seed 3, k = 4096/640).  With N ranks
the image grows to 4096 x (4096 N) with N x (256 + 64) primitives of the
same density and rank r renders rows [4096 r, 4096 (r+1)): per-GPU work is
fixed (weak scaling), no collective sits in the timed region.  The RCCL
gather that assembles the frame on rank 0 (north_star's Texture assembly)
is measured separately and reported under "gather".

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--height", type=int, default=4096, help="rows per rank")
    ap.add_argument("--spheres", type=int, default=256, help="per rank")
    ap.add_argument("--cubes", type=int, default=64, help="per rank")
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--k", type=float, default=None, help="object scale (default width/640)")
    ap.add_argument("--format", choices=sorted(BYTES_PER_RAY), default="i32x4")
    ap.add_argument("--cpu-rows", type=int, default=1,
                    help="CPU baseline samples every Nth row of rank 0's band (1 = the "
                         "whole band: the full config-3 frame at N=1, ~4 s on 16 threads)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the end-to-end rt_render (host buffers) measurement")
    ap.add_argument("--path", choices=("auto", "binned", "generic"), default="auto",
                    help="kernel path: generic = the brute-force per-pixel kernel (every ray "
                         "against every primitive), for the compute-bound comparison")
    ap.add_argument("--trace-mode", type=int, default=0,
                    help="diagnostics ablation: 1 = stores only, 2 = no per-pixel tests")
    ap.add_argument("--pmc", default=str(REPO / "profiles" / "r01_pmc_config3.json"),
                    help="committed PMC summary to read `traffic` from")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank renders on cuda:0 and the "
                         "collectives run over gloo on host copies")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torchrun with {args.gpus} ranks")
    distributed = world > 1
    backend = "gloo" if args.rehearse else args.backend
    gpu = 0 if args.rehearse else local
    if distributed:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", gpu)
    # collectives run on the GPU tensors with RCCL, on host copies with gloo
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    pkg = __graft_entry__.load_package()
    w, rows = args.width, args.height
    full_h = rows * world
    k = args.k if args.k is not None else w / 640.0
    n_sph, n_cub = args.spheres * world, args.cubes * world
    scene = pkg.Scene.synthetic(w, full_h, n_sph, n_cub, seed=args.seed, k=k)
    rb, re = rank * rows, (rank + 1) * rows

    rt = pkg.RayTracer(gpu)
    rt.set_trace_mode(args.trace_mode)
    t = {name: torch.from_numpy(np.ascontiguousarray(getattr(scene, name))).to(dev)
         for name in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                      "cube_colours")}
    dscene = {name: v.data_ptr() for name, v in t.items()}
    dscene.update(num_spheres=scene.num_spheres, num_cubes=scene.num_cubes)
    if args.format == "i32x4":
        out = torch.empty((rows, w, 4), dtype=torch.int32, device=dev)
    else:
        out = torch.empty((rows, w), dtype=torch.int32, device=dev)
    # A real stream object: the legacy default stream's handle is 0, which the
    # C ABI reads as "the context's own stream".
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    # ctypes arguments built once; each step enqueues prep + coarse + trace
    step = rt.bind_render_device(dscene, w, full_h, (rb, re), out.data_ptr(), fmt=args.format,
                                 path=args.path, stream=stream.cuda_stream)

    def barrier():
        if distributed:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)

    def timed(profiled: bool):
        """K steps between barrier + sync on both sides; wall ms per step
        (max over ranks) and the stream-event ms per step."""
        rt.profile(profiled)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(args.steps):
            step()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        # this rank's K steps end here; the trailing barrier's own latency
        # (an RCCL all-reduce, tens of us) is not part of them.  The max over
        # ranks below is the job's time: every rank started at the barrier.
        wall = (time.perf_counter() - t0) * 1e3 / args.steps
        barrier()
        torch.cuda.synchronize(dev)
        rt.profile(False)
        if distributed:
            tt = torch.tensor([wall], device=coll_dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            wall = float(tt.item())
        return wall, ev0.elapsed_time(ev1) / args.steps

    # The timed region: K steps, nothing attached to the kernels.
    wall_ms, event_ms = timed(False)

    # Per-kernel durations: the same K steps again with start/stop HIP events
    # attached to each kernel's own dispatch packet on the launch stream
    # (hipExtLaunchKernelGGL; events from a pool grown in an untimed pass).
    # Not the timed region itself: with the events attached the wall time per
    # step grows by 25-40% (58-60 -> 73-85 us measured), while the kernels'
    # own durations agree with rocprofv3's.
    rt.profile(True)
    for _ in range(args.steps):  # untimed: grows the event pool to K renders
        step()
    torch.cuda.synchronize(dev)
    rt.profile_read()
    prof_wall_ms, _ = timed(True)
    prof = rt.profile_read()
    n = max(prof["renders"], 1)
    trace_ms = prof["trace_ms"] / n
    prep_ms, bin_ms = prof["prep_ms"] / n, prof["bin_ms"] / n

    rays_rank = w * rows
    value = world * rays_rank / (wall_ms * 1e-3) / 1e6
    algo_bytes = BYTES_PER_RAY[args.format] * rays_rank
    achieved = algo_bytes / (trace_ms * 1e-3) / 1e9

    traffic = None
    pmc_path = Path(args.pmc)
    # measured for the 1-GPU workload of the real binned trace kernel only
    if world == 1 and args.path != "generic" and args.trace_mode == 0 and pmc_path.exists():
        try:
            pmc = json.loads(pmc_path.read_text())
            if pmc.get("config") == [w, rows, args.spheres, args.cubes, args.seed, args.format]:
                traffic = pmc.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None

    gather = None
    if distributed and not args.no_gather:
        # Texture assembly on rank 0 (north_star): one RCCL gather of the bands.
        from opencl_ray_tracer_amd import rowbands

        band = out if coll_dev == dev else out.cpu()
        for _ in range(2):
            rowbands.gather_frame(band, full_h, world, rank)
        torch.cuda.synchronize(dev)
        barrier()
        g0 = time.perf_counter()
        reps = max(3, args.steps // 4)
        for _ in range(reps):
            rowbands.gather_frame(band, full_h, world, rank)
        torch.cuda.synchronize(dev)
        barrier()
        g_ms = (time.perf_counter() - g0) * 1e3 / reps
        gather = {"collective": f"{'rccl' if backend == 'nccl' else 'gloo (host)'} gather of "
                                f"row bands to rank 0", "ms": round(g_ms, 4),
                  "bytes_to_root": algo_bytes * (world - 1),
                  "render_plus_gather_mrays": round(
                      world * rays_rank / ((wall_ms + g_ms) * 1e-3) / 1e6, 1)}
        if args.format == "i32x4":
            # The Texture assembly: the same bands rendered in
            # the Texture's RGBA8 packing (MainState.cpp:1023-1037) gather 4x
            # fewer bytes.  Rendered once, untimed; the gather is timed alone.
            tex = torch.empty((rows, w), dtype=torch.int32, device=dev)
            rt.bind_render_device(dscene, w, full_h, (rb, re), tex.data_ptr(), fmt="rgba8",
                                  stream=stream.cuda_stream)()
            torch.cuda.synchronize(dev)
            tband = tex if coll_dev == dev else tex.cpu()
            for _ in range(2):
                rowbands.gather_frame(tband, full_h, world, rank)
            torch.cuda.synchronize(dev)
            barrier()
            g0 = time.perf_counter()
            for _ in range(reps):
                rowbands.gather_frame(tband, full_h, world, rank)
            torch.cuda.synchronize(dev)
            barrier()
            t_ms = (time.perf_counter() - g0) * 1e3 / reps
            gather["texture_rgba8"] = {"ms": round(t_ms, 4),
                                       "bytes_to_root": 4 * rays_rank * (world - 1)}

    host = None
    if world == 1 and not args.no_host_path:
        # the reference's timer scope (MainState.cpp:
        # 662-894: scene upload, render, blocking readback of the frame),
        # through the synchronous host-buffer entry point rt_render.  Never
        # `value`: it includes the PCIe copy of the whole frame.
        host_buf = np.empty(tuple(out.shape), np.int32 if args.format == "i32x4" else np.uint32)
        runs = [rt.render(scene, w, full_h, fmt=args.format, out=host_buf)[1]
                for _ in range(4)][1:]
        best = min(runs, key=lambda t: t.total_us)
        host = {"scope": "rt_render: scene upload + kernels + frame download (PCIe) into a "
                         "reused host buffer",
                "total_ms": round(best.total_us / 1e3, 3),
                "upload_ms": round(best.upload_us / 1e3, 3),
                "kernel_ms": round(best.kernel_us / 1e3, 3),
                "download_ms": round(best.download_us / 1e3, 3),
                "mrays_end_to_end": round(rays_rank / best.total_us, 1)}

    cpu = None
    if world == 1 and not args.no_cpu_baseline:  # rank 0 at N=1 only
        sys.path.insert(0, str(REPO / "tests"))
        from oracle_lib import Oracle  # CPU baseline only

        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        orc = Oracle()
        sample_rows = list(range(rb, re, args.cpu_rows))
        c0 = time.perf_counter()
        orc.trace_rows(scene, w, full_h, sample_rows, threads=threads)
        c_s = time.perf_counter() - c0
        # SURVEY.md §8d CPU baseline (a): the serial path on one core, on a
        # deterministic row subset (every 32nd row of the same frame)
        serial_rows = list(range(rb, re, 32))
        c1 = time.perf_counter()
        orc.trace_rows(scene, w, full_h, serial_rows, threads=1)
        s_s = time.perf_counter() - c1
        cpu = {"value": len(sample_rows) * w / c_s / 1e6, "unit": "Mrays/s", "cores": threads,
               "kind": "port",
               "sample": (f"the whole {w}x{len(sample_rows)} frame" if args.cpu_rows == 1 else
                          f"{len(sample_rows)} rows (every {args.cpu_rows}th of rank 0's band) x {w}"
                          f" px") + f" of the same scene, oracle/rt_oracle.c orc_trace_rows_mt on "
                         f"{threads} threads, {c_s:.1f} s wall",
               "serial_1core": {"value": round(len(serial_rows) * w / s_s / 1e6, 3),
                                "sample": f"every 32nd row ({len(serial_rows)} rows x {w} px), "
                                          f"1 thread, {s_s:.1f} s wall"}}

    # BASELINE.json config names, by the per-rank workload
    names = {(1920, 1080, 16, 4): "config2", (4096, 4096, 256, 64): "config3",
             (8192, 8192, 192, 64): "config4", (16384, 16384, 4096, 0): "config5"}
    workload = names.get((w, rows, args.spheres, args.cubes), "custom")
    # the dominant kernel: scenes of at most 512 primitives take trace_small_kernel
    kernel = "trace_small_kernel" if 0 < n_sph + 12 * n_cub <= 512 else "trace3_kernel"
    if args.path == "generic":
        kernel = "generic_kernel"
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall_ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{workload}: {w}x{rows} rows/rank, {args.spheres} spheres + "
                                   f"{args.cubes} cubes per rank, dense k={k:.2f}, seed {args.seed}",
                       "width": w, "rows_per_rank": rows, "image_height": full_h,
                       "spheres": n_sph, "cubes": n_cub, "format": args.format,
                       "parallelism": f"row-bands x{world}"
                                      + (" (rehearsal: shared cuda:0, gloo)" if args.rehearse
                                         else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel": kernel,
                         "kernel_ms": round(trace_ms, 4), "prep_ms": round(prep_ms, 4),
                         "bin_ms": round(bin_ms, 4), "algo_bytes_per_launch": algo_bytes},
            "event_ms_per_step": round(event_ms, 4),
            "profiled_pass_ms_per_step": round(prof_wall_ms, 4),
            "cpu_baseline": cpu,
            "gather": gather,
            "host_path": host,
        }
        print(json.dumps(line), flush=True)
    rt.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

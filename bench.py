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
import datetime
import json
import threading
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
CONFIG_NAMES = {(512, 512, 4, 1): "config1", (1920, 1080, 16, 4): "config2", (4096, 4096, 256, 64): "config3",
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
    ap.add_argument("--app-calls", type=int, default=20,
                    help="host_path.app: warm rt_render calls per scene and format")
    ap.add_argument("--no-extras", action="store_true",
                    help="time only the headline workload (N=1: no RGBA8 Texture line; "
                         "N>1: no Texture / config 4 / weak-scaling keys)")
    ap.add_argument("--path", choices=("auto", "binned", "generic"), default="auto",
                    help="kernel path: generic = the brute-force per-pixel kernel (every ray "
                         "against every primitive), for the compute-bound comparison")
    ap.add_argument("--trace-mode", type=int, default=0,
                    help="diagnostics ablation (needs the RT_DIAG=1 build): 1 = stores only, "
                         "2 = no per-pixel tests")
    ap.add_argument("--pmc", default=str(REPO / "profiles" / "r06_pmc_config3.json"),
                    help="committed PMC summary to read `traffic` from")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL over xGMI)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank renders on cuda:0 and the "
                         "collectives run over gloo on host copies")
    ap.add_argument("--inflight", type=int, default=2,
                    help="N=1: frames in flight -- step i renders frame i on slot i %% S of S "
                         "(context, stream, frame buffer) slots, so one frame's prep and "
                         "binning kernels overlap the previous frame's trace (1 = one stream)")
    ap.add_argument("--sustained", type=int, default=600,
                    help="N=1: also time the in-flight loop over this many frames (both "
                         "formats; independent of --steps) and report it as "
                         "frames_in_flight.sustained, the rate without a K-frame window's "
                         "fill and drain (0 = off: for rocprofv3 runs, whose kernel average "
                         "the long window's overlapping launches would weigh on)")
    ap.add_argument("--slot-streams", default="cumask", choices=("hip", "cumask", "torch"),
                    help="the frames-in-flight slots' streams: cumask (default) = streams "
                         "created with hipExtStreamCreateWithCUMask over every CU, each on a "
                         "hardware queue of its own; hip = hipStreamCreateWithFlags; torch = "
                         "torch's pool (round 5: RGBA8 3 slots 39.5-40.0 us per frame on hip "
                         "streams, 33.0 on cumask, 32.8-33.8 on torch's; int32x4 2 slots "
                         "51.1-52.0 on all three, profiles/r05/slot_streams.txt)")
    ap.add_argument("--inflight-rgba8", type=int, default=4,
                    help="the same for the texture_rgba8 leg (its trace leaves more room "
                         "beside it: 4 slots measured best on the round-6 library, "
                         "DESIGN.md §3.4)")
    ap.add_argument("--pg-timeout", type=float, default=60.0,
                    help="N>1: seconds before a data-path collective that another rank left "
                         "unmatched raises (gloo) or has its communicator aborted (RCCL, "
                         "TORCH_NCCL_ASYNC_ERROR_HANDLING=2), so the phase fails and the "
                         "later phases still run; well below --phase-deadline")
    ap.add_argument("--init-timeout", type=float, default=600.0,
                    help="N>1: seconds the process-group rendezvous waits for every rank")
    ap.add_argument("--phase-deadline", type=float, default=150.0,
                    help="N>1: a phase still running after this long (a hang the collective "
                         "timeout did not end) makes rank 0 print the line so far and every "
                         "rank exit with status 3")
    ap.add_argument("--golden", default=str(REPO / "tests" / "golden"),
                    help="committed fixtures (data: scene arrays and frame hashes) the timed "
                         "frame is checked against after the timed region (frame_check_ref)")
    ap.add_argument("--fail-assembly", default="",
                    help=argparse.SUPPRESS)  # tests: NAME[:RANK] raises in that assembly
    ap.add_argument("--selftest-cpu", action="store_true",
                    help=argparse.SUPPRESS)  # tests: the N>1 plumbing on gloo, no GPU
    return ap.parse_args(argv)


# The ONE JSON line goes to the process's original stdout; everything else
# written to fd 1 (C/C++ libraries' logging, e.g. gloo's "[Gloo] Rank ...
# connected" lines at N > 1) is sent to stderr by claim_stdout().
_LINE_OUT = None


def claim_stdout():
    global _LINE_OUT
    if _LINE_OUT is not None:
        return
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    _LINE_OUT = os.fdopen(fd, "w", buffering=1)


def emit_line(text: str):
    out = _LINE_OUT if _LINE_OUT is not None else sys.stdout
    out.write(text + "\n")
    out.flush()


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
    """The fastest assembly whose frame was bit-exact: (name, entry), or
    (None, None) when none was (the line then carries value null)."""
    ok = [(v["ms_per_step"], k) for k, v in assemblies.items()
          if isinstance(v, dict) and v.get("ms_per_step") is not None
          and v.get("frame_check") == "bit-exact"]
    if not ok:
        return None, None
    ms, name = min(ok)
    return name, assemblies[name]


FIXTURE_HASH_KEYS = {"i32x4": "fnv1a64", "rgba8": "fnv1a64_rgba8"}
SCENE_ARRAYS = ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                "cube_colours")


def reference_hash(scene, width: int, height: int, fmt: str, golden) -> tuple:
    """(FNV-1a-64, fixture name) of the committed fixture for exactly this
    workload -- same frame size and bit-identical scene arrays -- in format
    `fmt`, or (None, why).  Fixtures are data (tests/golden/make_golden.py:
    the oracle's frame hashed when the fixture was made), not the oracle."""
    key = FIXTURE_HASH_KEYS[fmt]
    for path in sorted(Path(golden).glob(f"*_{width}x{height}.npz")):
        with np.load(path, allow_pickle=False) as z:
            if key not in z.files or int(z["width"]) != width or int(z["height"]) != height:
                continue
            if all(np.array_equal(np.asarray(getattr(scene, n), np.float32).ravel(),
                                  np.asarray(z[n], np.float32).ravel()) for n in SCENE_ARRAYS):
                return int(z[key]), path.name
    return None, f"no committed fixture with this {width}x{height} scene in {fmt}"


def frame_check_ref(pkg, frame, scene, width: int, height: int, fmt: str, golden) -> dict:
    """The timed frame against the committed fixture's hash (after the timed
    region): {"frame_check_ref": "bit-exact" | "MISMATCH" | None, "source":
    ...}.  `frame`: a device or host tensor / array of the whole frame."""
    want, src = reference_hash(scene, width, height, fmt, golden)
    if want is None:
        return {"frame_check_ref": None, "source": src}
    host = frame.cpu() if hasattr(frame, "cpu") else frame
    got = pkg.fnv1a64(host)
    return {"frame_check_ref": "bit-exact" if got == want else "MISMATCH",
            "source": f"tests/golden/{src} {FIXTURE_HASH_KEYS[fmt]} {want:016x}",
            "fnv1a64": f"{got:016x}"}


def cpu_quota(root: str = "/sys/fs/cgroup"):
    """The job's CPU quota from its cgroup, in CPUs, and the file it came
    from: cgroup v2 `cpu.max` ("quota period" or "max ..."), else v1
    `cpu/cpu.cfs_quota_us` / `cpu.cfs_period_us` (-1 = none).  (None, path)
    when no quota is set, (None, None) when neither file exists."""
    v2 = Path(root) / "cpu.max"
    try:
        q, per = v2.read_text().split()[:2]
        return (None if q == "max" else int(q) / int(per)), str(v2)
    except (OSError, ValueError):
        pass
    v1 = Path(root) / "cpu" / "cpu.cfs_quota_us"
    try:
        q = int(v1.read_text())
        per = int((Path(root) / "cpu" / "cpu.cfs_period_us").read_text())
        return (None if q <= 0 or per <= 0 else q / per), str(v1)
    except (OSError, ValueError):
        return None, None


def cpu_threads(requested: int) -> tuple:
    """(threads to use, description).  0 = every CPU this job may run on:
    the affinity set, capped by the job's CPU share -- its cgroup CPU quota,
    and the launcher's OMP_NUM_THREADS where it states one (the GPU box
    grants 16 CPUs per GPU)."""
    affinity = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    quota, quota_src = cpu_quota()
    n = affinity
    if quota is not None:
        n = min(n, max(1, int(quota)))
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    if requested > 0:
        n = min(requested, affinity)
    return max(1, n), {"affinity_cpus": affinity, "os_cpu_count": os.cpu_count(),
                       "omp_num_threads": share,
                       "cgroup_cpu_quota": None if quota is None else round(quota, 2),
                       "cgroup_quota_file": quota_src}


class Ctx:
    """Process / device / collective plumbing of one bench run."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} with WORLD_SIZE={self.world}: the launcher "
                             f"must start {args.gpus} ranks (or leave WORLD_SIZE unset and let "
                             f"bench.py start them)")
        self.distributed = self.world > 1
        self.backend = "gloo" if args.rehearse else args.backend
        self.gpu = 0 if args.rehearse else local
        if self.distributed:
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            torch.cuda.set_device(self.gpu)
            # the rendezvous waits up to --init-timeout (on a fresh box the
            # ranks' first `import torch` can take minutes and need not end
            # together); the data-path group below, created right after,
            # carries --pg-timeout: a stuck collective there raises (gloo) or
            # has its communicator aborted (RCCL) after that long
            timeout = datetime.timedelta(seconds=max(args.init_timeout, args.pg_timeout))
            if self.backend == "nccl":
                # a collective left unmatched by a rank that failed out of a
                # phase: after --pg-timeout the communicator is aborted and
                # the blocked call fails (CleanUpOnly), instead of the
                # process being torn down with the line unprinted
                os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.gpu),
                                        timeout=timeout)
            else:
                dist.init_process_group("gloo", timeout=timeout)
        self.pg_timeout = args.pg_timeout
        # the data-path group (every measurement's collectives; replaced after
        # a phase fails, renew_group)
        self.pg = None
        if self.distributed:
            self.pg = dist.new_group(backend=self.backend,
                                     timeout=datetime.timedelta(seconds=args.pg_timeout))
        self.dev = torch.device("cuda", self.gpu)
        # collectives move GPU tensors with RCCL, host copies with gloo
        self.coll_dev = self.dev if self.backend == "nccl" else torch.device("cpu")
        # A real stream object: the legacy default stream's handle is 0, which
        # the C ABI reads as "the context's own stream".
        self.stream = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream)
        self.slot_streams = getattr(args, "slot_streams", "cumask")
        # N>1: a collective-free step (this rank's band into a private
        # buffer) for the clock ramp before each timed window (run_multi)
        self.ramp_step = None

    def renew_group(self):
        """A fresh data-path group for the phases after a failed one: a rank
        that raised out of a phase left the others' collectives of that phase
        unmatched, so the old group's sequence of operations no longer lines
        up across ranks (every rank calls this, after the agreement)."""
        if self.distributed:
            self.pg = self.dist.new_group(backend=self.backend,
                                          timeout=datetime.timedelta(seconds=self.pg_timeout))

    def barrier(self):
        if self.distributed:
            self.dist.barrier(group=self.pg)

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
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.pg)
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


# Exit status of an N>1 run (every rank): 0 = every phase completed and the
# line has a value; EXIT_HUNG = a phase hung past --phase-deadline (the
# watchdog ended the run, rank 0 printed the line first) or a rank left the
# run; EXIT_NO_VALUE = every phase completed but no assembly was bit-exact.
EXIT_HUNG = 3
EXIT_NO_VALUE = 4


class Phases:
    """The N>1 run as named phases, so one failing or hanging measurement
    never costs the JSON line (rank 0 prints it in every case), and the exit
    status tells a launcher what happened.

    run(key, fn): fn() on every rank; its value goes to target[key].  An
    exception on any rank becomes {"error": ...} under that key on every
    rank: the ranks agree over a separate gloo group (`ctrl`), so the
    agreement never pairs with a data-path collective another rank is still
    blocked in (that rank's collective fails after --pg-timeout and it joins
    the agreement); the later phases then run on a fresh data-path group.
    A caught exception is a completed phase: the run still exits 0.
    A phase still running after `deadline_s` is a hang: rank 0's watchdog
    prints the line built so far, that phase marked {"error": "timeout
    ..."}, and ends the process with EXIT_HUNG; the other ranks end with
    EXIT_HUNG too (their own watchdog a little later, or the agreement
    failing once rank 0 is gone)."""

    GRACE_S = 20.0  # non-root ranks outlive rank 0's deadline by this much

    def __init__(self, c, deadline_s: float, finish, pg_timeout_s: float = 180.0):
        self.c = c
        self.deadline = deadline_s
        self.finish = finish  # () -> the line dict to print (rank 0)
        self.current = None   # (key, target dict, start time)
        self.printed = False
        self.lock = threading.Lock()
        self.ctrl = None
        if c.distributed:
            # longer than the data-path timeout: a rank that failed early
            # waits here while the others' collective of that phase times out
            self.ctrl = c.dist.new_group(
                backend="gloo", timeout=datetime.timedelta(seconds=3 * pg_timeout_s + 60))
        if c.distributed or c.rank == 0:
            threading.Thread(target=self._watch, daemon=True).start()

    def _quit(self, why: str, status: int = EXIT_HUNG):
        """End this process with `status` once the line is out (rank 0
        prints it first, with the current phase marked as failed)."""
        with self.lock:
            if self.c.rank == 0 and not self.printed and self.current is not None:
                key, target, _ = self.current
                target[key] = {"error": why}
            self.emit()
        sys.stdout.flush()
        sys.stderr.write(f"bench.py rank {self.c.rank}: {why}; exiting with status {status}\n")
        sys.stderr.flush()
        os._exit(status)

    def _watch(self):
        limit = self.deadline + (0.0 if self.c.rank == 0 else self.GRACE_S)
        while True:
            time.sleep(0.5)
            with self.lock:
                cur = self.current
                if cur is None or self.printed or time.monotonic() - cur[2] < limit:
                    continue
            self._quit(f"timeout: phase still running after {self.deadline:.0f} s "
                       f"(rank {self.c.rank}'s watchdog)")

    def emit(self):
        """Print the line once (rank 0).  From the watchdog thread the main
        thread may still be filling the state, so a failed serialisation is
        retried before a minimal line goes out."""
        if self.c.rank != 0 or self.printed:
            return
        self.printed = True
        for attempt in range(5):
            try:
                text = json.dumps(self.finish())
                break
            except Exception as e:  # e.g. a dict resized during json.dumps
                time.sleep(0.05)
                text = json.dumps({"metric": METRIC, "value": None, "unit": "Mrays/s",
                                   "n_gpus": self.c.world, "error": f"line: {e!r}"})
        emit_line(text)

    def agree(self, ok: bool) -> bool:
        if self.ctrl is None:
            return ok
        t = self.c.torch.tensor([1 if ok else 0], dtype=self.c.torch.int32)
        try:
            self.c.dist.all_reduce(t, op=self.c.dist.ReduceOp.MIN, group=self.ctrl)
        except Exception as e:  # a rank is gone (rank 0 after printing, or a crash)
            self._quit(f"a rank left the run: {type(e).__name__}")
        return bool(int(t.item()))

    def run(self, key: str, fn, target: dict):
        with self.lock:
            self.current = (key, target, time.monotonic())
        err = None
        try:
            val = fn()
        except Exception as e:  # recorded; the other phases still run
            val, err = None, f"rank {self.c.rank}: {type(e).__name__}: {e}"
        ok = self.agree(err is None)
        with self.lock:
            self.current = None
            target[key] = val if ok else {"error": err or "failed on another rank"}
        if not ok and hasattr(self.c, "renew_group"):
            self.c.renew_group()
        return target[key]


def failing(args, c, name: str) -> bool:
    """--fail-assembly NAME[:RANK[:hang]] (tests): does assembly NAME raise
    on this rank?  With ":hang" the rank hangs in it instead (a collective
    that never completes, for the watchdog's end-to-end test)."""
    if not args.fail_assembly:
        return False
    what, rank, mode = (args.fail_assembly.split(":") + ["", ""])[:3]
    hit = what == name and (rank == "" or int(rank) == c.rank)
    if hit and mode == "hang":
        while True:
            time.sleep(1.0)
    return hit


class HipStreams:
    """`n` new non-blocking HIP streams (libamdhip64 through ctypes), each
    created now, so each takes the next hardware queue; close() destroys
    them (after a device synchronisation by the caller)."""

    def __init__(self, n: int, cu_mask_words: int = 0, masks=None):
        import ctypes
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                                      ctypes.c_uint]
        self.hip.hipExtStreamCreateWithCUMask.argtypes = [
            ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        self.hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
        self.handles = []
        for _ in range(n):
            st = ctypes.c_void_p()
            if cu_mask_words:  # every CU (or masks[i]), a stream of its own hardware queue
                words = masks[len(self.handles)] if masks else [0xFFFFFFFF] * cu_mask_words
                mask = (ctypes.c_uint32 * cu_mask_words)(*words)
                rc = self.hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), cu_mask_words, mask)
            else:
                rc = self.hip.hipStreamCreateWithFlags(ctypes.byref(st), 1)  # NonBlocking
            if rc != 0:
                self.close()
                raise RuntimeError(f"HIP stream creation failed ({rc})")
            self.handles.append(st.value)

    def close(self):
        for h in self.handles:
            self.hip.hipStreamDestroy(h)
        self.handles = []


def inflight_step(pkg, c: Ctx, ds, w, h, fmt, path, slots: int):
    """A step callable rendering frame i on slot i % slots: each slot has its
    own context (workspace), stream and frame buffer, so consecutive frames'
    kernels are independent and the GPU overlaps them (the small prep and
    binning kernels of one frame run beside the previous frame's trace).
    Returns (step, frames, keep-alive)."""
    rts = [pkg.RayTracer(c.gpu) for _ in range(slots)]
    # fresh streams of hardware queues of their own (--slot-streams cumask,
    # every CU in the mask: hipExtStreamCreateWithCUMask always makes a new
    # queue); plain hipStreamCreateWithFlags streams share the process's
    # few hardware queues round-robin with streams made earlier, which
    # serialised the RGBA8 leg's 3 slots (39.5 vs 33.0 us per frame, round 5)
    kind = getattr(c, "slot_streams", "cumask")
    n_words = (c.torch.cuda.get_device_properties(c.dev).multi_processor_count + 31) // 32
    streams = (HipStreams(slots, n_words if kind == "cumask" else 0)
               if kind in ("hip", "cumask")
               else [c.torch.cuda.Stream(c.dev) for _ in range(slots)])
    handles = streams.handles if isinstance(streams, HipStreams) else [st.cuda_stream
                                                                      for st in streams]
    frames = [frame_tensor(c, h, w, fmt) for _ in range(slots)]
    fns = [rt.bind_render_device(ds, w, h, (0, h), f.data_ptr(), fmt=fmt, path=path,
                                 stream=st)
           for rt, st, f in zip(rts, handles, frames)]
    n = [0]

    def step():
        fns[n[0] % slots]()
        n[0] += 1
    return step, frames, (rts, streams)


def measure_inflight(args, c: Ctx, pkg, ds, w, h, fmt, ref_frame, slots=None, ramp_step=None):
    """Throughput with `slots` (default args.inflight) frames in flight (the
    N=1 `value`): the timed region is K whole frames, every one a full prep +
    bin + trace pass; each slot's frame is compared with the one-stream
    frame."""
    slots = slots or args.inflight
    step, frames, keep = inflight_step(pkg, c, ds, w, h, fmt, args.path, slots)
    for _ in range(4 * slots + args.warmup):
        step()
    # untimed: a clock ramp right before the window.  Setting the slots up
    # (contexts, streams, frame buffers) leaves the GPU idle long enough for
    # its clock to fall back, and a K = 20 window that starts there runs its
    # first frames slow (config 3: 55-57 us per frame against 48-49 after a
    # ramp, scripts/inflight_state.py).  The ramp runs `ramp_step` (the
    # one-stream loop's step) when given, so that a rocprofv3 run of the
    # bench sees these launches one at a time, as in the pass that measures
    # the trace kernel's duration, not stretched by overlap.
    ramp = c.clock_ramp(ramp_step or step, args.warmup_ms)
    ms = c.timed(step, args.steps)
    out = {"frames_in_flight": slots, "ms_per_step": round(ms, 4),
           "value": round(mrays_per_s(w * h, ms), 1), "clock_ramp_steps": ramp}
    if getattr(args, "sustained", 0) > 0:
        # the same loop over --sustained frames (a fixed count, independent
        # of K): the rate without the pipeline's fill and drain and the first
        # dispatch after an idle GPU, which a K-frame window pays once
        # (reported beside `value`, never it)
        n_long = args.sustained
        ms_long = c.timed(step, n_long)
        out["sustained"] = {"steps": n_long, "ms_per_step": round(ms_long, 4),
                            "value": round(mrays_per_s(w * h, ms_long), 1),
                            "vs_window": round(ms / ms_long, 4)}
        if abs(ms / ms_long - 1.0) > 0.05:
            out["sustained"]["note"] = (
                f"the K = {args.steps} window with {slots} slots pays the pipeline's fill and "
                f"drain once (its first frames start on an idle GPU, its last drain alone); "
                f"over {n_long} frames that is amortised (DESIGN.md section 3.4)")
    same = all(bool(c.torch.equal(f, ref_frame)) for f in frames)
    c.sync()
    for rt in keep[0]:
        rt.close()
    if isinstance(keep[1], HipStreams):
        keep[1].close()
    out["frame_check"] = "bit-exact" if same else "MISMATCH"
    return out


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
APP_W, APP_H = 640, 480  # resources/defaultSettings.xml:1 (and Platform.cpp:264's minimum)


def _timing_ms(t) -> dict:
    return {"total_ms": round(t.total_us / 1e3, 4), "upload_ms": round(t.upload_us / 1e3, 4),
            "kernel_ms": round(t.kernel_us / 1e3, 4), "download_ms": round(t.download_us / 1e3, 4)}


def measure_app(args, c: Ctx, pkg) -> dict:
    """SURVEY.md §8f row f4 at the app's own workload: reference scenes 1-3
    (MainState.cpp:419-639, the golden fixtures' packed arrays) at 640x480
    (resources/defaultSettings.xml:1), through rt_render -- the replacement
    of executeRayTracerOpenCL, timed over the reference's timer scope
    (MainState.cpp:662-894: scene upload, render, blocking readback) into a
    reused, pageable host buffer like the app's `pixels` (:215).  Per scene
    and format, on a fresh context: rt_init (openCLInit's place,
    :1181-1326), the first call (cold) and the median of the warm calls --
    the number that replaces the app's "Time: X ms" label (:896-904).  Every
    frame is compared with the golden frame (RGBA8: its Texture packing,
    :1023-1037) in the same run."""
    import statistics

    golden = REPO / "tests" / "golden"
    res = {"scope": "rt_render: scene upload + kernels + frame download into a reused pageable "
                    "host buffer (MainState.cpp:662-894); first call of a fresh context "
                    "(after rt_init + rt_reserve, openCLInit's one-time setup: init_ms) and "
                    f"the median of {args.app_calls} warm calls",
           "resolution": f"{APP_W}x{APP_H}", "scenes": {}}
    for sid in (1, 2, 3):
        z = np.load(golden / f"scene{sid}_{APP_W}x{APP_H}.npz")
        scene = pkg.Scene(z["sphere_origins"], z["sphere_radius"], z["sphere_colours"],
                          z["cube_vertices"], z["cube_colours"])
        want32 = z["frame"]
        ent = {"spheres": scene.num_spheres, "cubes": scene.num_cubes}
        for fmt in ("i32x4", "rgba8"):
            want = want32 if fmt == "i32x4" else pkg.pack_rgba8(want32)
            out = np.empty(want.shape, want.dtype)
            out.fill(0)  # touched once, like a reserved `pixels` vector
            # openCLInit's place (MainState.cpp:1181-1326, once, before any
            # trace): rt_init + rt_reserve for the app's frame
            t0 = time.perf_counter()
            rt = pkg.RayTracer(c.gpu)
            rt.reserve(APP_W, APP_H, scene.num_spheres, scene.num_cubes, fmt)
            init_ms = (time.perf_counter() - t0) * 1e3
            try:
                ok = True
                _, first = rt.render(scene, APP_W, APP_H, fmt=fmt, out=out)
                ok &= bool(np.array_equal(out, want))
                warm = []
                for _ in range(args.app_calls):
                    out.fill(0)
                    _, t = rt.render(scene, APP_W, APP_H, fmt=fmt, out=out)
                    ok &= bool(np.array_equal(out, want))
                    warm.append(t)
                kernel = rt.last_kernel()
            finally:
                rt.close()
            med = {key: round(statistics.median(getattr(t, key) for t in warm) / 1e3, 4)
                   for key in ("total_us", "upload_us", "kernel_us", "download_us")}
            ent[fmt] = {"init_ms": round(init_ms, 3), "first": _timing_ms(first),
                        "warm_median": {k.replace("_us", "_ms"): v for k, v in med.items()},
                        "first_over_warm_kernel": round(first.kernel_us / max(
                            statistics.median(t.kernel_us for t in warm), 1e-9), 2),
                        "kernel": kernel,
                        "frame_check": "bit-exact" if ok else "MISMATCH"}
        res["scenes"][f"scene{sid}"] = ent
    return res


def run_single(args, c: Ctx, pkg):
    torch = c.torch
    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640.0
    # the app's own workload first, so its first rt_init is the process's
    app = None if args.no_host_path else measure_app(args, c, pkg)
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

    # One stream (the latency form): K steps, nothing attached to the kernels.
    wall_ms = c.timed(step, args.steps, events=(ev0, ev1))
    event_ms = ev0.elapsed_time(ev1) / args.steps
    # Per-kernel durations: the same K steps again with start/stop HIP events
    # attached to each kernel's own dispatch packet on the launch stream
    # (hipExtLaunchKernelGGL; events from a pool grown in an untimed pass),
    # right after the one-stream loop, in the same steady state as the
    # clock-ramp loop that makes up most of a rocprofv3 run's launches (two
    # frames in flight stretch each trace by ~8 %, so the pass runs first).
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
    # The timed region of `value`: K frames with args.inflight in flight
    # (a frame loop's throughput; 1 = the one-stream number above)
    inflight = None
    if args.inflight > 1 and args.trace_mode == 0:
        inflight = measure_inflight(args, c, pkg, ds, w, h, args.format, out, ramp_step=step)
    # `value`: the faster frame loop.  Frames in flight win at config 3; on
    # frames of 1 GiB and more two traces at once write the HBM less
    # efficiently than one after the other, and the one-stream loop wins
    # (DESIGN.md §3.4).  Both are reported.
    value_ms = (inflight["ms_per_step"]
                if inflight and inflight["frame_check"] == "bit-exact"
                and inflight["ms_per_step"] < wall_ms else wall_ms)

    kernel = rt.last_kernel()  # the kernel the library actually ran
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
                         "reused host buffer; total_ms is the wall time of the whole call, "
                         "upload_ms starts after the scene is packed into page-locked staging "
                         "(rt_timing, include/rt_hip.h)", **host_runs(), "app": app}
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
        t_inf = (measure_inflight(args, c, pkg, ds, w, h, "rgba8", tex, args.inflight_rgba8,
                                  ramp_step=tstep)
                 if args.inflight_rgba8 > 1 else None)
        rt.profile(True)
        for _ in range(args.steps):
            tstep()
        tp = rt.profile_read()
        rt.profile(False)
        t_kernel = rt.last_kernel()
        # the Texture frame against the fixture's RGBA8 hash (the in-flight
        # slots' frames were compared with this one-stream frame)
        t_ref = frame_check_ref(pkg, tex, scene, w, h, "rgba8", args.golden)
        t_trace = tp["trace_ms"] / max(tp["renders"], 1)
        t_bytes = BYTES_PER_RAY["rgba8"] * w * h
        t_ach = t_bytes / (t_trace * 1e-3) / 1e9
        t_ms = (t_inf["ms_per_step"] if t_inf and t_inf["frame_check"] == "bit-exact"
                and t_inf["ms_per_step"] < t_wall else t_wall)
        texture = {"format": "rgba8", "ms_per_step": round(t_ms, 4),
                   "value": round(mrays_per_s(w * h, t_ms), 1), "unit": "Mrays/s",
                   "frames_in_flight": t_inf,
                   "frame_check_ref": t_ref.pop("frame_check_ref"),
                   "frame_check_ref_source": t_ref,
                   "one_stream": {"ms_per_step": round(t_wall, 4),
                                  "value": round(mrays_per_s(w * h, t_wall), 1)},
                   "roofline": {"bound": "hbm", "achieved": round(t_ach, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(t_ach / HBM_PEAK_GBS, 4),
                                "kernel": t_kernel, "kernel_ms": round(t_trace, 4),
                                "algo_bytes_per_launch": t_bytes,
                                # the metric's own scope: the whole frame loop
                                "frame_frac": round(t_bytes / (t_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "note": "bound by per-wave test chains, not HBM (DESIGN.md §3.3, "
                                        "profiles/r04/pmc_mix_rgba8_final.txt)"}}
        del tex

    # the headline frame against the committed fixture's hash (outside every
    # timed region; the in-flight slots' frames were compared with this one)
    ref = frame_check_ref(pkg, out, scene, w, h, args.format, args.golden)
    cpu = None if args.no_cpu_baseline else cpu_baseline(args, scene, w, h)
    workload = CONFIG_NAMES.get((w, h, args.spheres, args.cubes), "custom")
    rt.close()
    return {
        "metric": METRIC, "value": round(mrays_per_s(rays, value_ms), 1), "unit": "Mrays/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(value_ms, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{workload}: {w}x{h} frame, {args.spheres} spheres + "
                               f"{args.cubes} cubes, dense k={k:.2f}, seed {args.seed}",
                   "width": w, "height": h, "spheres": args.spheres, "cubes": args.cubes,
                   "format": args.format,
                   "parallelism": "1 GPU (the whole frame)" + (
                       f", {args.inflight} frames in flight (one stream, context and frame "
                       f"buffer each)" if value_ms != wall_ms else ", one stream")},
        "frames_in_flight": inflight,
        "frame_check_ref": ref.pop("frame_check_ref"),
        "frame_check_ref_source": ref,
        "one_stream": {"ms_per_step": round(wall_ms, 4),
                       "value": round(mrays_per_s(rays, wall_ms), 1),
                       "event_ms_per_step": round(event_ms, 4)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel": kernel, "kernel_ms": round(trace_ms, 4),
                     "prep_ms": round(prep_ms, 4), "bin_ms": round(bin_ms, 4),
                     "algo_bytes_per_launch": algo_bytes,
                     # the frame level: the same bytes over ms_per_step (what
                     # `value` measures: prep + binning + trace, frames in flight)
                     "frame_frac": round(algo_bytes / (value_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "event_ms_per_step": round(event_ms, 4),
        "profiled_pass_ms_per_step": round(prof_wall_ms, 4),
        "clock_ramp": {"ms": args.warmup_ms, "untimed_steps": ramp_steps},
        "texture_rgba8": texture,
        "cpu_baseline": cpu,
        "host_path": host,
    }


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
    res = {"value": round(len(sample_rows) * w / c_s / 1e6, 3), "unit": "Mrays/s",
           "cores": threads, "kind": "port",
           "cores_scope": "the job's CPU share: the affinity set capped by the cgroup quota "
                          "and OMP_NUM_THREADS (host_cpus)",
           "host_cpus": cpus,
           "sample": (f"the whole {w}x{len(sample_rows)} frame" if args.cpu_rows == 1 else
                      f"{len(sample_rows)} rows (every {args.cpu_rows}th) x {w} px")
                     + f" of the same scene, oracle/rt_oracle.c orc_trace_rows_mt on "
                       f"{threads} threads (one row band per thread), {c_s:.1f} s wall",
           "serial_1core": {"value": round(len(serial_rows) * w / s_s / 1e6, 3),
                            "sample": f"every 32nd row ({len(serial_rows)} rows x {w} px), "
                                      f"1 thread, {s_s:.1f} s wall"}}
    # SURVEY.md §8d (b) asks for all host cores: when no cgroup quota caps the
    # job below its affinity set, a second leg on every CPU of the affinity
    # set (a sample of rows, so it stays short); `cores` stays the first leg
    aff = cpus["affinity_cpus"]
    quota = cpus["cgroup_cpu_quota"]
    share = cpus["omp_num_threads"]
    capped = (quota is not None and quota < aff) or (
        share is not None and share.isdigit() and 0 < int(share) < aff)
    if args.cpu_threads == 0 and aff > threads and not capped:
        step = max(1, args.cpu_rows, h * aff // (threads * 4096) if threads else 1)
        rows_all = list(range(0, h, step))
        c2 = time.perf_counter()
        orc.trace_rows(scene, w, h, rows_all, threads=aff)
        a_s = time.perf_counter() - c2
        res["all_affinity_cpus"] = {
            "value": round(len(rows_all) * w / a_s / 1e6, 3), "cores": aff,
            "sample": f"every {step}th row ({len(rows_all)} rows x {w} px), {aff} threads, "
                      f"{a_s:.1f} s wall"}
    else:
        res["all_affinity_cpus"] = None
        res["all_affinity_cpus_skipped"] = (
            "the first leg already uses every CPU of the affinity set" if aff <= threads else
            f"the cgroup quota ({quota} CPUs) or the launcher's share "
            f"(OMP_NUM_THREADS={cpus['omp_num_threads']}) caps this job at {threads} of the "
            f"{aff} CPUs in its affinity set")
    return res


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
                                               c.rank, handle_device=c.coll_dev, group=c.pg)
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
                                                      c.rank, async_op=True, bands=self.bands,
                                                      group=c.pg):
                    q.wait()  # the stream waits; the host does not
            else:
                c.sync()
                hf = self.host_frame
                self.rowbands.assemble_frame(hf, self.band.cpu(), self.height, c.world, c.rank,
                                             bands=self.bands, group=c.pg)
                if self.root:  # the other ranks' rows, host -> device
                    for r in range(1, c.world):
                        rb, re = self.bands[r]
                        self.frame[rb:re].copy_(hf[rb:re])
        else:
            # every band landed in rank 0's frame once every rank's render
            # finished: a one-element all-reduce behind the render on each
            # rank's stream (RCCL), or a host barrier after a sync (gloo)
            if c.backend == "nccl":
                c.dist.all_reduce(self.signal, async_op=True, group=c.pg).wait()
            else:
                c.sync()
                c.dist.barrier(group=c.pg)

    def step(self):
        self.render_only()
        self.assemble_only()

    def check(self, ds, pkg=None, scene=None, golden=None) -> tuple:
        """Rank 0: the assembled frame against a one-GPU render of the whole
        frame (bit-exact or not) and, when a committed fixture holds this
        workload (`scene` given), against the fixture's hash; broadcast so
        every rank agrees.  Returns (frame_check, frame_check_ref)."""
        c = self.c
        ok = c.torch.tensor([1, -1], dtype=c.torch.int32, device=c.coll_dev)
        if self.root:
            c.sync()
            ref = frame_tensor(c, self.height, self.width, self.fmt)
            self.rt.bind_render_device(ds, self.width, self.height, (0, self.height),
                                       ref.data_ptr(), fmt=self.fmt,
                                       stream=c.stream.cuda_stream)()
            c.sync()
            ok[0] = int(c.torch.equal(ref, self.frame))
            del ref
            if scene is not None:
                r = frame_check_ref(pkg, self.frame, scene, self.width, self.height, self.fmt,
                                    golden)["frame_check_ref"]
                ok[1] = -1 if r is None else int(r == "bit-exact")
        c.dist.broadcast(ok, 0, group=c.pg)
        ref_state = int(ok[1].item())
        return ("bit-exact" if int(ok[0].item()) else "MISMATCH",
                None if ref_state < 0 else "bit-exact" if ref_state else "MISMATCH")

    def close(self):
        if self.shared is not None:
            self.c.sync()
            self.shared.close(group=self.c.pg)


def _wrap_device(c: Ctx, ptr: int, rows, width, fmt):
    """A torch int32 tensor viewing `rows` x `width` pixels at device address
    `ptr` (memory owned by librt_hip.so, e.g. the shared frame)."""
    torch = c.torch
    shape = (rows, width, 4) if fmt == "i32x4" else (rows, width)

    class _Arr:
        __cuda_array_interface__ = {"shape": shape, "typestr": "<i4", "data": (ptr, False),
                                    "version": 2, "strides": None}
    return torch.as_tensor(_Arr(), device=c.dev)


def measure_assembly(args, c, pkg, rt, ds, width, height, fmt, how, split=False, bands=None,
                     name=None, scene=None):
    if failing(args, c, name or how):
        raise RuntimeError(f"--fail-assembly {args.fail_assembly}")
    a = Assembly(c, pkg, rt, ds, width, height, fmt, how, bands=bands)
    if a.error:
        a.close()  # frees what the root allocated; a barrier on every rank
        return {"ms_per_step": None, "error": a.error}
    for _ in range(args.warmup):
        a.step()
    # untimed: this rank's clock ramp (its own band into a private buffer, no
    # collective, so the ranks need not agree on a step count) right before
    # the window -- setting the assembly up leaves the GPU idle long enough
    # for its clock to fall back (measure_inflight)
    ramp_step = getattr(c, "ramp_step", None)
    if ramp_step is not None:
        c.clock_ramp(ramp_step, args.warmup_ms)
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
    res["frame_check"], res["frame_check_ref"] = a.check(ds, pkg, scene, args.golden)
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
    # two band sizes of at least 16 rows per rank must fit the frame (the
    # same decision on every rank, so no rank is left in a collective)
    if height < 2 * 16 * c.world:
        return None
    shared = rowbands.SharedFrame(rt, row_bytes * height, row_bytes, c.rank,
                                  handle_device=c.coll_dev, group=c.pg)
    try:
        if not shared.ok:
            return None
        times = []
        sizes = [height // c.world, max(16, height // (2 * c.world))]
        for n in sizes:
            rb = c.rank * n  # rb + n <= height: n <= height // world
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
        c.dist.all_gather(every, mine, group=c.pg)
        return [(float(e[0]), float(e[1])) for e in every]
    finally:
        c.sync()
        shared.close(group=c.pg)


def measure_host_frame(args, c: Ctx, pkg, rt, scene, w, h, fmt="i32x4"):
    """The reference's own consumer, a host frame (`pixels`, MainState.cpp:
    215/676, read back at :876-907, or the Texture's RGBA8 pixels,
    :984-994, :1023-1037), filled by N GPUs at once: every rank calls
    rt_render (the executeRayTracerOpenCL replacement: scene upload, render,
    download -- the app's timer scope, :662-894) for its band, straight into
    its rows of ONE page-locked host frame shared by the ranks
    (rowbands.HostFrame), each over its own GPU's PCIe link.  A step ends
    when every rank's rows are in (barrier).  The same scope with rank 0
    alone rendering the whole frame into the same buffer, in the same run,
    gives `scaling` = t(N=1) / t(N).  Checked bit-exactly on rank 0 against
    a one-GPU device render."""
    from opencl_ray_tracer_amd.rowbands import HostFrame, band_rows

    nbytes = BYTES_PER_RAY[fmt] * w * h
    rb, re = band_rows(h, c.world, c.rank)
    hf = HostFrame(h, w, fmt, c.rank, group=c.pg, register=pkg.host_register,
                   unregister=pkg.host_unregister)
    try:
        def step():
            if re > rb:
                rt.render(scene, w, h, rows=(rb, re), fmt=fmt, out=hf.band(rb, re))
            c.dist.barrier(group=c.pg)

        def step_one():  # rank 0 alone, the whole frame, same buffer and scope
            if c.rank == 0:
                rt.render(scene, w, h, fmt=fmt, out=hf.frame)
            c.dist.barrier(group=c.pg)
        for _ in range(max(1, args.warmup)):
            step_one()
            step()
        ms1 = c.timed(step_one, args.steps)
        ms = c.timed(step, args.steps)
        # the check: rank 0 poisons the frame, then one more N-rank step must
        # rewrite every row (the one-GPU steps left a complete frame behind)
        if c.rank == 0:
            hf.frame.fill(0x5A5A5A5A)
        c.dist.barrier(group=c.pg)
        step()
        ok = c.torch.ones(1, dtype=c.torch.int32, device=c.coll_dev)
        if c.rank == 0:
            keep, ds = device_scene_from(c, scene)
            ref = frame_tensor(c, h, w, fmt)
            rt.bind_render_device(ds, w, h, (0, h), ref.data_ptr(), fmt=fmt,
                                  stream=c.stream.cuda_stream)()
            c.sync()
            ok.fill_(int(np.array_equal(ref.cpu().numpy().view(hf.dtype), hf.frame)))
            del ref, keep
        c.dist.broadcast(ok, 0, group=c.pg)
        return {"scope": "rt_render per rank (scene upload + render + band download over its "
                         "own PCIe link) into one shared page-locked host frame, then a barrier",
                "format": fmt, "ms_per_step": round(ms, 4),
                "mrays_end_to_end": round(mrays_per_s(w * h, ms), 1),
                "host_gbs": round(nbytes / (ms * 1e-3) / 1e9, 1),
                "one_gpu": {"ms_per_step": round(ms1, 4),
                            "mrays_end_to_end": round(mrays_per_s(w * h, ms1), 1),
                            "scope": "rank 0 alone renders the whole frame into the same buffer "
                                     "(same run, same scope)"},
                "scaling": round(ms1 / ms, 3),
                "frame_check": "bit-exact" if int(ok.item()) else "MISMATCH"}
    finally:
        step = step_one = None
        hf.close()


def device_scene_from(c: Ctx, scene):
    t = {name: c.torch.from_numpy(np.ascontiguousarray(getattr(scene, name))).to(c.dev)
         for name in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                      "cube_colours")}
    ds = {name: v.data_ptr() for name, v in t.items()}
    ds.update(num_spheres=scene.num_spheres, num_cubes=scene.num_cubes)
    return t, ds


def measure_assemblies(args, c, pkg, rt, ds, w, h, fmt, phases, res, split=False, scene=None):
    """The frame assembled on rank 0 three ways: equal bands by RCCL
    point-to-point, equal bands by xGMI peer stores, and cost-balanced bands
    by xGMI peer stores.  The equal split makes every other rank wait on its
    link while rank 0's own rows need no transfer, so the balanced split
    sizes the bands by each rank's measured cost (render + stores into rank
    0's frame) for all ranks to finish together (rowbands.balanced_bands).
    Same frame, same end point, each checked bit-exactly.  Each assembly is
    its own phase: one that raises or hangs is recorded as {"error": ...}
    in `res` and the others still run."""
    from opencl_ray_tracer_amd import rowbands

    for how in ("rccl_p2p", "xgmi_peer_store"):
        phases.run(how, lambda how=how: measure_assembly(args, c, pkg, rt, ds, w, h, fmt, how,
                                                         split=split, scene=scene), res)

    def balanced():
        costs = calibrate_peer_store(args, c, pkg, rt, ds, w, h, fmt)
        if costs is None:
            return {"ms_per_step": None, "error": "no calibration (frame too short or no "
                                                  "shared mapping)"}
        bal = rowbands.balanced_bands(h, costs)
        r = measure_assembly(args, c, pkg, rt, ds, w, h, fmt, "xgmi_peer_store", split=split,
                             bands=bal, name="xgmi_peer_store_balanced", scene=scene)
        r["cost_model_us"] = [{"fixed": round(a * 1e6, 2), "per_row": round(s * 1e6, 4)}
                              for a, s in costs]
        return r
    phases.run("xgmi_peer_store_balanced", balanced, res)
    return res


def multi_line(args, c: Ctx, state: dict) -> dict:
    """The N>1 JSON line from the phases that have finished (`state`); a
    phase that failed or timed out appears as {"error": ...}."""
    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640.0
    asm = state.get("assembly", {})
    best, entry = pick_value(asm)
    ms = entry["ms_per_step"] if entry else None
    workload = CONFIG_NAMES.get((w, h, args.spheres, args.cubes), "custom")
    line = {
        "metric": METRIC, "value": round(mrays_per_s(w * h, ms), 1) if ms else None,
        "unit": "Mrays/s", "n_gpus": c.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4) if ms else None, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{workload}: {w}x{h} frame, {args.spheres} spheres + "
                               f"{args.cubes} cubes, dense k={k:.2f}, seed {args.seed}",
                   "width": w, "height": h, "spheres": args.spheres, "cubes": args.cubes,
                   "format": args.format,
                   "parallelism": f"row-bands x{c.world}, frame assembled on rank 0 by "
                                  f"{best or 'none (no bit-exact assembly)'}"
                                  + (" (rehearsal: shared cuda:0, gloo)" if args.rehearse
                                     else "")},
        "assembly": asm,
        "roofline": state.get("roofline"),
    }
    rl = line["roofline"]
    if ms and isinstance(rl, dict) and "error" not in rl:
        # the frame level over every GPU's HBM: the assembled frame's bytes
        # over ms_per_step against N x the one-GPU peak
        line["roofline"] = dict(rl, frame_frac=round(
            BYTES_PER_RAY[args.format] * w * h / (ms * 1e-3) / 1e9 / (HBM_PEAK_GBS * c.world), 4))
    for key in ("texture_rgba8", "config4", "weak_scaling", "host_frame", "one_gpu"):
        if key in state:
            line[key] = state[key]
    line["frame_check_ref"] = entry.get("frame_check_ref") if entry else None
    line.update(scaling_keys(c.world, ms, state.get("one_gpu"), state.get("weak_scaling")))
    line["scaling_host_frame"] = host_frame_scaling(state.get("host_frame"))
    line["clock_ramp"] = (state.get("setup") or {}).get("clock_ramp")
    line["cpu_baseline"] = state.get("cpu_baseline")
    errors = sorted(f"{key}.{sub}" if sub else key
                    for key, v in state.items() if isinstance(v, dict)
                    for sub in ([None] if "error" in v else
                                [s for s, e in v.items() if isinstance(e, dict) and "error" in e]))
    if errors:
        line["phase_errors"] = errors
    return line


SCALING_NOTE = (
    "north_star's >= 6x row-tile scaling at 8 GPUs is read from scaling_host_frame: the app's "
    "own consumer (pixels / the Texture's RGBA8 pixels) filled by N GPUs, each over its own "
    "PCIe link, against one GPU filling the same buffer in the same run and scope. "
    "scaling_assembled = t(N=1)/t(N) of `value` (the frame assembled in rank 0's HBM) cannot "
    "reach it: 7/8 of the frame must cross xGMI into one GPU (at most 7 links x ~153 GB/s) "
    "while one GPU writes the whole frame into its own HBM at ~6 TB/s (DESIGN.md section 7). "
    "scaling_weak = N x t(N=1)/t(N) with every GPU rendering a frame-sized band of an N-times "
    "taller frame.")


def scaling_keys(world: int, ms, one_gpu, weak) -> dict:
    """The N>1 line's scaling contract: scaling_assembled = t(N=1)/t(N) of
    `value`'s assembly, scaling_weak = N t(N=1)/t(N) of the weak-scaling
    frame (each rank one frame-sized band), both against rank 0 rendering
    the whole frame alone in the same run (`one_gpu`), and the note saying
    which number north_star's target is read from."""
    t1 = one_gpu.get("ms_per_step") if isinstance(one_gpu, dict) else None
    tw = weak.get("ms_per_step") if isinstance(weak, dict) else None
    return {"scaling_assembled": round(t1 / ms, 4) if t1 and ms else None,
            "scaling_weak": round(world * t1 / tw, 4) if t1 and tw else None,
            "scaling_note": SCALING_NOTE}


def host_frame_scaling(hf) -> dict:
    """`scaling_host_frame`: t(N=1) / t(N) of the app's host frame (the
    `host_frame` phases: every rank fills its rows of one page-locked host
    frame over its own PCIe link, against rank 0 alone filling it in the same
    run and scope), per format, only for bit-exact frames (else None).  This,
    not `value`, is the number north_star's row-tile scaling target is judged
    by: `value` at N > 1 is the frame assembled in rank 0's
    HBM, which no N > 1 can deliver faster than one GPU writing it locally."""
    out = {"definition": "t(N=1)/t(N), rt_render into one shared page-locked host frame, "
                         "same run and scope (host_frame.*.scaling)"}
    for fmt in ("i32x4", "rgba8"):
        e = (hf or {}).get(fmt)
        ok = isinstance(e, dict) and e.get("frame_check") == "bit-exact" and "scaling" in e
        out[fmt] = e["scaling"] if ok else None
    return out


def run_multi(args, c: Ctx, pkg):
    """N>1: every measurement is a phase (Phases), so the line is printed on
    rank 0 whatever one of them does."""
    from opencl_ray_tracer_amd import rowbands

    w, h = args.width, args.height
    k = args.k if args.k is not None else w / 640.0
    state = {"assembly": {}}
    env = {}
    phases = Phases(c, args.phase_deadline, lambda: multi_line(args, c, state), args.pg_timeout)
    rb, re = rowbands.band_rows(h, c.world, c.rank)

    def setup():
        env["scene"], env["ds"] = device_scene(pkg, c, w, h, args.spheres, args.cubes,
                                               args.seed, k)
        env["rt"] = rt = pkg.RayTracer(c.gpu)
        # untimed: bring every GPU to its steady clock (renders of this rank's band)
        ramp_out = frame_tensor(c, max(re - rb, 1), w, args.format)
        ramp = (rt.bind_render_device(env["ds"], w, h, (rb, re), ramp_out.data_ptr(),
                                      fmt=args.format, stream=c.stream.cuda_stream)
                if re > rb else (lambda: None))
        steps = c.clock_ramp(ramp, args.warmup_ms)
        c.sync()
        env["ramp_out"] = ramp_out
        c.ramp_step = ramp  # again right before each assembly's window
        return {"clock_ramp": {"ms": args.warmup_ms, "untimed_steps": steps}}
    phases.run("setup", setup, state)
    if "error" in state["setup"]:
        phases.emit()
        return EXIT_NO_VALUE
    rt, ds, scene = env["rt"], env["ds"], env["scene"]

    measure_assemblies(args, c, pkg, rt, ds, w, h, args.format, phases, state["assembly"],
                       split=True, scene=scene)

    def roofline():
        # the trace kernel on this rank's band, local stores (the roofline of
        # the dominant kernel; rank 0's band)
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
        kernel = rt.last_kernel() if re > rb else None
        trace_ms = prof["trace_ms"] / max(prof["renders"], 1)
        band_bytes = BYTES_PER_RAY[args.format] * w * (re - rb)
        achieved = band_bytes / (trace_ms * 1e-3) / 1e9 if trace_ms > 0 else 0.0
        return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": kernel, "kernel_ms": round(trace_ms, 4),
                "algo_bytes_per_launch": band_bytes, "scope": "rank 0's band, local stores"}
    phases.run("roofline", roofline, state)

    def one_gpu():
        # t(N=1) in the same run, the baseline of scaling_assembled and
        # scaling_weak: rank 0 alone renders the whole frame into a frame of
        # its own HBM (the N=1 line's one-stream step), the others idle
        if c.rank == 0:
            full = frame_tensor(c, h, w, args.format)
            step = rt.bind_render_device(ds, w, h, (0, h), full.data_ptr(), fmt=args.format,
                                         stream=c.stream.cuda_stream)
            for _ in range(args.warmup):
                step()
            c.clock_ramp(step, args.warmup_ms)
        else:
            step = (lambda: None)
        ms = c.timed(step, args.steps)
        return {"ms_per_step": round(ms, 4), "mrays": round(mrays_per_s(w * h, ms), 1),
                "scope": "rank 0 alone renders the whole frame into its own HBM (one stream), "
                         "same run"}
    phases.run("one_gpu", one_gpu, state)

    if not args.no_extras:
        # the Texture (RGBA8, MainState.cpp:1023-1037) assembled the same way
        state["texture_rgba8"] = {}
        measure_assemblies(args, c, pkg, rt, ds, w, h, "rgba8", phases, state["texture_rgba8"],
                           scene=scene)
        # BASELINE config 4: 8192^2, 192 + 64, row-tiled with the assembly
        c4 = CONFIG4
        k4 = c4["width"] / 640.0
        state["config4"] = {
            "workload": f"config4: {c4['width']}x{c4['height']} frame, {c4['spheres']} "
                        f"spheres + {c4['cubes']} cubes, dense k={k4:.1f}, seed {c4['seed']}, "
                        f"{c.world} row bands (BASELINE names 8 GPUs)"}

        def scene4():
            env["ds4"] = device_scene(pkg, c, c4["width"], c4["height"], c4["spheres"],
                                      c4["cubes"], c4["seed"], k4)[1]
            return "ok"
        if phases.run("scene", scene4, state["config4"]) == "ok":
            del state["config4"]["scene"]
            measure_assemblies(args, c, pkg, rt, env.pop("ds4"), c4["width"], c4["height"],
                               "i32x4", phases, state["config4"])

        def weak():
            # weak scaling (secondary): a 4096 x 4096N frame with N x (256 +
            # 64) primitives of the same density; rank r renders rows
            # [4096 r, 4096 (r + 1))
            hw = h * c.world
            _, dsw = device_scene(pkg, c, w, hw, args.spheres * c.world, args.cubes * c.world,
                                  args.seed, k)
            outw = frame_tensor(c, h, w, args.format)
            stepw = rt.bind_render_device(dsw, w, hw, (c.rank * h, (c.rank + 1) * h),
                                          outw.data_ptr(), fmt=args.format,
                                          stream=c.stream.cuda_stream)
            for _ in range(args.warmup):
                stepw()
            c.clock_ramp(stepw, args.warmup_ms)
            wms = c.timed(stepw, args.steps)
            return {"workload": f"{w}x{hw} frame, {args.spheres * c.world} spheres + "
                                f"{args.cubes * c.world} cubes; each rank renders {w}x{h} "
                                f"rows, no assembly",
                    "ms_per_step": round(wms, 4), "mrays": round(mrays_per_s(w * hw, wms), 1)}
        phases.run("weak_scaling", weak, state)
        # the app's host frame -- `pixels` (int32x4) and the Texture (RGBA8) --
        # filled by every GPU over its own PCIe link, beside one GPU filling it
        state["host_frame"] = {}
        for fmt in ("i32x4", "rgba8"):
            phases.run(fmt, lambda fmt=fmt: measure_host_frame(args, c, pkg, rt, scene, w, h, fmt),
                       state["host_frame"])

    # the CPU path beside the GPU numbers, timed on rank 0's
    # host CPUs while the other ranks wait
    if not args.no_cpu_baseline:
        phases.run("cpu_baseline",
                   lambda: cpu_baseline(args, scene, w, h) if c.rank == 0 else None, state)
    rt.close()
    phases.emit()
    return exit_status(state)


def exit_status(state: dict) -> int:
    """Every phase completed (a caught exception included): 0 when an
    assembly gave the line its value, else EXIT_NO_VALUE.  Every rank holds
    the same assembly results (frame checks are broadcast), so every rank
    returns the same status."""
    return 0 if pick_value(state.get("assembly", {}))[0] else EXIT_NO_VALUE


# ---------------------------------------------------------------------------
# `python bench.py --gpus N` without a launcher: one child process per rank
# ---------------------------------------------------------------------------
def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 with no WORLD_SIZE in the environment: start N fresh
    processes running this script with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set -- what torchrun would do -- and
    wait for them.  This process never touches the GPU (nothing here imports
    torch), and it starts children rather than exec'ing over itself.  Rank
    0's JSON line goes straight to the inherited stdout.  Exit status: 0
    when every rank exits 0; EXIT_HUNG when a rank reports a hang (3) or has
    to be killed because it outlived a failed rank by more than the phase
    deadline (plus the watchdogs' grace); else the first non-zero status in
    rank order (a signal -> 128 + its number).  SIGTERM / SIGINT are passed
    on to the ranks.  (The reference picks one device and never starts
    more, MainState.cpp:1241-1266.)"""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    base = dict(os.environ)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for r in range(args.gpus):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv],
                                      env=env))

    def forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    grace = args.phase_deadline + Phases.GRACE_S + 30.0
    failed_at, killed = None, False
    try:
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
                failed_at = time.monotonic()
            if failed_at is not None and time.monotonic() - failed_at > grace:
                for p in procs:  # our own children, by PID
                    if p.poll() is None:
                        p.kill()
                        killed = True
            time.sleep(0.2)
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
    codes = [p.wait() for p in procs]
    if all(rc == 0 for rc in codes):
        return 0
    if killed or EXIT_HUNG in codes:
        return EXIT_HUNG
    rc = next(rc for rc in codes if rc != 0)
    return rc if rc > 0 else 128 - rc


class CpuCtx(Ctx):
    """Ctx on the CPU (--selftest-cpu): the gloo process group and the
    barrier / timing / max-over-ranks plumbing, no device."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.distributed = self.world > 1
        self.backend = "gloo"
        self.gpu = None
        timeout = datetime.timedelta(seconds=max(args.init_timeout, args.pg_timeout))
        if self.distributed:
            dist.init_process_group("gloo", timeout=timeout)
        self.pg_timeout = args.pg_timeout
        self.pg = (dist.new_group(backend="gloo",
                                  timeout=datetime.timedelta(seconds=args.pg_timeout))
                   if self.distributed else None)
        self.dev = self.coll_dev = torch.device("cpu")
        self.ramp_step = None

    def sync(self):
        pass


def run_selftest_cpu(args) -> int:
    """The N>1 plumbing without a GPU (tests): launcher, rendezvous, phases,
    the frame assembled on rank 0 over gloo (rowbands.assemble_frame, the
    rccl_p2p path's collective), the one-rank baseline, weak scaling and
    the line with its scaling keys.  Bands are filled with a known pattern
    (pixel (y, x, c) = 1000 y + 10 x + c), not traced: no rays, no oracle."""
    c = CpuCtx(args)
    pkg = __graft_entry__.load_package()
    from opencl_ray_tracer_amd import rowbands

    w, h = args.width, args.height
    torch = c.torch
    state = {"assembly": {}}
    phases = Phases(c, args.phase_deadline, lambda: dict(
        multi_line(args, c, state), data="selftest: CPU pattern frame over gloo, no rays traced"),
        args.pg_timeout)

    def rows(a, b, width=w):
        y = torch.arange(a, b, dtype=torch.int32).view(-1, 1, 1)
        x = torch.arange(width, dtype=torch.int32).view(1, -1, 1)
        return (1000 * y + 10 * x + torch.arange(4, dtype=torch.int32).view(1, 1, -1)).contiguous()

    def assembly():
        if failing(args, c, "rccl_p2p"):
            raise RuntimeError(f"--fail-assembly {args.fail_assembly}")
        rb, re = rowbands.band_rows(h, c.world, c.rank)
        frame = torch.full((h, w, 4), -7, dtype=torch.int32) if c.rank == 0 else None
        band = frame[rb:re] if c.rank == 0 else torch.empty((re - rb, w, 4), dtype=torch.int32)

        def step():
            band.copy_(rows(rb, re))
            rowbands.assemble_frame(frame, band, h, c.world, c.rank, group=c.pg)
        ms = c.timed(step, args.steps)
        ok = torch.tensor([int(c.rank != 0 or bool(torch.equal(frame, rows(0, h))))],
                          dtype=torch.int32)
        c.dist.broadcast(ok, 0, group=c.pg)
        return {"ms_per_step": round(ms, 4), "mrays": round(mrays_per_s(w * h, ms), 1),
                "frame_check": "bit-exact" if int(ok.item()) else "MISMATCH",
                "frame_check_ref": None,
                "rows_per_rank": [e - b for b, e in (rowbands.band_rows(h, c.world, r)
                                                     for r in range(c.world))]}
    phases.run("rccl_p2p", assembly, state["assembly"])

    def one_gpu():
        full = torch.empty((h, w, 4), dtype=torch.int32)
        step = (lambda: full.copy_(rows(0, h))) if c.rank == 0 else (lambda: None)
        ms = c.timed(step, args.steps)
        return {"ms_per_step": round(ms, 4), "mrays": round(mrays_per_s(w * h, ms), 1)}
    phases.run("one_gpu", one_gpu, state)

    def weak():
        own = torch.empty((h, w, 4), dtype=torch.int32)
        ms = c.timed(lambda: own.copy_(rows(c.rank * h, (c.rank + 1) * h)), args.steps)
        return {"ms_per_step": round(ms, 4), "mrays": round(mrays_per_s(w * h * c.world, ms), 1)}
    phases.run("weak_scaling", weak, state)
    phases.emit()
    if c.distributed:
        c.dist.destroy_process_group()
    return exit_status(state)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start one process per rank (before any GPU call here)
        sys.exit(launch_ranks(args, sys.argv[1:]))
    claim_stdout()
    if args.selftest_cpu:
        sys.exit(run_selftest_cpu(args))
    c = Ctx(args)
    pkg = __graft_entry__.load_package()
    if c.distributed:
        status = run_multi(args, c, pkg)  # rank 0 prints the line
        c.dist.destroy_process_group()
        sys.exit(status)
    line = run_single(args, c, pkg)
    emit_line(json.dumps(line))


if __name__ == "__main__":
    main()

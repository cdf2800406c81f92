"""Row-band sharding of one frame over ranks (one process per GPU).

No reference counterpart: the reference is single-device (MainState.cpp:
1241-1266 picks one OpenCL device).  Pixels are independent, so rank r
renders a contiguous band of rows -- a contiguous slice of the row-major
frame -- and the frame is assembled on the root rank by one gather
(RCCL over xGMI with backend "nccl", gloo on CPU for tests).  The scene is
tiny and read-only and is broadcast from the root once.

The collectives here are device-agnostic: they move whatever torch tensors
they are given, so the same code drives the GPU path (librt_hip.so's
rt_render_device into a cuda tensor) and the CPU tests (gloo).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

SCENE_FIELDS = ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                "cube_colours")


def band_rows(height: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [row_begin, row_end) of `rank` (sizes differ by
    at most one row)."""
    if not (0 <= rank < world) or height <= 0:
        raise ValueError("bad band request")
    return rank * height // world, (rank + 1) * height // world


def balanced_bands(height: int, costs) -> List[Tuple[int, int]]:
    """Contiguous row bands, in rank order, sized so that every rank
    finishes together under its own cost model t_r(n) = a_r + s_r * n
    (fixed cost a_r, cost per row s_r): the water-filling solution of
    min max_r t_r(n_r) subject to sum_r n_r = height, n_r >= 0.  Ranks whose
    fixed cost alone exceeds the common finish time get no rows.  Rounding
    leftovers go, one row at a time, to the active rank that would finish
    its extra row soonest (never to a dropped rank); rows the float
    solution over-assigns come back from the rank finishing last."""
    n = len(costs)
    if n == 0 or height <= 0:
        raise ValueError("bad band request")
    a = [max(0.0, float(c[0])) for c in costs]
    s = [float(c[1]) for c in costs]
    if any(not (x > 0.0) for x in s):
        raise ValueError("every rank needs a positive cost per row")
    active = set(range(n))
    while True:
        t = (height + sum(a[r] / s[r] for r in active)) / sum(1.0 / s[r] for r in active)
        drop = {r for r in active if t - a[r] < 0.0}
        if not drop:
            break
        active -= drop
    rows = [max(0, int((t - a[r]) / s[r] + 1e-6)) if r in active else 0 for r in range(n)]
    while sum(rows) < height:
        r = min(active, key=lambda q: (a[q] + s[q] * (rows[q] + 1), q))
        rows[r] += 1
    while sum(rows) > height:
        r = max((q for q in active if rows[q] > 0), key=lambda q: (a[q] + s[q] * rows[q], -q))
        rows[r] -= 1
    assert all(k >= 0 for k in rows) and sum(rows) == height, rows
    bands, at = [], 0
    for k in rows:
        bands.append((at, at + k))
        at += k
    return bands


def broadcast_scene(arrays: Optional[Dict[str, "np.ndarray"]], root: int, device,
                    group=None) -> Dict[str, "torch.Tensor"]:
    """Broadcast the packed scene arrays from `root` (None elsewhere) and
    return them as tensors on `device` on every rank."""
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    counts = torch.zeros(2, dtype=torch.int64, device=device)
    if rank == root:
        counts[0] = len(arrays["sphere_radius"])
        counts[1] = len(arrays["cube_colours"])
    dist.broadcast(counts, root, group=group)
    n, m = int(counts[0]), int(counts[1])
    shapes = {"sphere_origins": (n, 4), "sphere_radius": (n,), "sphere_colours": (n, 4),
              "cube_vertices": (m, 36, 4), "cube_colours": (m, 4)}
    out = {}
    for name in SCENE_FIELDS:
        if rank == root:
            t = torch.from_numpy(np.ascontiguousarray(arrays[name], np.float32)).to(device)
        else:
            t = torch.empty(shapes[name], dtype=torch.float32, device=device)
        if t.numel():
            dist.broadcast(t, root, group=group)
        out[name] = t
    return out


def gather_frame(band: "torch.Tensor", height: int, world: int, rank: int, root: int = 0,
                 group=None) -> Optional["torch.Tensor"]:
    """Assemble the full frame on `root` from every rank's band (rows
    band_rows(height, world, r)).  Bands are padded to the largest band so
    one equal-size gather moves them; root trims and concatenates."""
    import torch
    import torch.distributed as dist

    max_rows = max(band_rows(height, world, r)[1] - band_rows(height, world, r)[0]
                   for r in range(world))
    rows = band.shape[0]
    if rows < max_rows:
        pad = torch.zeros((max_rows - rows,) + tuple(band.shape[1:]), dtype=band.dtype,
                          device=band.device)
        send = torch.cat([band, pad])
    else:
        send = band.contiguous()
    gl: Optional[List[torch.Tensor]] = (
        [torch.empty_like(send) for _ in range(world)] if rank == root else None)
    dist.gather(send, gl, dst=root, group=group)
    if rank != root:
        return None
    parts = []
    for r in range(world):
        rb, re = band_rows(height, world, r)
        parts.append(gl[r][: re - rb])
    return torch.cat(parts)


def assemble_frame(frame: Optional["torch.Tensor"], band: "torch.Tensor", height: int,
                   world: int, rank: int, root: int = 0, group=None, async_op: bool = False,
                   bands: Optional[List[Tuple[int, int]]] = None):
    """Assemble the frame on `root` by point-to-point transfers straight
    into the root's frame rows (RCCL P2P over xGMI with backend "nccl").

    `frame` is the root's whole frame (None elsewhere); the root renders its
    own band directly into frame[band_rows(root)], so nothing of it moves.
    Every other rank sends its band, which lands in frame[rb:re] with no
    padding, staging list or concatenation on the root (unlike
    gather_frame).  Empty bands (height < world) send nothing.  With
    async_op the requests are returned (wait() orders the caller's stream
    after them, without a host sync).  `bands`: each rank's (row_begin,
    row_end) when not band_rows' equal split (e.g. balanced_bands)."""
    import torch.distributed as dist

    ops = []
    if rank == root:
        for r in range(world):
            rb, re = bands[r] if bands is not None else band_rows(height, world, r)
            if r != root and re > rb:
                ops.append(dist.P2POp(dist.irecv, frame[rb:re], r, group))
    elif band.shape[0]:
        ops.append(dist.P2POp(dist.isend, band, root, group))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    if async_op:
        return reqs
    for q in reqs:
        q.wait()
    return None


class SharedFrame:
    """The root's frame mapped into every rank's device (xGMI peer stores).

    The root allocates the whole frame with rt_shared_alloc and broadcasts
    its 64-byte IPC handle; every other rank maps it with rt_shared_open.
    rank r then renders its band with `ptr_of_row(rb)` as the device output,
    so the trace kernel's stores land in the root's HBM and no gather copy
    runs.  `handle_device` is where the handle tensor lives for the
    broadcast (the GPU for RCCL, the CPU for gloo)."""

    def __init__(self, tracer, nbytes: int, row_bytes: int, rank: int, root: int = 0,
                 group=None, handle_device="cpu"):
        import torch
        import torch.distributed as dist

        self.tracer, self.rank, self.root = tracer, rank, root
        self.row_bytes = row_bytes
        self.owner = rank == root
        ok = torch.ones(1, dtype=torch.int32, device=handle_device)
        h = torch.zeros(64, dtype=torch.uint8, device=handle_device)
        self.ptr = 0
        self.error: Optional[str] = None
        if self.owner:
            try:
                self.ptr, hb = tracer.shared_alloc(nbytes)
                h.copy_(torch.frombuffer(bytearray(hb), dtype=torch.uint8))
            except Exception as e:  # reported, and every rank skips the path
                self.error = f"rank {rank}: {e}"
                ok.zero_()
        dist.broadcast(h, root, group=group)
        if not self.owner:
            try:
                self.ptr = tracer.shared_open(bytes(h.cpu().numpy().tobytes()))
            except Exception as e:
                self.error = f"rank {rank}: {e}"
                ok.zero_()
        # every rank learns whether all of them hold a mapping
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        self.ok = bool(int(ok.item()))
        if not self.ok and self.error is None:
            self.error = "another rank could not allocate or map the frame"

    def ptr_of_row(self, row: int) -> int:
        return self.ptr + row * self.row_bytes

    def close(self, group=None) -> None:
        """Unmap on every rank, then (after a barrier) free on the root."""
        import torch.distributed as dist

        if self.ptr and not self.owner:
            self.tracer.shared_close(self.ptr)
        dist.barrier(group=group)
        if self.ptr and self.owner:
            self.tracer.shared_free(self.ptr)
        self.ptr = 0


class HostFrame:
    """One host frame shared by the ranks of a node: the app's own consumer
    buffer -- `pixels` (int32x4, MainState.cpp:215, read back at :876-907)
    or the Texture's RGBA8 surface pixels (uint32, :984-994, :1023-1037) --
    in POSIX shared memory, so every rank's band lands in it straight over
    its own GPU's PCIe link and no rank-to-rank copy exists.

    The root creates the segment and broadcasts its name (`group`'s
    broadcast_object_list); every rank maps it and takes `band(rb, re)`, a
    view of its rows.  `register` / `unregister` (e.g. rt_host_register)
    page-lock the mapping on each rank for direct DMA.  close(): every rank
    unmaps, then (after a barrier) the root unlinks."""

    def __init__(self, height: int, width: int, fmt: str, rank: int, root: int = 0,
                 group=None, register=None, unregister=None):
        import numpy as np
        import torch.distributed as dist
        from multiprocessing import resource_tracker, shared_memory

        self.rank, self.root, self.group = rank, root, group
        self.shape = (height, width, 4) if fmt == "i32x4" else (height, width)
        self.dtype = np.int32 if fmt == "i32x4" else np.uint32
        nbytes = int(np.prod(self.shape)) * 4
        self.unregister = unregister
        self.shm = None
        self.frame = None
        name = [None]
        if rank == root:
            self.shm = shared_memory.SharedMemory(create=True, size=nbytes)
            name = [self.shm.name]
        dist.broadcast_object_list(name, root, group=group)
        if rank != root:
            self.shm = shared_memory.SharedMemory(name=name[0])
            resource_tracker.unregister(self.shm._name, "shared_memory")  # the root unlinks it
        self.frame = np.ndarray(self.shape, self.dtype, buffer=self.shm.buf)
        self.registered = False
        if register is not None:
            register(self.frame)
            self.registered = True

    def band(self, row_begin: int, row_end: int):
        return self.frame[row_begin:row_end]

    def close(self) -> None:
        """Unregister and unmap; the root unlinks the segment.  No collective:
        POSIX keeps every other rank's mapping valid until that rank unmaps
        it, so the root unlinks at once and a rank that failed mid-phase can
        neither pair this with another phase's collective nor leak the
        frame-sized /dev/shm segment (the unlink runs even if unmapping
        raises)."""
        try:
            if self.registered and self.unregister is not None:
                self.registered = False
                self.unregister(self.frame)
        finally:
            self.frame = None
            shm, self.shm = self.shm, None
            if shm is not None:
                try:
                    shm.close()
                finally:
                    if self.rank == self.root:
                        shm.unlink()


def interleaved_blocks(height: int, world: int, rank: int, block: int = 64) -> List[Tuple[int, int]]:
    """Row blocks of `block` rows dealt round-robin over the ranks (SURVEY.md
    §8e: for scenes whose load is not uniform down the frame).  64 rows is
    one coarse bin row, so no bin is split between ranks."""
    if not (0 <= rank < world) or height <= 0 or block <= 0:
        raise ValueError("bad block request")
    starts = range(rank * block, height, world * block)
    return [(s, min(s + block, height)) for s in starts]


def gather_frame_interleaved(blocks: "torch.Tensor", height: int, world: int, rank: int,
                             block: int = 64, root: int = 0,
                             group=None) -> Optional["torch.Tensor"]:
    """Assemble the frame on `root` from every rank's interleaved row blocks
    (this rank's blocks concatenated in order): one padded gather, then the
    root puts every rank's blocks back in frame order."""
    import torch
    import torch.distributed as dist

    counts = [sum(e - s for s, e in interleaved_blocks(height, world, r, block))
              for r in range(world)]
    max_rows = max(counts)
    rows = blocks.shape[0]
    if rows < max_rows:
        pad = torch.zeros((max_rows - rows,) + tuple(blocks.shape[1:]), dtype=blocks.dtype,
                          device=blocks.device)
        send = torch.cat([blocks, pad])
    else:
        send = blocks.contiguous()
    gl: Optional[List[torch.Tensor]] = (
        [torch.empty_like(send) for _ in range(world)] if rank == root else None)
    dist.gather(send, gl, dst=root, group=group)
    if rank != root:
        return None
    frame = torch.empty((height,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
    for r in range(world):
        at = 0
        for s, e in interleaved_blocks(height, world, r, block):
            frame[s:e] = gl[r][at:at + (e - s)]
            at += e - s
    return frame


def render_distributed(render_band: Callable[[int, int], "torch.Tensor"], height: int,
                       world: int, rank: int, root: int = 0, group=None,
                       interleave: int = 0) -> Optional["torch.Tensor"]:
    """render_band(row_begin, row_end) -> that band's tensor; the frame is
    returned on root, None elsewhere.  interleave > 0 deals row blocks of
    that many rows round-robin instead of one contiguous band per rank."""
    if interleave > 0:
        import torch

        parts = [render_band(s, e) for s, e in interleaved_blocks(height, world, rank, interleave)]
        # a rank with no block still sends a (padded) empty part
        blocks = torch.cat(parts) if parts else render_band(0, 1)[:0]
        return gather_frame_interleaved(blocks, height, world, rank, interleave, root=root,
                                        group=group)
    rb, re = band_rows(height, world, rank)
    if re > rb:
        band = render_band(rb, re)
    else:
        # height < world: this rank has no rows.  It renders nothing (an
        # empty row range is not a legal render) and still joins the gather
        # with a padded empty band, so no rank blocks in the collective.
        band = render_band(0, 1)[:0]
    return gather_frame(band, height, world, rank, root=root, group=group)

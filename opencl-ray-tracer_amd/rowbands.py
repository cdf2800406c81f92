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
    band = render_band(rb, re)
    return gather_frame(band, height, world, rank, root=root, group=group)

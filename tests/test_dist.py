"""Multi-rank row-band path on the CPU: world_size 2 over gloo.  Each rank
renders its band (the oracle stands in for the per-GPU band renderer -- test
infrastructure only), the scene is broadcast from rank 0 and the frame is
gathered on rank 0 with the same rowbands.py code the GPU path uses."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, width, height, scene_id, result_path, interleave=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "tests"))
    import torch
    import torch.distributed as dist

    import __graft_entry__
    from oracle_lib import Oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = __graft_entry__.load_package()
        from opencl_ray_tracer_amd import rowbands

        oracle = Oracle()
        arrays = None
        if rank == 0:
            sc = oracle.scene_reference(scene_id, 1)
            arrays = {k: getattr(sc, k) for k in rowbands.SCENE_FIELDS}
        scene = rowbands.broadcast_scene(arrays, 0, torch.device("cpu"))
        ns = pkg.Scene(*(scene[k].numpy() for k in rowbands.SCENE_FIELDS))

        def render_band(rb, re):
            return torch.from_numpy(oracle.trace(ns, width, height, rows=(rb, re)))

        frame = rowbands.render_distributed(render_band, height, world, rank,
                                            interleave=interleave)
        if rank == 0:
            np.save(result_path, frame.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("height,scene_id,interleave", [(480, 1, 0), (97, 3, 0), (480, 1, 64),
                                                       (200, 3, 64), (97, 2, 16),
                                                       (1, 1, 0), (1, 1, 64)])
def test_two_rank_row_bands_gloo(tmp_path, oracle, height, scene_id, interleave):
    import torch.multiprocessing as mp

    width, world = 640, 2
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, _free_port(), width, height, scene_id, str(out), interleave),
             nprocs=world, join=True)
    frame = np.load(out)
    want = oracle.trace(oracle.scene_reference(scene_id, 1), width, height)
    assert np.array_equal(frame, want)


@pytest.mark.parametrize("world,height,scene_id,interleave", [(4, 97, 3, 0), (8, 480, 1, 64),
                                                             (8, 480, 2, 0)])
def test_more_rank_row_bands_gloo(tmp_path, oracle, world, height, scene_id, interleave):
    """The N = 4 / 8 layouts the driver's scaling run uses, rehearsed on the
    CPU over gloo; the assembled 640x480 frames of scenes 1 and 2 are the
    reference's own CPU frames (the survey probe's known answers)."""
    import torch.multiprocessing as mp

    from conftest import SURVEY_FNV, probe_fnv

    width = 640
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, _free_port(), width, height, scene_id, str(out), interleave),
             nprocs=world, join=True)
    frame = np.load(out)
    want = oracle.trace(oracle.scene_reference(scene_id, 1), width, height)
    assert np.array_equal(frame, want)
    if height == 480:
        assert probe_fnv(frame) == SURVEY_FNV[scene_id]


def test_band_rows_partition():
    sys.path.insert(0, str(REPO))
    import __graft_entry__
    __graft_entry__.load_package()
    from opencl_ray_tracer_amd.rowbands import band_rows

    for h in (1, 7, 480, 4096, 4097):
        for world in (1, 2, 3, 4, 8):
            if world > h:
                continue
            bands = [band_rows(h, world, r) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == h
            assert all(a[1] == b[0] for a, b in zip(bands, bands[1:]))
            sizes = [e - b for b, e in bands]
            assert max(sizes) - min(sizes) <= 1


def test_interleaved_blocks_partition():
    sys.path.insert(0, str(REPO))
    import __graft_entry__
    __graft_entry__.load_package()
    from opencl_ray_tracer_amd.rowbands import interleaved_blocks

    for h in (1, 63, 64, 65, 480, 4097):
        for world in (1, 2, 3, 8):
            rows = sorted(r for rank in range(world)
                          for s, e in interleaved_blocks(h, world, rank) for r in range(s, e))
            assert rows == list(range(h))
            for rank in range(world):
                assert all(s % 64 == 0 for s, _ in interleaved_blocks(h, world, rank))


def _host_frame_worker(rank, world, port, width, height, fmt, result_path):
    """Each rank renders its band (the oracle stands in for rt_render) into
    its rows of one shared host frame (rowbands.HostFrame, what bench.py's
    host_frame fills over every GPU's own PCIe link); rank 0 saves it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(REPO))
    sys.path.insert(0, str(REPO / "tests"))
    import torch.distributed as dist

    import __graft_entry__
    from oracle_lib import Oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = __graft_entry__.load_package()
        from opencl_ray_tracer_amd import rowbands

        oracle = Oracle()
        scene = oracle.scene_reference(3, 1)
        hf = rowbands.HostFrame(height, width, fmt, rank)
        if rank == 0:
            hf.frame[...] = 0x5A5A5A5A  # poison: every row must be overwritten
        dist.barrier()
        rb, re = rowbands.band_rows(height, world, rank) if height >= world else \
            (min(rank, height), min(rank + 1, height))
        if re > rb:
            band = oracle.trace(scene, width, height, rows=(rb, re))
            hf.band(rb, re)[...] = band if fmt == "i32x4" else pkg.pack_rgba8(band)
        dist.barrier()  # every band is in
        if rank == 0:
            np.save(result_path, hf.frame.copy())
        seg = "/dev/shm/" + hf.shm.name.lstrip("/")
        hf.close()
        if rank == 0:  # the root unlinks at once, no collective in close()
            assert not os.path.exists(seg), seg
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt,world,height", [("rgba8", 2, 97), ("i32x4", 2, 97),
                                              ("rgba8", 3, 64), ("rgba8", 3, 2)])
def test_host_frame_assembly_gloo(tmp_path, oracle, fmt, world, height):
    """bench.py's host_frame: N ranks fill one shared host frame, the app's
    `pixels` (int32x4) or its Texture's RGBA8 pixels (MainState.cpp:984-994,
    :1023-1037), each writing only its own rows; rank 0 sees the whole
    frame, equal to the oracle's (packed for RGBA8)."""
    import torch.multiprocessing as mp

    sys.path.insert(0, str(REPO))
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    width = 96
    out = tmp_path / "frame.npy"
    mp.spawn(_host_frame_worker, args=(world, _free_port(), width, height, fmt, str(out)),
             nprocs=world, join=True)
    frame = np.load(out)
    want = oracle.trace(oracle.scene_reference(3, 1), width, height)
    if fmt == "rgba8":
        want = pkg.pack_rgba8(want)
        assert frame.dtype == np.uint32 and frame.shape == (height, width)
    assert np.array_equal(frame, want)

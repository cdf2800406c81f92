"""Regenerate the golden fixtures in tests/golden/ (run in the build container).

Each fixture is data only: the packed scene arrays (the reference's flattened
kernel-argument layout, MainState.cpp:646-658), the expected int32x4 frame or
its FNV-1a-64 hash, and the metadata of how it was made.

Frames come from the oracle (oracle/rt_oracle.c), the C restatement of the
reference's executeRayTracerCPU (MainState.cpp:936-972) that
tests/test_oracle.py pins against the survey's recorded reference-run
statistics and the reference's own Cube.cpp.  Reference scenes 2 and 3 depend
on glibc rand()/cosf(); storing the packed arrays freezes them.

    python tests/golden/make_golden.py            # small fixtures
    python tests/golden/make_golden.py --large    # + 4096^2 config-3 hash
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
from oracle_lib import Oracle  # noqa: E402

# name: (kind, width, height, spheres, cubes, lights, seed, k, store_frame)
CONFIGS = {
    "scene1_640x480": ("ref", 640, 480, 1, None, None, 1, None, True),
    "scene2_640x480": ("ref", 640, 480, 2, None, None, 1, None, True),
    "scene3_640x480": ("ref", 640, 480, 3, None, None, 1, None, True),
    # BASELINE.json configs[0..1]; dense objects (k = width/640), SURVEY.md §8d
    "config1_512x512": ("syn", 512, 512, 4, 1, 1, 1, 512 / 640, True),
    "config2_1920x1080": ("syn", 1920, 1080, 16, 4, 2, 2, 1920 / 640, True),
    # sparse (reference object units) variant of config 2
    "config2s_1920x1080": ("syn", 1920, 1080, 16, 4, 2, 2, 1.0, True),
}
LARGE = {
    # BASELINE.json configs[2]: 4096^2, 256 spheres + 64 cubes, dense
    "config3_4096x4096": ("syn", 4096, 4096, 256, 64, 0, 3, 4096 / 640, False),
}


def make(name, spec, oracle: Oracle, threads: int) -> None:
    kind, w, h, a, b, lights, seed, k, store = spec
    if kind == "ref":
        sc = oracle.scene_reference(a, seed)
        meta = dict(kind="reference", scene_id=a, seed=seed)
    else:
        sc = oracle.scene_synthetic(w, h, a, b, seed, k)
        meta = dict(kind="synthetic", spheres=a, cubes=b, lights=lights, seed=seed, k=k)
    t0 = time.time()
    frame = oracle.trace(sc, w, h, threads=threads)
    dt = time.time() - t0
    fnv = oracle.fnv(frame)
    # the Texture packing of the same frame (MainState.cpp:1023-1037): the
    # hash the benchmark's RGBA8 leg checks its frame against
    fnv_rgba8 = oracle.fnv(np.ascontiguousarray(oracle.pack_rgba8(frame)).view(np.int32))
    arrays = dict(sphere_origins=sc.sphere_origins, sphere_radius=sc.sphere_radius,
                  sphere_colours=sc.sphere_colours, cube_vertices=sc.cube_vertices,
                  cube_colours=sc.cube_colours, ray_dir=oracle.ray_dir(),
                  width=np.int32(w), height=np.int32(h), fnv1a64=np.uint64(fnv),
                  fnv1a64_rgba8=np.uint64(fnv_rgba8),
                  meta=np.array(repr(meta)))
    if store:
        arrays["frame"] = frame
    np.savez_compressed(HERE / f"{name}.npz", **arrays)
    size = (HERE / f"{name}.npz").stat().st_size
    print(f"{name}: fnv {fnv:016x} (rgba8 {fnv_rgba8:016x}), {dt:.1f}s oracle, {size / 1024:.0f} KiB")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--only", default=None)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    oracle = Oracle()
    todo = dict(CONFIGS)
    if args.large:
        todo.update(LARGE)
    for name, spec in todo.items():
        if args.only and args.only != name:
            continue
        make(name, spec, oracle, args.threads)


if __name__ == "__main__":
    main()

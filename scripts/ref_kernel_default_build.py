"""Informational (not a test): the reference's rayTracer.cl built as the app
builds it -- clBuildProgram(program, 0, NULL, NULL, NULL, NULL) with no
options (MainState.cpp:1302), i.e. OpenCL's default FP contraction and
relaxed divide / sqrt (oracle/_ref/rayTracer_gfx950_default.co) -- against
the IEEE build the oracle is pinned to (rayTracer_gfx950.co: no contraction,
correctly rounded divide and sqrt), on the golden fixtures.  Prints one JSON
object per fixture: pixels where the two builds differ, and where each
differs from the CPU path (the golden frame).

    python scripts/ref_kernel_default_build.py > profiles/r03/reference_kernel_default_build.jsonl
"""
import json
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tests"))
from conftest import load_golden  # noqa: E402
from ref_kernel import CODE_OBJECT, ReferenceKernel  # noqa: E402

FIELDS = ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices", "cube_colours")
FIXTURES = ["scene1_640x480", "scene2_640x480", "scene3_640x480", "config1_512x512",
            "config2_1920x1080", "config2s_1920x1080"]


def main():
    ieee = ReferenceKernel(CODE_OBJECT)
    default = ReferenceKernel(CODE_OBJECT.with_name("rayTracer_gfx950_default.co"))
    for name in FIXTURES:
        g = load_golden(name)
        scene = SimpleNamespace(**{k: g[k] for k in FIELDS})
        w, h = int(g["width"]), int(g["height"])
        a = ieee.trace(scene, w, h, g["ray_dir"])
        b = default.trace(scene, w, h, g["ray_dir"])
        px = lambda x, y: int((x != y).any(-1).sum())  # noqa: E731
        print(json.dumps({"fixture": name, "pixels": w * h,
                          "default_vs_ieee_build": px(b, a),
                          "max_channel_diff_default_vs_ieee": int(np.abs(
                              b.astype(np.int64) - a).max()),
                          "ieee_build_vs_cpu_path": px(a, g["frame"]),
                          "default_build_vs_cpu_path": px(b, g["frame"])}), flush=True)
    ieee.close()
    default.close()


if __name__ == "__main__":
    main()

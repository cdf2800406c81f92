"""Frames the automatic path choice takes to follow a jump in box overdraw
(low -> high -> low scene, int32x4, 2048^2, synchronous renders): the
kernel each frame ran.  Library from RT_HIP_LIBRARY (default in-tree)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import __graft_entry__  # noqa: E402


def main():
    pkg = __graft_entry__.load_package()
    low = pkg.Scene.synthetic(2048, 2048, 256, 64, seed=3, k=3.2)
    high = pkg.Scene.synthetic(2048, 2048, 256, 64, seed=3, k=12.8)
    seq = []
    with pkg.RayTracer(0) as rt:
        for scene, name, n in ((low, "low", 4), (high, "high", 10), (low, "low", 10)):
            for _ in range(n):
                rt.render(scene, 2048, 2048)
                seq.append((name, rt.last_kernel()))
    print(json.dumps({"library": str(pkg.library_path()),
                      "frames": seq}))


if __name__ == "__main__":
    main()

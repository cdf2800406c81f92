"""Per-frame time of the config-3 render launched directly (3 kernel
launches per frame from the host) against a hipGraph replay of the same
launches (torch.cuda.CUDAGraph captures rt_render_device's kernels on the
capture stream).  Frames are checked bit-exact between the two."""
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main(frames=200, per_graph=10):
    import torch
    import __graft_entry__
    pkg = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    w = h = 4096
    scene = pkg.Scene.synthetic(w, h, 256, 64, seed=3, k=w / 640)
    t = {n: torch.from_numpy(np.ascontiguousarray(getattr(scene, n))).to(dev)
         for n in ("sphere_origins", "sphere_radius", "sphere_colours", "cube_vertices",
                   "cube_colours")}
    ds = {n: v.data_ptr() for n, v in t.items()}
    ds.update(num_spheres=scene.num_spheres, num_cubes=scene.num_cubes)
    rt = pkg.RayTracer(0)
    out = torch.empty((h, w, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    step = rt.bind_render_device(ds, w, h, (0, h), out.data_ptr(), stream=stream.cuda_stream)
    with torch.cuda.stream(stream):
        for _ in range(5):
            step()
    torch.cuda.synchronize()
    ref = out.clone()

    def direct():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / frames

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(per_graph):
            step()
    torch.cuda.synchronize()

    def graphed():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames // per_graph):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / (frames // per_graph * per_graph)

    res = {"direct_us": [], "graph_us": []}
    for _ in range(7):
        res["direct_us"].append(direct())
        res["graph_us"].append(graphed())
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    res["bit_exact"] = bool(torch.equal(out, ref))
    res["direct_median_us"] = float(np.median(res["direct_us"]))
    res["graph_median_us"] = float(np.median(res["graph_us"]))
    print(json.dumps(res))
    rt.close()


if __name__ == "__main__":
    main()

import numpy as np, sys
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import __graft_entry__ as g
from oracle_lib import Oracle
from test_gpu_parity import EDGE_CASES, _scene_from
pkg = g.load_package(); orc = Oracle()
rt = pkg.RayTracer(0)
full = EDGE_CASES["slivers"]["cubes"]
for i in range(len(full)):
    sc = _scene_from(pkg, cubes=[full[i]])
    got,_ = rt.render(sc, 101, 77, path="binned"); want = orc.trace(sc, 101, 77)
    bad = (got!=want).any(-1)
    print("cube", i, "bad", bad.sum(), np.argwhere(bad)[:3].tolist(), got[bad][:2].tolist(), want[bad][:2].tolist())
sc = _scene_from(pkg, cubes=full)
got,_ = rt.render(sc, 101, 77, path="binned"); want = orc.trace(sc, 101, 77)
bad = (got!=want).any(-1); ys,xs = np.nonzero(bad)
print("all bad", bad.sum(), "x range", xs.min(), xs.max(), "y range", ys.min(), ys.max())
print(np.unique(got[bad].reshape(-1,4), axis=0))

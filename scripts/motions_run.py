"""C3 motion checks only (512 OBBs, 1M edges, analytic then discrete32, 5 launches each):
a short program for rocprofv3 counter passes on the motion kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
g3, o3 = synth.track_world(42, n_obstacles=472)
w = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
N = 1 << 20
s1, s2 = synth.edges(43, 8, *synth.C2_BOUNDS, N)
d1, d2 = capi.DeviceBuffer.from_array(s1), capi.DeviceBuffer.from_array(s2)
dv = capi.DeviceBuffer(N)
for mode in (0, 1):
    for r in range(5):
        w.check_motions_dev(d1.ptr, d2.ptr, N, 0, mode, dv.ptr)
    capi.sync()
print("ok")

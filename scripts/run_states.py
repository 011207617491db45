"""Runs k_states on the C2 world (PMC profiling driver): 20 launches of 1M states,
then 4 launches of 16M states."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

N, NB = 1 << 20, 16
L = capi.lib()
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
gates, obstacles = synth.track_world(42)
w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
lo, hi = synth.C2_BOUNDS
d = capi.DeviceBuffer(NB * N * 24)
for b in range(NB):
    pts = synth.sample_states(7, lo, hi, N, start=b * N)
    capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, None))
dv = capi.DeviceBuffer(NB * N)
for r in range(20):
    w.check_states_dev(d.ptr + (r % NB) * N * 24, N, 0, dv.ptr)
for r in range(0 if "1m" in sys.argv else 4):
    w.check_states_dev(d.ptr, NB * N, 0, dv.ptr)
capi.sync()
print("ok", int(dv.download(np.uint8, N).sum()))

"""Per-wave timeline of one k_states launch (debug entry epp_dbg_states_timeline):
s_memrealtime (100 MHz) at wave entry, data arrival (forced vmcnt(0)), after LDS
staging, after the item groups.  Prints percentiles of each phase in microseconds."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

L = capi.lib()
f = L.epp_dbg_states_timeline
f.restype = C.c_int32
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.c_void_p]
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
gates, obstacles = synth.track_world(42)
w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
lo, hi = synth.C2_BOUNDS
res = {}
for n in (1 << 20, 1 << 24):
    pts = synth.sample_states(7, lo, hi, n)
    d = capi.DeviceBuffer.from_array(pts)
    dv = capi.DeviceBuffer(n)
    tl = capi.DeviceBuffer(8 * 8 * 65536)
    gw = C.c_int32(0)
    for _ in range(5):
        tl.zero()
        capi.check(f(w.handle, d.ptr, n, dv.ptr, tl.ptr, C.byref(gw), None))
        capi.sync()
    t = tl.download(np.uint64, 8 * gw.value).reshape(-1, 8).astype(np.int64)
    t0 = t[:, 0].min()
    us = lambda x: x * 0.01  # noqa: E731  (100 MHz ticks)
    ph = {"entry": us(t[:, 0] - t0), "data": us(t[:, 1] - t[:, 0]), "stage": us(t[:, 2] - t[:, 1]),
          "groups": us(t[:, 3] - t[:, 2]), "end": us(t[:, 3] - t0)}
    if n == 1 << 20:  # one group per wave: its sub-phases (bitmap words, exact path)
        has = t[:, 5] > 0
        ph["words"] = us(t[:, 4] - t[:, 2])
        ph["exact"] = us(t[has, 5] - t[has, 4])
        ph["after_exact"] = us(t[has, 3] - t[has, 5])
        ph["needy_per_wave"] = (t[:, 7] >> 32).astype(np.float64)
    out = {k: {p: float(np.percentile(v, p)) for p in (0, 10, 50, 90, 100)} for k, v in ph.items()}
    out["waves"] = int(gw.value)
    xcc = t[:, 7] & 0xFFFFFFFF
    out["end_by_xcc_max"] = {int(x): float(us(t[xcc == x, 3] - t0).max()) for x in np.unique(xcc)}
    res[str(n)] = out
    print(n, json.dumps(out, indent=None))
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "timeline.json"), "w"), indent=1)

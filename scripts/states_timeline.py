"""Per-wave timeline of the headline kernel (k_states_v5, C2: 64 OBBs, 1M states): builds
a diagnostics copy of libepp.so with -DEPP_STATES_TL into scripts/dbg/ (not the product),
runs 200 launches, and prints percentiles of each wave's stamps relative to the launch's
first stamp: staging barrier, data arrived + classified, exact path done, end."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

out = os.path.join(ROOT, "scripts", "dbg")
variant = sys.argv[1] if len(sys.argv) > 1 else ""  # "" or "noexact" (-DEPP_STATES_NOEXACT: wrong answers)
lib_path = os.path.join(out, f"libepp_stl{variant}.so")
if not os.path.exists(lib_path):
    extra = "-DEPP_STATES_TL" + (" -DEPP_STATES_NOEXACT" if variant == "noexact" else "")
    subprocess.run(["make", "-s", "-j16", "-C", os.path.join(ROOT, "efficient-path-planner_amd"),
                    f"BUILD={out}/build_stl{variant}", f"LIB={lib_path}", f"EXTRA={extra}", lib_path], check=True)
capi.LIB_PATH = lib_path  # the diagnostics build behind the usual binding
L = capi.lib()
L.epp_dbg_states_tl.argtypes = [C.c_void_p, C.c_int64]
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
gates, obstacles = synth.track_world(42)
w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
N, NB = 1 << 20, 16
d = capi.DeviceBuffer(NB * N * 24)
for b in range(NB):
    pts = synth.sample_states(7, *synth.C2_BOUNDS, N, start=b * N)
    capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, None))
dv = capi.DeviceBuffer(N)
waves = 256 * 16  # single pass: 16 waves per CU
rows = []
for r in range(200):
    w.check_states_dev(d.ptr + (r % NB) * N * 24, N, 0, dv.ptr)
    if r >= 150 and r % 5 == 0:
        capi.sync()
        tl = np.zeros((waves, 6), np.uint64)
        capi.check(L.epp_dbg_states_tl(tl.ctypes.data, waves))
        rows.append(tl.astype(np.int64))
for name, k in (("staging barrier", 1), ("classified", 2), ("exact done", 3), ("end", 4)):
    v = np.concatenate([(t[:, k] - t[:, 0].min()) * 10 for t in rows]) / 1000.0  # us
    print(f"{name:16s} p1 {np.percentile(v, 1):6.2f}  p10 {np.percentile(v, 10):6.2f}  p50 {np.percentile(v, 50):6.2f}"
          f"  p90 {np.percentile(v, 90):6.2f}  p99 {np.percentile(v, 99):6.2f}  max {v.max():6.2f} us")
v = np.concatenate([(t[:, 0] - t[:, 0].min()) * 10 for t in rows]) / 1000.0
print(f"{'entry':16s} p50 {np.percentile(v, 50):6.2f} max {v.max():6.2f} us")
ex = np.concatenate([(t[:, 3] - t[:, 2]) * 10 for t in rows]) / 1000.0
print(f"exact path per wave: p50 {np.percentile(ex, 50):.2f} p90 {np.percentile(ex, 90):.2f} max {ex.max():.2f} us")
nd = np.concatenate([(t[:, 5] >> 32) & 0xFFFF for t in rows])
pr = np.concatenate([(t[:, 5] >> 48) & 0xFFFF for t in rows])
print(f"queued states per wave: p50 {np.percentile(nd, 50):.0f} p90 {np.percentile(nd, 90):.0f} max {nd.max()}"
      f"; pairs per wave: p50 {np.percentile(pr, 50):.0f} p90 {np.percentile(pr, 90):.0f} max {pr.max()}"
      f"; > 64 pairs: {np.mean(pr > 64):.2f}, > 128: {np.mean(pr > 128):.3f}")

"""Per-wave time split of the motion kernels on C3 (512 OBBs, 1M analytic edges): builds a
diagnostics copy of libepp.so with -DEPP_MOTIONS_TL into scripts/dbg/ (not the product),
runs the launch, and prints per-wave shader-clock cycles in the candidate walk, in the
flushes (exact tests) and in total, with the pairs walked / queued per wave."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

out = os.path.join(ROOT, "scripts", "dbg")
lib_path = os.path.join(out, "libepp_mtl.so")
if not os.path.exists(lib_path):
    subprocess.run(["make", "-s", "-j16", "-C", os.path.join(ROOT, "efficient-path-planner_amd"),
                    f"BUILD={out}/build_mtl", f"LIB={lib_path}", "EXTRA=-DEPP_MOTIONS_TL", lib_path], check=True)
capi.LIB_PATH = lib_path
L = capi.lib()
L.epp_dbg_motions_tl.argtypes = [C.c_void_p, C.c_int64]
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
g3, o3 = synth.track_world(42, n_obstacles=472)
w = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
N = 1 << 20
s1, s2 = synth.edges(43, 8, *synth.C2_BOUNDS, N)
d1, d2 = capi.DeviceBuffer.from_array(s1), capi.DeviceBuffer.from_array(s2)
dv = capi.DeviceBuffer(N)
kernel = sys.argv[1] if len(sys.argv) > 1 else "v5"
if kernel == "v4":
    os.environ["EPP_MOTIONS_KERNEL"] = "v4"
names = (("walk cycles", "flush cycles", "total cycles", "entries", "queued", "cell pairs") if kernel == "v4" else
         ("filter+queue", "flush cycles", "total cycles", "cand loop", "pairs", "staging"))
for mode in (0, 1):
    for r in range(20):
        w.check_motions_dev(d1.ptr, d2.ptr, N, 0, mode, dv.ptr)
    capi.sync()
    waves = N // 64
    tl = np.zeros((waves, 6), np.uint64)
    capi.check(L.epp_dbg_motions_tl(tl.ctypes.data, waves))
    tl = tl.astype(np.int64)
    live = tl[:, 2] > 0
    tl = tl[live]
    print(f"waves with work: {len(tl)}")
    print(f"-- {kernel} mode {mode}")
    for k, name in enumerate(names):
        v = tl[:, k]
        print(f"{name:14s} p10 {np.percentile(v, 10):9.0f} p50 {np.percentile(v, 50):9.0f} p90 {np.percentile(v, 90):9.0f}"
              f" max {v.max():9.0f} mean {v.mean():9.0f}")

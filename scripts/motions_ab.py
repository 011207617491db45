"""A/B timing of the C3 motion kernels (1M edges, both modes) for one library build and
environment: python scripts/motions_ab.py [lib.so] [ENV=VALUE ...]; 3 x 20 launches per
mode, HIP events, the median per-launch time (diagnostics only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
args = sys.argv[1:]
lib = args.pop(0) if args and args[0].endswith(".so") else None
for a in args:
    k, v = a.split("=", 1)
    os.environ[k] = v
from eppamd import capi, config, synth  # noqa: E402
if lib:
    capi.LIB_PATH = lib
from bench import timed_kernel_ms  # noqa: E402

L = capi.lib()
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
g3, o3 = synth.track_world(42, n_obstacles=472)
w = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
N = 1 << 20
s1, s2 = synth.edges(43, 8, *synth.C2_BOUNDS, N)
d1, d2 = capi.DeviceBuffer.from_array(s1), capi.DeviceBuffer.from_array(s2)
dv = capi.DeviceBuffer(N)
import ctypes as C  # noqa: E402
st = C.c_void_p()
capi.check(L.epp_stream_create(C.byref(st)))
out = {}
for mode in (0, 1):
    f = lambda r: w.check_motions_dev(d1.ptr, d2.ptr, N, 0, mode, dv.ptr, stream=st.value)  # noqa
    for r in range(5):
        f(r)
    ms = [timed_kernel_ms(capi, st.value, f, 20) for _ in range(3)]
    out[mode] = float(np.median(ms)) * 1e3
    capi.check(L.epp_stream_sync(st.value))
    fl = dv.download(np.uint8, N)  # (a digest of the flags: builds must agree)
    import hashlib
    out[f"h{mode}"] = hashlib.sha1(fl.tobytes()).hexdigest()[:10]
print(os.path.basename(lib or "libepp.so"), " ".join(args), f"mode0 {out[0]:.2f} us  mode1 {out[1]:.2f} us  "
      f"sha1 {out['h0']} {out['h1']}", flush=True)

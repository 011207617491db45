"""A/B timing of the headline kernel (C2: 64 OBBs, 1M states per launch over 16 resident
batches, as bench.py) for one library build: python scripts/states_ab.py [lib.so]
[ENV=VALUE ...]; 3 x 200 launches, HIP events, the median per-launch time (diagnostics
only).  With --stream also the streaming floor of the same bytes (scripts/diag_stream.hip)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
args = sys.argv[1:]
lib = args.pop(0) if args and args[0].endswith(".so") else None
stream_floor = "--stream" in args
for a in args:
    if "=" in a:
        k, v = a.split("=", 1)
        os.environ[k] = v
from eppamd import capi, config, synth  # noqa: E402
if lib:
    capi.LIB_PATH = lib
from bench import timed_kernel_ms  # noqa: E402

L = capi.lib()
N, NB = 1 << 20, 16
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
g, o = synth.track_world(42)
w = capi.World(capi.build_obbs(geom, g, o), rg, ro)
st = C.c_void_p()
capi.check(L.epp_stream_create(C.byref(st)))
st = st.value
lo, hi = synth.C2_BOUNDS
d = capi.DeviceBuffer(NB * N * 24)
for b in range(NB):
    pts = synth.sample_states(7, lo, hi, N, start=b * N)
    capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, st))
dv = capi.DeviceBuffer(N)
f = lambda r: w.check_states_dev(d.ptr + (r % NB) * N * 24, N, 0, dv.ptr, stream=st)  # noqa
for r in range(50):
    f(r)
us = float(np.median([timed_kernel_ms(capi, st, f, 200) for _ in range(3)])) * 1e3
# the flags of the last launch's batch (199 % 16): a digest to compare builds (variants must agree)
import hashlib  # noqa: E402
capi.check(L.epp_stream_sync(st))
flags = dv.download(np.uint8, N)
digest = hashlib.sha1(flags.tobytes()).hexdigest()[:12]
print(os.path.basename(lib or "libepp.so"), " ".join(a for a in args if "=" in a),
      f"c2 {us:.3f} us  {25 * N / us / 1e6:.2f} TB/s  valid {int(flags.sum())} sha1 {digest}", flush=True)
if stream_floor:
    so = os.path.join(ROOT, "scripts", "dbg", "libdiag.so")
    diag = C.CDLL(so)
    diag.diag_stream.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    for mode in (0, 1, 2):
        for blocks in (1024, 2048):
            fs = lambda r: diag.diag_stream(mode, d.ptr + (r % NB) * N * 24, N, dv.ptr, blocks, st)  # noqa
            for r in range(20):
                fs(r)
            us = float(np.median([timed_kernel_ms(capi, st, fs, 200) for _ in range(3)])) * 1e3
            print(f"stream mode{mode} blocks {blocks}: {us:.3f} us  {25 * N / us / 1e6:.2f} TB/s", flush=True)

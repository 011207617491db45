"""In-process A/B of k_states_v5 launch shapes on the bench's C2 headline (1M states per
launch, 16 resident batches rotated): configurations alternate round by round so box- and
allocation-level noise hits all of them alike.  argv: env settings, e.g.
  python scripts/v5_ab.py "" "EPP_V5_BLOCK=1024"
"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
import bench  # noqa: E402
from eppamd import capi, config, synth  # noqa: E402

cfgs = sys.argv[1:] or ["", "EPP_V5_BLOCK=1024"]
L = capi.lib()
st = C.c_void_p()
capi.check(L.epp_stream_create(C.byref(st)))
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
gates, obstacles = synth.track_world(42)
world = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
lo, hi = synth.C2_BOUNDS
N, B = 1 << 20, 16
d = capi.DeviceBuffer(N * B * 24)
for b in range(B):
    pts = synth.sample_states(7, lo, hi, N, start=b * N)
    capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, st))
dv = capi.DeviceBuffer(N)
keys = ["EPP_V5_BLOCK", "EPP_WG_PER_CU5", "EPP_V5_LDS_MIN", "EPP_V5_SPL", "EPP_BITMAP_BITS", "EPP_V5_PAIRS"]
res = {c: [] for c in cfgs}


def setenv(c):
    for k in keys:
        os.environ.pop(k, None)
    for kv in c.split():
        k, v = kv.split("=")
        os.environ[k] = v


worlds = {}
info = (C.c_int64 * 6)()
L.epp_dbg_world_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
L.epp_dbg_world_info.restype = C.c_int
for c in cfgs:  # the class grid is sized at world build (EPP_BITMAP_BITS)
    setenv(c)
    worlds[c] = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    capi.check(L.epp_dbg_world_info(worlds[c].handle, info))
    print(f"{c or 'default'}: blob {info[0]} B, staged from {info[1]}, lists {info[2]}, class cells {info[3]}",
          flush=True)
for rnd in range(12):
    for c in cfgs:
        setenv(c)
        world = worlds[c]
        f = lambda r: world.check_states_dev(d.ptr + (r % B) * N * 24, N, 0, dv.ptr, stream=st)  # noqa: E731
        f(0)
        res[c].append(bench.timed_kernel_ms(capi, st, f, 200) * 1e3)
for c in cfgs:
    v = res[c]
    print(f"{c or 'default':45s} median {statistics.median(v):.3f} us  min {min(v):.3f}  max {max(v):.3f}", flush=True)

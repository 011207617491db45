"""Diagnostics: is the k_states_v5 per-process timing spread tied to the input buffer's
placement?  Allocates the 16 x 1M-state batches several times in one process (old buffers
kept alive, so each copy lands elsewhere) and times both launch shapes on each copy."""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
import bench  # noqa: E402
from eppamd import capi, config, synth  # noqa: E402

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
batches = [synth.sample_states(7, lo, hi, N, start=b * N) for b in range(B)]
keep = []
for copy in range(4):
    d = capi.DeviceBuffer(N * B * 24)
    keep.append(d)
    for b in range(B):
        capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, batches[b].ctypes.data, batches[b].nbytes, st))
    dv = capi.DeviceBuffer(N)
    keep.append(dv)
    row = []
    for shape in ("", "1024"):
        os.environ["EPP_V5_BLOCK"] = shape
        f = lambda r: world.check_states_dev(d.ptr + (r % B) * N * 24, N, 0, dv.ptr, stream=st)  # noqa: E731
        for _ in range(50):
            f(0)
        v = [bench.timed_kernel_ms(capi, st, f, 50) * 1e3 for _ in range(6)]
        row.append(f"{shape or '2x512'}: {statistics.median(v):.3f} us")
    print(f"copy {copy} @ {d.ptr:#x}: " + "  ".join(row), flush=True)

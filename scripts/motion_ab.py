"""A/B of the C3 motion-check kernels (1M edges, 512 OBBs): EPP_MOTIONS_IMPL x EPP_MOTIONS_BLOCK,
analytic and discrete32, device time per launch from HIP events (bench.timed_kernel_ms)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
import bench  # noqa: E402
from eppamd import capi, config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
# argv[1] == "c2": the planner's case (C4 track world, 64 OBBs, short k-NN-like edges)
c2 = len(sys.argv) > 1 and sys.argv[1] == "c2"
g3, o3 = synth.track_world(100) if c2 else synth.track_world(42, n_obstacles=472)
w3 = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
lo, hi = synth.C2_BOUNDS
n = 1 << 20
s1, s2 = synth.edges(43, 8, lo, hi, n, max_len=0.25 if c2 else 0.5)
import ctypes as C  # noqa: E402
st = C.c_void_p()
capi.check(capi.lib().epp_stream_create(C.byref(st)))
d1, d2 = capi.DeviceBuffer.from_array(s1, st), capi.DeviceBuffer.from_array(s2, st)
dv = capi.DeviceBuffer(n)
out = {}
for impl, block in [tuple(x.split(":")) for x in os.environ.get("AB_CFGS", "2:512,2:1024,3:512,3:1024").split(",")]:
    os.environ["EPP_MOTIONS_IMPL"], os.environ["EPP_MOTIONS_BLOCK"] = impl, block
    for mode in [int(m) for m in os.environ.get("AB_MODES", "0,1").split(",")]:
        f = lambda r: w3.check_motions_dev(d1.ptr, d2.ptr, n, 0, mode, dv.ptr, stream=st)  # noqa: E731
        f(0)
        ms = bench.timed_kernel_ms(capi, st, f, 20)
        out[f"impl{impl}_b{block}_mode{mode}"] = round(ms * 1e3, 2)
        print(f"impl {impl} block {block} mode {mode}: {ms * 1e3:.1f} us", flush=True)
print(json.dumps(out))

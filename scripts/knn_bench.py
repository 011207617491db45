"""k-NN microbench (diagnostics): grid k-NN on the planner's node count under EPP_KNN_NPC
values, HIP events on one stream (the cached-workspace entry point)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd"), ROOT]
from eppamd import capi, synth  # noqa: E402
from bench import timed_kernel_ms  # noqa: E402

L = capi.lib()
st = C.c_void_p()
capi.check(L.epp_stream_create(C.byref(st)))
st = st.value
nodes = synth.sample_states(5, [-6, -6, 0], [6, 6, 2], 63000)
d_n = capi.DeviceBuffer.from_array(nodes)
d_k = capi.DeviceBuffer(4 * 16 * len(nodes))
ref = capi.knn(nodes, 16, method="brute")
cfgs = (("0", "2"), ("1", "2"), ("2", "2"), ("1", "1.5"), ("1", "2.5"))
if len(sys.argv) > 1:  # e.g. "1:2" -> tile 1, npc 2 only
    cfgs = [tuple(a.split(":")) for a in sys.argv[1:]]
for tile, npc in cfgs:
    os.environ["EPP_KNN_TILE"] = tile
    os.environ["EPP_KNN_NPC"] = npc
    f = lambda r: capi.check(L.epp_knn_grid(d_n.ptr, len(nodes), 16, 0.0, d_k.ptr, st))  # noqa: E731
    f(0)
    ms = timed_kernel_ms(capi, st, f, 10)
    ok = np.array_equal(d_k.download(np.int32, 16 * len(nodes)).reshape(-1, 16), ref)
    print(f"tile {tile} npc {npc}: {ms * 1e3:.1f} us per call, exact={ok}", flush=True)

"""Timed-region overhead probe (diagnostics): the bench's 20-step headline shape (one captured
graph of 20 k_states_v5 launches over rotating 1M-state batches), its wall time per step
with the closing synchronisation done three ways -- hipStreamSynchronize (the bench),
spinning on hipStreamQuery, spinning on hipEventQuery of the closing event -- beside the
HIP-event time of the kernels.  Median of 40 repetitions each."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd"), ROOT]
from eppamd import capi, config, synth  # noqa: E402

K, NB, N = 20, 16, 1 << 20
L = capi.lib()
hip = C.CDLL("libamdhip64.so")
hip.hipStreamQuery.argtypes = [C.c_void_p]
hip.hipEventQuery.argtypes = [C.c_void_p]
st = C.c_void_p()
capi.check(L.epp_stream_create(C.byref(st)))
st = st.value
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
geom = config.geometry(cfg)
rg, ro = config.inflate_radii(cfg)
g, o = synth.track_world(42)
w = capi.World(capi.build_obbs(geom, g, o), rg, ro)
lo, hi = synth.C2_BOUNDS
d = capi.DeviceBuffer(NB * N * 24)
for b in range(NB):
    pts = synth.sample_states(7, lo, hi, N, start=b * N)
    capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, st))
dv = capi.DeviceBuffer(N)
gr = C.c_void_p()
capi.check(L.epp_graph_begin(st))
for i in range(K):
    w.check_states_dev(d.ptr + (i % NB) * N * 24, N, 0, dv.ptr, stream=st)
capi.check(L.epp_graph_end(st, C.byref(gr)))
ev0, ev1 = C.c_void_p(), C.c_void_p()
capi.check(L.epp_event_create(C.byref(ev0)))
capi.check(L.epp_event_create(C.byref(ev1)))
for _ in range(5):
    capi.check(L.epp_graph_launch(gr, st))
capi.check(L.epp_stream_sync(st))


def once(mode):
    t0 = time.perf_counter()
    capi.check(L.epp_event_record(ev0, st))
    capi.check(L.epp_graph_launch(gr, st))
    capi.check(L.epp_event_record(ev1, st))
    if mode == "sync":
        capi.check(L.epp_stream_sync(st))
    elif mode == "stream_query":
        while hip.hipStreamQuery(st) != 0:
            pass
    else:
        while hip.hipEventQuery(ev1) != 0:
            pass
    t1 = time.perf_counter()
    ms = C.c_float()
    capi.check(L.epp_event_elapsed_ms(ev0, ev1, C.byref(ms)))
    return (t1 - t0) * 1e3 / K, ms.value / K


for mode in ("sync", "stream_query", "event_query", "sync"):
    r = np.array([once(mode) for _ in range(40)])
    print(f"{mode:13s} wall {np.median(r[:, 0]) * 1e3:7.3f} us/step  events {np.median(r[:, 1]) * 1e3:7.3f} us/step", flush=True)

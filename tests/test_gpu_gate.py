"""GPU tests of the stream gate (epp_gate_*, include/epp.h): the launch-overhead tool
bench.py uses so that the HIP events of its kernel-duration measurement bracket the K
kernels and not the graph's submission.  No reference counterpart."""
import ctypes as C
import time

import numpy as np
import pytest

from eppamd import capi, config, synth

pytestmark = pytest.mark.gpu


def _stream():
    L = capi.lib()
    s = C.c_void_p()
    capi.check(L.epp_stream_create(C.byref(s)))
    return L, s.value


def test_gate_holds_until_released_and_times_out():
    L, s = _stream()
    g = C.c_void_p()
    capi.check(L.epp_gate_create(C.byref(g)))
    try:
        # released: the work behind it completes right after the release
        capi.check(L.epp_gate_hold(g, 5000, s))
        time.sleep(0.05)
        t = time.perf_counter()
        capi.check(L.epp_gate_release(g))
        capi.check(L.epp_stream_sync(s))
        assert time.perf_counter() - t < 1.0
        # never released: the gate ends by itself at its timeout (no hang)
        t = time.perf_counter()
        capi.check(L.epp_gate_hold(g, 200, s))
        capi.check(L.epp_stream_sync(s))
        el = time.perf_counter() - t
        assert 0.15 < el < 3.0, el
        # out-of-range timeouts are rejected
        with pytest.raises(capi.EppError):
            capi.check(L.epp_gate_hold(g, 0, s))
    finally:
        L.epp_gate_destroy(g)
        L.epp_stream_destroy(s)


def test_gated_graph_replay_equals_plain_launch(cfg, geom):
    """A graph of state checks queued behind the gate gives the same flags as the plain
    launches, and its events bracket the kernels (a positive, sub-millisecond time)."""
    L, s = _stream()
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    n = 1 << 20
    pts = synth.sample_states(7, *synth.C2_BOUNDS, n)
    d_x = capi.DeviceBuffer.from_array(pts, s)
    d_a, d_b = capi.DeviceBuffer(n), capi.DeviceBuffer(n)
    w.check_states_dev(d_x.ptr, n, 0, d_a.ptr, stream=s)
    capi.check(L.epp_stream_sync(s))
    graph = C.c_void_p()
    capi.check(L.epp_graph_begin(s))
    for _ in range(4):
        w.check_states_dev(d_x.ptr, n, 0, d_b.ptr, stream=s)
    capi.check(L.epp_graph_end(s, C.byref(graph)))
    g = C.c_void_p()
    e0, e1 = C.c_void_p(), C.c_void_p()
    capi.check(L.epp_gate_create(C.byref(g)))
    capi.check(L.epp_event_create(C.byref(e0)))
    capi.check(L.epp_event_create(C.byref(e1)))
    try:
        capi.check(L.epp_gate_hold(g, 5000, s))
        capi.check(L.epp_event_record(e0, s))
        capi.check(L.epp_graph_launch(graph, s))
        capi.check(L.epp_event_record(e1, s))
        capi.check(L.epp_gate_release(g))
        capi.check(L.epp_stream_sync(s))
        ms = C.c_float()
        capi.check(L.epp_event_elapsed_ms(e0, e1, C.byref(ms)))
        assert 0.0 < ms.value < 1.0, ms.value
        assert np.array_equal(d_a.download(np.uint8, n), d_b.download(np.uint8, n))
    finally:
        L.epp_gate_destroy(g)
        L.epp_event_destroy(e0)
        L.epp_event_destroy(e1)
        L.epp_graph_destroy(graph)
        L.epp_stream_destroy(s)

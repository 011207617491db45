"""Kernel microbenchmarks (diagnostics; not the driver's bench).  Times the validity
kernels under different inputs / launch knobs with HIP events on one stream."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, config, synth  # noqa: E402

sys.path.insert(0, ROOT)
from bench import timed_kernel_ms  # noqa: E402

N = 1 << 20
NB = 16


def main():
    L = capi.lib()
    st = C.c_void_p()
    capi.check(L.epp_stream_create(C.byref(st)))
    st = st.value
    cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    w2 = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    w0 = capi.World(np.zeros(0, capi.OBB_DTYPE), rg, ro)
    lo, hi = synth.C2_BOUNDS
    d = capi.DeviceBuffer(NB * N * 24)
    for b in range(NB):
        pts = synth.sample_states(7, lo, hi, N, start=b * N)
        capi.check(L.epp_memcpy_h2d(d.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, st))
    dz = capi.DeviceBuffer(NB * N * 24)
    for b in range(NB):
        pts = synth.sample_states(9, np.array([-6, -6, 1.6]), hi, N, start=b * N)
        capi.check(L.epp_memcpy_h2d(dz.ptr + b * N * 24, pts.ctypes.data, pts.nbytes, st))
    dv = capi.DeviceBuffer(N)
    res = {}

    import re
    pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None

    def run(name, world, buf, env=None):
        if pat and not pat.search(name):
            return
        for k, v in (env or {}).items():
            os.environ[k] = str(v)
        f = lambda r: world.check_states_dev(buf.ptr + (r % NB) * N * 24, N, 0, dv.ptr, stream=st)  # noqa
        for r in range(3):
            f(r)
        ms = timed_kernel_ms(capi, st, f, 32)
        for k in (env or {}):
            del os.environ[k]
        res[name] = {"us": ms * 1e3, "GBs": 25 * N / (ms * 1e-3) / 1e9}
        print(name, res[name], flush=True)

    if not os.path.exists(os.path.join(ROOT, "scripts", "libdiag.so")):
        os.system(f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o {ROOT}/scripts/libdiag.so "
                  f"{ROOT}/scripts/diag_stream.hip")
    diag = C.CDLL(os.path.join(ROOT, "scripts", "libdiag.so"))
    diag.diag_stream.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    dbig = capi.DeviceBuffer(NB * N)
    for mode in (0,):
        f = lambda r: diag.diag_stream(mode, d.ptr + (r % NB) * N * 24, N, dv.ptr, 1024, st)  # noqa
        f(0)
        ms = timed_kernel_ms(capi, st, f, 32)
        res[f"stream_mode{mode}"] = {"us": ms * 1e3, "GBs": 25 * N / (ms * 1e-3) / 1e9}
        print(f"stream_mode{mode}", res[f"stream_mode{mode}"], flush=True)
        f = lambda r: diag.diag_stream(mode, d.ptr, NB * N, dbig.ptr, 4096, st)  # noqa
        f(0)
        ms = timed_kernel_ms(capi, st, f, 8)
        res[f"stream_mode{mode}_16M"] = {"us": ms * 1e3, "GBs": 25 * NB * N / (ms * 1e-3) / 1e9}
        print(f"stream_mode{mode}_16M", res[f"stream_mode{mode}_16M"], flush=True)

    def big(name, world, env=None):
        if pat and not pat.search(name):
            return
        for k, v in (env or {}).items():
            os.environ[k] = str(v)
        f = lambda r: world.check_states_dev(d.ptr, NB * N, 0, dbig.ptr, stream=st)  # noqa
        f(0)
        ms = timed_kernel_ms(capi, st, f, 8)
        for k in (env or {}):
            del os.environ[k]
        res[name] = {"us": ms * 1e3, "GBs": 25 * NB * N / (ms * 1e-3) / 1e9}
        print(name, res[name], flush=True)

    for kern in ("v5", "v4", "generic"):
        e = {"EPP_STATES_KERNEL": kern}
        run(f"c2_{kern}", w2, d, e)
        big(f"c2_{kern}_16M", w2, e)
        run(f"c2_{kern}_empty_world", w0, d, e)
    run("c2_v5_b1024", w2, d, {"EPP_V5_BLOCK": 1024})
    big("c2_v5_b1024_16M", w2, {"EPP_V5_BLOCK": 1024})
    # motions, C3
    g3, o3 = synth.track_world(42, n_obstacles=472)
    w3 = capi.World(capi.build_obbs(geom, g3, o3), rg, ro)
    s1, s2 = synth.edges(43, 8, lo, hi, N)
    d1, d2 = capi.DeviceBuffer.from_array(s1), capi.DeviceBuffer.from_array(s2)
    for mode in (0, 1):
        for env in ({},):
            for k, v in env.items():
                os.environ[k] = str(v)
            f = lambda r: w3.check_motions_dev(d1.ptr, d2.ptr, N, 0, mode, dv.ptr, stream=st)  # noqa
            f(0)
            ms = timed_kernel_ms(capi, st, f, 5)
            for k in env:
                del os.environ[k]
            key = f"c3_motion_mode{mode}" + "".join(f"_{k}={v}" for k, v in env.items())
            res[key] = {"us": ms * 1e3, "edges_per_s": N / (ms * 1e-3)}
            print(key, res[key], flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "kbench.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

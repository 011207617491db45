"""bench.py's native CPU baseline driver (oracle/cpu_bench, test infrastructure) on CPU:
the C5 input file bench.py writes is read back by the native driver, whose refit and
online loops produce the oracle's row counts."""
import json
import os
import subprocess
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_cpu_bench_reads_bench_input(cfg, geom):
    import bench
    import oracle as O
    from eppamd import config, synth
    rg, ro = config.inflate_radii(cfg)
    g, o = synth.track_world(42)
    wp = synth.random_track_waypoints(3, 12)
    refit = synth.random_track_waypoints(10_000, 12)
    window = [(0, 2), (1, 5)]
    path = bench.write_c5_input(geom, g, o, rg, ro, 0.2, 1.0, 2.0, 0.1, wp, window, refit, steps=50)
    try:
        exe = os.path.join(ROOT, "oracle", "cpu_bench")
        r = subprocess.run([exe, path], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        out = json.loads(r.stdout)
    finally:
        os.unlink(path)
    assert out["c5_refit_native"]["steps"] == 180 and out["c5_online_native"]["steps"] == 50
    assert out["refit_rows"] == len(O.generate_trajectory(refit, 1.0, 2.0, 0.1))
    # the last step's refit: the window with the last perturbed gate's centre moved
    (gate, wi), d = bench.c5_steps(window, 50)[-1]
    wp2 = wp.copy()
    wp2[wi, :2] = [g[gate, 0] + d[0], g[gate, 1] + d[1]]
    assert out["online_rows"] == len(O.generate_trajectory(wp2, 1.0, 2.0, 0.1, 0.0, bench.C5_V0, bench.C5_A0))
    assert out["c5_online_native"]["p50_us"] > 0 and np.isfinite(out["c5_refit_native"]["p99_us"])

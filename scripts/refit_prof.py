"""Latency probe of the single-track refit path (C5): 300 calls of generate_trajectory
(12 segments, dt = 0.1) through ctypes; prints the per-call wall-clock percentiles.  Run
under `rocprofv3 --kernel-trace --stats` for the kernel durations."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
from eppamd import capi, synth  # noqa: E402

wp = synth.random_track_waypoints(10_000, 12)
lat = np.zeros(300)
for r in range(len(lat)):
    t = time.perf_counter()
    capi.generate_trajectory(wp, 1.0, 2.0, 0.1)
    lat[r] = time.perf_counter() - t
lat = lat[30:] * 1e6
print(f"refit: p50 {np.percentile(lat, 50):.1f} us  p99 {np.percentile(lat, 99):.1f} us  min {lat.min():.1f} us")

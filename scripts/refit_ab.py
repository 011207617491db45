"""Refit latency A/B (round 6): p50 / p90 microseconds of capi.generate_trajectory (the
native k_refit path, host buffers in and out) over a 12-segment C5 problem, in this
process's EPP_REFIT_REFINE setting.  Usage: EPP_REFIT_REFINE=0|1 python scripts/refit_ab.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd")]
import numpy as np  # noqa: E402

from eppamd import capi, synth  # noqa: E402

wp = synth.random_track_waypoints(10_000, 12)
for _ in range(200):
    capi.generate_trajectory(wp, 1.0, 2.0, 0.1)
lat = np.zeros(3000)
for i in range(len(lat)):
    t = time.perf_counter()
    capi.generate_trajectory(wp, 1.0, 2.0, 0.1)
    lat[i] = time.perf_counter() - t
print(f"refine={os.environ.get('EPP_REFIT_REFINE', '1')} generate_trajectory p50 {np.median(lat) * 1e6:.1f} us "
      f"p90 {np.quantile(lat, 0.9) * 1e6:.1f} us", flush=True)

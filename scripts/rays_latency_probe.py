"""Latency of the small ray batches (diagnostics): World::checkRaysBoth / checkRayValid on
the C4 track world through the PathPlanner binding, wall time per call for batch sizes
1..1024 (the shortcut's batch is ~700 rays).  python scripts/rays_latency_probe.py
(scripts/small_rays_trace.py reads the kernel durations from a kernel trace of it)"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# EPP_PKG: another build of the package (scripts/ab_pkg.sh) for a same-box A/B
sys.path[:0] = [ROOT, os.environ.get("EPP_PKG") or os.path.join(ROOT, "efficient-path-planner_amd")]
import numpy as np  # noqa: E402

import online_traj_planner as otp  # noqa: E402
from eppamd import config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
cfg["world_properties"]["upper_bound"] = [6, 6, 2]
fd, path = tempfile.mkstemp(suffix=".json")
with os.fdopen(fd, "w") as f:
    json.dump(cfg, f)
gates, obstacles = synth.track_world(100)
pp = otp.PathPlanner(gates, obstacles, path)
os.unlink(path)
rs = np.random.RandomState(1)
for n in (1, 16, 64, 256, 512, 768, 1024):
    s1 = synth.sample_states(3, [-6, -6, 0], [6, 6, 2], n)
    s2 = s1 + rs.uniform(-1, 1, (n, 3))
    for _ in range(50):
        pp.check_rays_both(s1, s2)
    ts = []
    for _ in range(500):
        t = time.perf_counter()
        pp.check_rays_both(s1, s2)
        ts.append((time.perf_counter() - t) * 1e6)
    print(f"check_rays_both n {n}: p50 {np.median(ts):.1f} us, p10 {np.percentile(ts, 10):.1f}, p90 {np.percentile(ts, 90):.1f}",
          flush=True)
a, b = (0.0, 0.0, 1.0), (0.5, 0.5, 1.0)
ts = []
for _ in range(500):
    t = time.perf_counter()
    pp.check_ray_valid(a, b, False)
    ts.append((time.perf_counter() - t) * 1e6)
print(f"check_ray_valid (one ray): p50 {np.median(ts):.1f} us", flush=True)

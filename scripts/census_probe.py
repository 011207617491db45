"""Diagnostics: the symmetrised search on the restricted rows after the whole table's goal-edge
count (host_planner.cpp solve) against the whole-table search, timed on goals outside the
sampling box (the C4 box, track world 100, 65,536 samples): plan_once per seed, the
planner's own split."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
import numpy as np  # noqa: E402
import online_traj_planner as otp  # noqa: E402
from eppamd import config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
cfg["world_properties"]["upper_bound"] = [6, 6, 2]
cfg["path_planner_properties"]["samples_fmt"] = 65536
fd, path = tempfile.mkstemp(suffix=".json")
with os.fdopen(fd, "w") as f:
    json.dump(cfg, f)
gates, obstacles = synth.track_world(100)
pp = otp.PathPlanner(gates, obstacles, path)
s, g = np.array([0, 5.0, 1.0]), np.array([0, 6.4, 1.0])
pp.plan_once(s, g, 65536, 999)  # warm
ts, keys = [], ("ms_device", "ms_search", "ms_restricted_max", "symmetrised_after_census", "fallbacks", "astar_pops")
for seed in range(int(os.environ.get("EPP_PROBE_CALLS", "20"))):
    before = pp.last_stats()
    t = time.perf_counter()
    pp.plan_once(s, g, 65536, seed)
    ts.append((time.perf_counter() - t) * 1e3)
    after = pp.last_stats()
    d = {k: round(after.get(k, 0) - before.get(k, 0), 4) for k in keys}
    print(f"seed {seed}: {ts[-1]:.3f} ms {d}", flush=True)
print(f"EPP_PLAN_ELLIPSE {os.environ.get('EPP_PLAN_ELLIPSE', 'default')}: plan_once p50 {np.median(ts):.3f} ms", flush=True)
os.unlink(path)

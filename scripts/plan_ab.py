"""Full-plan A/B (diagnostics): OnlineTrajGenerator.pre_compute_traj on the C4 track with
the segments planned concurrently (default) or one after the other (EPP_PLAN_CONCURRENT=0)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "efficient-path-planner_amd"), ROOT]
import online_traj_planner as otp  # noqa: E402
from eppamd import config, synth  # noqa: E402

cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
cfg["world_properties"]["lower_bound"] = [-6, -6, 0]
cfg["world_properties"]["upper_bound"] = [6, 6, 2]
cfg["path_planner_properties"]["samples_fmt"] = 65536
geom = config.geometry(cfg)
fd, path = tempfile.mkstemp(suffix=".json")
with os.fdopen(fd, "w") as f:
    json.dump(cfg, f)
gates, obstacles = synth.track_world(100)
cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
modes = sys.argv[1:] or ["1:4", "0:1"]  # concurrent:threads
res = {m: [] for m in modes}
for rep in range(12):
    for mode in modes:
        os.environ["EPP_PLAN_CONCURRENT"], os.environ["EPP_PLAN_THREADS"] = mode.split(":")
        t = time.perf_counter()
        otg.pre_compute_traj(0.0)
        res[mode].append((time.perf_counter() - t) * 1e3)
for mode, v in res.items():
    v = sorted(v[2:])
    print(f"concurrent={mode}: min {v[0]:.2f} median {v[len(v) // 2]:.2f} max {v[-1]:.2f} ms per track", flush=True)
os.unlink(path)

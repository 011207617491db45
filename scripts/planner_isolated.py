"""One planner thread, 20 gate-to-gate segments (C4 world, 65,536 samples, k = 16), for an
isolated rocprofv3 kernel trace of the planner's kernels (profiles/rNN_planner_isolated.csv):

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plan -o run -- python3 scripts/planner_isolated.py

EPP_PLAN_THREADS=1 and plan_path one segment at a time: no other planner thread's kernels
overlap, so each kernel's average is its time alone.  Two warm-up plans come first (their
launches are in the trace as well: 22 plans, first 2 cold)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
os.environ["EPP_PLAN_THREADS"] = "1"

import numpy as np  # noqa: E402

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
pp = otp.PathPlanner(gates, obstacles, path)
pairs = [(cps[2 * s], cps[2 * s + 1]) for s in range(len(cps) // 2)]
for s, g in pairs[:2]:
    pp.plan_path(s, g, 2.0)
ts, st = [], []
for i in range(20):
    s, g = pairs[i % len(pairs)]
    t = time.perf_counter()
    pp.plan_path(s, g, 2.0)
    ts.append((time.perf_counter() - t) * 1e3)
    st.append(pp.last_stats())
os.unlink(path)
print(json.dumps({"segments": 20, "ms_p50": float(np.median(ts)), "ms_mean": float(np.mean(ts)),
                  "device_ms_p50": float(np.median([x["ms_device"] for x in st])),
                  "search_ms_p50": float(np.median([x["ms_search"] for x in st])),
                  "nodes_p50": float(np.median([x["states_valid"] for x in st])),
                  "rows_down": [int(x["rows_downloaded"]) for x in st]}), flush=True)

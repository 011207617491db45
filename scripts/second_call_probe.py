import json, os, sys, tempfile, time
ROOT='/root/repo' if os.path.exists('/root/repo') else os.environ['GRAFT_REPO_ROOT']
sys.path[:0]=[ROOT, os.path.join(ROOT,'efficient-path-planner_amd')]
import numpy as np
import online_traj_planner as otp
from eppamd import config, synth
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
cfg["world_properties"]["lower_bound"] = [-6, -6, 0]; cfg["world_properties"]["upper_bound"] = [6, 6, 2]
cfg["path_planner_properties"]["samples_fmt"] = 65536
geom = config.geometry(cfg)
fd, path = tempfile.mkstemp(suffix=".json"); os.write(fd, json.dumps(cfg).encode()); os.close(fd)
gates, obstacles = synth.track_world(100)
cps = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
otg = otp.OnlineTrajGenerator(cps[0], cps[-1], gates, obstacles, path)
for c in range(4):
    t = time.perf_counter(); otg.pre_compute_traj(0.0); el = (time.perf_counter() - t) * 1e3
    s = otg.planner_stats()
    print(c, round(el,3), {k: (round(v,3) if isinstance(v,float) else v) for k,v in s.items() if k.startswith('ms') or k in ('astar_pops','fallbacks')}, flush=True)

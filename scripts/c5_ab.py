"""A/B of the native C5 loops (tools/c5_native) between the current libepp.so and other
builds (diagnostics only): python scripts/c5_ab.py BIN [BIN ...] -- each BIN a c5_native
built against one library (scripts/c5_ab_build.sh); the binaries run alternately, 3
times each, and the JSON lines are printed as they come."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd")]
import bench  # noqa: E402
from eppamd import config, synth  # noqa: E402

bins = sys.argv[1:] or [os.path.join(ROOT, "tools", "c5_native")]
cfg = config.load(os.path.join(ROOT, "configs", "config.json"))
rg, ro = config.inflate_radii(cfg)
tg = cfg["trajectory_generator_properties"]
md = cfg["path_planner_properties"]["min_dist_check_traj_collision"]
c5cfg, c5path, geom, g, o, wp, window = bench.c5_setup()
f = bench.write_c5_input(geom, g, o, rg, ro, md, tg["max_velocity"], tg["max_acceleration"], tg["sampling_interval"],
                         wp, window, synth.random_track_waypoints(10_000, 12))
for rep in range(3):
    for b in bins:
        r = subprocess.run([b, c5path, f], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            print(b, "failed", r.returncode, r.stderr[-400:], flush=True)
            sys.exit(1)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        print(os.path.basename(b), rep, json.dumps({k: v.get("p50_us") if isinstance(v, dict) else v
                                                     for k, v in d.items()}), flush=True)

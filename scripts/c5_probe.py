"""Writes the C5 probe's inputs (config, gates, obstacles, waypoints, 100 lookahead rows)
under gpurun_out/ and runs scripts/c5_probe (diagnostics only)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd"), os.path.join(ROOT, "oracle")]
import bench  # noqa: E402

cfg, path, geom, gates, obstacles, wp, window = bench.c5_setup()
import polynomial_trajectory as pt  # noqa: E402

tg = cfg["trajectory_generator_properties"]
rows = np.asarray(pt.generate_trajectory(wp, tg["max_velocity"], tg["max_acceleration"], tg["sampling_interval"]))
out = os.path.join(ROOT, "gpurun_out")
os.makedirs(out, exist_ok=True)


def dump(name, m):
    m = np.atleast_2d(np.asarray(m, float))
    with open(os.path.join(out, name), "w") as f:
        f.write(f"{m.shape[0]} {m.shape[1]}\n")
        np.savetxt(f, m, fmt="%.17g")


dump("c5_gates.txt", gates)
dump("c5_obst.txt", obstacles)
dump("c5_wp.txt", wp)
dump("c5_rows.txt", rows[:100])
with open(os.path.join(out, "c5_cfg.txt"), "w") as f:
    f.write(path + "\n")
r = subprocess.run([os.path.join(ROOT, "scripts", "c5_probe"), out])
os.unlink(path)
sys.exit(r.returncode)

"""C5 step broken into its three calls (p50 over 500 steps each, microseconds): the
product (PathPlanner.update_gate_pos, check_trajectory_validity, polynomial_trajectory.
generate_trajectory) and the CPU oracle's counterparts (world rebuild, minDistance check,
min-snap + sampling)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-path-planner_amd"), os.path.join(ROOT, "oracle")]
import bench  # noqa: E402
from eppamd import config  # noqa: E402

cfg, path, geom, gates, obstacles, wp, window = bench.c5_setup()
tg = cfg["trajectory_generator_properties"]
vmax, amax, dt = tg["max_velocity"], tg["max_acceleration"], tg["sampling_interval"]
md = cfg["path_planner_properties"]["min_dist_check_traj_collision"]
v0, a0 = np.array([0.4, -0.2, 0.1]), np.array([0.0, 0.3, 0.0])
import online_traj_planner as otp  # noqa: E402
import polynomial_trajectory as pt  # noqa: E402
import oracle as O  # noqa: E402

pp = otp.PathPlanner(gates, obstacles, path)
rows = pt.generate_trajectory(wp, vmax, amax, dt, 0.0, v0, a0)
pp.check_trajectory_validity(rows[:100], md)
g, wi = window[0]
N = 500


def p50(f):
    lat = np.zeros(N)
    for s in range(N):
        t = time.perf_counter()
        f(s)
        lat[s] = time.perf_counter() - t
    return f"p50 {np.percentile(lat[50:], 50) * 1e6:7.1f}  p99 {np.percentile(lat[50:], 99) * 1e6:7.1f} us"


def upd(s):
    pose = gates[g, :6].copy()
    pose[0] += 0.01 * (s % 7)
    pp.update_gate_pos(g, pose)


print("gpu update_gate_pos        ", p50(upd))
print("gpu check_trajectory_valid ", p50(lambda s: pp.check_trajectory_validity(rows[:100], md)))
print("gpu generate_trajectory    ", p50(lambda s: pt.generate_trajectory(wp, vmax, amax, dt, 0.0, v0, a0)))
rg = float(cfg["world_properties"]["inflate_radius"]["gate"])
ro = float(cfg["world_properties"]["inflate_radius"]["obstacle"])
w = O.world_build(geom, gates, obstacles, rg, ro)
print("cpu world_build            ", p50(lambda s: O.world_build(geom, gates, obstacles, rg, ro)))
print("cpu check_states_mindist   ", p50(lambda s: O.check_states_mindist(w, rows[:100][:, [0, 3, 6]], md)))
print("cpu generate_trajectory    ", p50(lambda s: O.generate_trajectory(wp, vmax, amax, dt, 0.0, v0, a0)))
os.unlink(path)

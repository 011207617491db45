"""C5 online step A/B (diagnostics): bench.py's c5_online GPU leg (update_gate_pos ->
check_trajectory_validity_and_generate, the check and the refit in one launch), p50 / p90
microseconds over 3 x 1000 steps, with the package of EPP_PKG (scripts/ab_pkg.sh) or this
tree's.  python scripts/c5_step_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.environ.get("EPP_PKG") or os.path.join(ROOT, "efficient-path-planner_amd")]
import online_traj_planner  # noqa: E402,F401  (first: bench's own path entry comes later)
import numpy as np  # noqa: E402

import bench  # noqa: E402

tg_cfg, path, geom, gates, obstacles, wp, window = bench.c5_setup()
tg = tg_cfg["trajectory_generator_properties"]
md = tg_cfg["path_planner_properties"]["min_dist_check_traj_collision"]
for r in range(3):
    lat = bench.c5_online(path, geom, gates, obstacles, wp, window, tg["max_velocity"], tg["max_acceleration"],
                          tg["sampling_interval"], md)
    print(f"{os.path.basename(os.environ.get('EPP_PKG', '') or 'cur')} run {r}: C5 step p50 {np.median(lat):.1f} us, "
          f"p90 {np.percentile(lat, 90):.1f} us", flush=True)
os.unlink(path)

import os, sys, numpy as np
sys.path[:0] = ["/root/repo/efficient-path-planner_amd", "/root/repo/oracle", "/root/repo/tests"]
import online_traj_planner as otp
from eppamd import synth, config
import oracle as O
CONFIG = "/root/repo/configs/config.json"
cfg = config.load(CONFIG); geom = config.geometry(cfg); rg, ro = config.inflate_radii(cfg)
g, o, start, goal = synth.c1_world()
w = O.world_build(geom, g, o, rg, ro)
for trial in range(3):
    a = otp.PathPlanner(g, o, CONFIG); b = otp.PathPlanner(g, o, CONFIG)
    pa = a.plan_path(start, goal, 2.0); sa = a.last_stats()
    pb = b.plan_path(start, goal, 2.0); sb = b.last_stats()
    print(trial, len(pa), len(pb), sa["fallbacks"], sb["fallbacks"], sa["edges_checked"], sb["edges_checked"], sa["states_valid"], sb["states_valid"], flush=True)
    print("   ray s->g a:", a.check_ray_valid(start, goal, False) if hasattr(a, "check_ray_valid") else "-", flush=True)
lo, hi = synth.C1_BOUNDS
for seed in (1, 2, 3):
    pp = otp.PathPlanner(g, o, CONFIG)
    got = pp.plan_once(start, goal, 4096, seed)
    exp, st = O.plan_once(w, rg, ro, lo, hi, start, goal, 4096, seed, 16, False, 8)
    print("seed", seed, None if got is None else len(got), None if exp is None else len(exp), got is not None and exp is not None and np.array_equal(got, exp), pp.last_stats())

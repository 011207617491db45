"""CPU checks of the "ompl" path simplification's restatement (oracle/track_planner.py
smooth_bspline: OMPL 1.6 PathSimplifier::smoothBSpline, src/PathPlanner.cpp:282-313).

In free space every state and motion check passes, so smoothBSpline reduces to its
geometric iteration: subdivide, move every even interior state to the midpoint of its
neighbours' midpoints with it, stop after 5 steps or a step that moves nothing.  That
iteration is written here a second, independent way (numpy over whole arrays) and
compared bit for bit; near obstacles the restatement must keep every state and motion it
produces valid (the validators decide which moves happen)."""
import numpy as np

import oracle as O
import track_planner as TP
from eppamd import config, synth

from conftest import CONFIG


def _free_space_smoothing(seg, steps=5):
    s = np.asarray(seg, float)
    if len(s) < 3:
        return s
    for _ in range(steps):
        sub = np.empty((2 * len(s) - 1, 3))
        sub[0::2] = s
        sub[1::2] = s[:-1] + (s[1:] - s[:-1]) * 0.5
        s = sub
        prev, cur, nxt = s[1:-2:2], s[2:-1:2], s[3::2]
        t1 = prev + (cur - prev) * 0.5
        t2 = cur + (nxt - cur) * 0.5
        t = t1 + (t2 - t1) * 0.5
        d = np.sqrt(((cur[:, 0] - t[:, 0]) ** 2 + (cur[:, 1] - t[:, 1]) ** 2) + (cur[:, 2] - t[:, 2]) ** 2)
        move = d > np.finfo(np.float64).eps
        s[2:-1:2][move] = t[move]
        if not move.any():
            break
    return s


def _world(obstacles_far: bool):
    cfg = config.load(CONFIG)
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    if obstacles_far:  # every object moved 100 m away: free space around the paths
        gates = gates.copy()
        obstacles = obstacles.copy()
        gates[:, 0] += 100.0
        obstacles[:, 0] += 100.0
    return O.world_build(geom, gates, obstacles, rg, ro), rg, ro


def test_smooth_bspline_free_space_equals_geometric_iteration():
    w, rg, ro = _world(True)
    rs = np.random.RandomState(3)
    for n in (2, 3, 4, 7):
        seg = np.cumsum(rs.uniform(-0.5, 0.5, (n, 3)), 0) + [0, 0, 1.0]
        got = np.array(TP.smooth_bspline(seg, w, rg, ro, False))
        exp = _free_space_smoothing(seg)
        assert got.shape == exp.shape == ((len(seg) - 1) * 32 + 1, 3) if n >= 3 else got.shape == (n, 3)
        assert np.array_equal(got, exp), n
        assert np.array_equal(got[0], seg[0]) and np.array_equal(got[-1], seg[-1])


def test_smooth_bspline_near_obstacles_validators_decide():
    """Planned paths hug the obstacles: smoothing them, the validators reject some moves
    (the result differs from the free-space iteration), and every state the restatement
    keeps is valid, with valid motions between consecutive states."""
    cfg = config.load(CONFIG)
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    g, o, start, goal = synth.c1_world()
    w = O.world_build(geom, g, o, rg, ro)
    lo = np.array(cfg["world_properties"]["lower_bound"], float)
    hi = np.array(cfg["world_properties"]["upper_bound"], float)
    differs = 0
    for call in range(3):
        path = TP.plan_path(w, rg, ro, lo, hi, start, goal, call, 4096)
        assert path is not None
        got = np.array(TP.smooth_bspline(path, w, rg, ro, False))
        geo = _free_space_smoothing(path)
        differs += int(got.shape != geo.shape or not np.array_equal(got, geo))
        assert np.array_equal(got[0], path[0]) and np.array_equal(got[-1], path[-1])
        assert O.check_states(w, rg, ro, got, False).all()
        assert O.check_motions(w, rg, ro, got[:-1], got[1:], False, 0).all()
    assert differs >= 1

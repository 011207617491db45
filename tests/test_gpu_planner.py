"""GPU tests of the batch planner building blocks and the C++ API shell.

* epp_sample_uniform / epp_knn / epp_knn_edges vs CPU restatements (bit-exact).
* PathPlanner (include/epp/PathPlanner.h, the drop-in of src/PathPlanner.cpp): paths are
  checked against the oracle's StateValidator/MotionValidator semantics; includeGates2's
  "custom" pruning is replayed on the oracle's ray answers (src/PathPlanner.cpp:175-265);
  checkTrajectoryValidity vs the oracle's minDistance check (:267-280).
* OnlineTrajGenerator through the online_traj_planner module (src/pybind.cpp:10-27,
  src/OnlineTrajGenerator.cpp): checkpoints, offline trajectory, sampling, gate updates.

The batch planner is a re-design (OMPL's RRT*/FMT* are third-party): its paths are not
the reference's paths, so the bar is validity under the oracle, not equality.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from eppamd import capi, config, synth

from conftest import CONFIG, ROOT

pytestmark = pytest.mark.gpu


def _write_config(tmp_path, **over):
    c = json.load(open(CONFIG))
    for k, v in over.items():
        sect, key = k.split("__")
        c[sect][key] = v
    p = tmp_path / "config.json"
    p.write_text(json.dumps(c))
    return str(p), c


def _ot():
    import online_traj_planner
    return online_traj_planner


# ---------------------------------------------------------------------------- device blocks
@pytest.mark.parametrize("start", [0, 1, 12345])
def test_sample_uniform_bit_exact(start):
    lo, hi = np.array([-6.0, -6.0, 0.0]), np.array([6.0, 6.0, 2.0])
    n = 5000
    got = capi.sample_uniform(0xC0FFEE, lo, hi, n, start)
    ref = synth.sample_states(0xC0FFEE, lo, hi, n, start)
    assert np.array_equal(got, ref)
    if start == 0:
        assert np.array_equal(got, O.sample_states(0xC0FFEE, lo, hi, n))


def _knn_ref(nodes, k, max_dist=0.0):
    n = len(nodes)
    out = np.full((n, k), -1, np.int32)
    r2 = max_dist * max_dist if max_dist > 0 else 1e300
    for i in range(n):
        d = nodes - nodes[i]
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        cand = np.nonzero((d2 < r2) & (np.arange(n) != i))[0]
        order = cand[np.lexsort((cand, d2[cand]))][:k]  # distance, then lower index
        out[i, :len(order)] = order
    return out


@pytest.mark.parametrize("method", ["brute", "grid"])
@pytest.mark.parametrize("k", [4, 8, 16, 32])
def test_knn_vs_bruteforce(k, method):
    nodes = synth.sample_states(7 + k, [-2, -2, 0], [2, 2, 2], 700)
    nodes[10] = nodes[3]              # duplicate: tie broken by index
    nodes[500:520] = nodes[0] + 0.01  # a cluster of identical distances
    got = capi.knn(nodes, k, method=method)
    assert np.array_equal(got, _knn_ref(nodes, k))


@pytest.mark.parametrize("tile", ["1", "2", "0"])
@pytest.mark.parametrize("k", [4, 8, 16, 32])
def test_knn_grid_large(k, tile, monkeypatch):
    """Grid k-NN (used above 2048 nodes) vs the all-pairs kernel and numpy: clustered,
    duplicated and lattice (many exact ties) nodes; with the tiled LDS kernel (k 4/8/16)
    and with the per-query walk."""
    monkeypatch.setenv("EPP_KNN_TILE", tile)
    rs = np.random.RandomState(k)
    nodes = synth.sample_states(100 + k, [-6, -6, 0], [6, 6, 2], 4000)
    nodes[:300] = rs.normal(0, 0.05, (300, 3)) + [1, 1, 1]          # a dense cluster
    nodes[300:400] = nodes[400:500]                                  # duplicates
    g = np.stack(np.meshgrid(np.arange(8), np.arange(8), np.arange(4)), -1).reshape(-1, 3) * 0.25
    nodes[500:756] = g                                               # lattice: exact ties
    got = capi.knn(nodes, k, method="grid")
    assert np.array_equal(got, capi.knn(nodes, k, method="brute"))
    assert np.array_equal(got, _knn_ref(nodes, k))
    assert np.array_equal(capi.knn(nodes, k), got)                   # auto -> grid
    assert np.array_equal(capi.knn(nodes, k, method="ws"), got)      # caller workspace
    assert np.array_equal(capi.knn(nodes, k, method="grid_ws"), got)
    # the caller-box variants: the grid over a given box that holds every node (tight,
    # wider, and lopsided)
    lo, hi = nodes.min(0), nodes.max(0)
    for box in ((lo, hi), (lo - 1.0, hi + 2.0), (lo - [0.0, 3.0, 0.0], hi + [0.5, 0.0, 4.0])):
        assert np.array_equal(capi.knn(nodes, k, method="grid_ws", box=box), got)
        assert np.array_equal(capi.knn(nodes, k, method="ws", box=box), got)


@pytest.mark.parametrize("tile", ["1", "2", "0"])
@pytest.mark.parametrize("k", [8, 16])
def test_knn_tile_crowded_halo(k, tile, monkeypatch):
    """A cluster far denser than the grid's cell size: the tiles around it overflow their
    LDS capacity and walk from global memory; the answer stays exact."""
    monkeypatch.setenv("EPP_KNN_TILE", tile)
    rs = np.random.RandomState(3)
    nodes = synth.sample_states(200 + k, [-6, -6, 0], [6, 6, 2], 6000)
    nodes[:3000] = rs.normal(0, 0.02, (3000, 3)) + [0.5, -0.5, 1]
    got = capi.knn(nodes, k, method="grid")
    assert np.array_equal(got, capi.knn(nodes, k, method="brute"))


@pytest.mark.parametrize("tile", ["1", "2"])
def test_knn_tile_spilled_block(tile, monkeypatch):
    """One 4^3-cell block holds 129..160 nodes: k_knn_tile keeps two lanes per query for its
    first 128 and sends the rest to the retry list (k_knn_wave has no such limit); the
    table equals the all-pairs one.  The grid is replicated here (knn_grid_shape: ~1.5
    nodes per cell over the nodes' bounding box) to place the extra nodes in one block."""
    monkeypatch.setenv("EPP_KNN_TILE", tile)
    rs = np.random.RandomState(11)
    n0 = 20000
    nodes = rs.uniform(0.0, 8.0, (n0, 3))
    nodes[0], nodes[1] = [0.0, 0.0, 0.0], [8.0, 8.0, 8.0]  # the bounding box
    h = np.cbrt(1.5 * 512.0 / (n0 + 64))
    lo, hi = 4 * h, 8 * h  # block (1, 1, 1) of 4 cells per axis
    inside = lambda p: np.all((p >= lo) & (p < hi), axis=1)
    extra = 140 - int(inside(nodes).sum())
    assert 0 < extra <= 64
    pad = rs.uniform(lo + 1e-3, hi - 1e-3, (64, 3))
    pad[extra:] = rs.uniform(0.0, 8.0, (64 - extra, 3))  # (the rest anywhere outside)
    pad[extra:][inside(pad[extra:])] += 8.0 * h
    pad = np.minimum(pad, 8.0)
    nodes = np.concatenate([nodes, pad])
    assert 128 < int(inside(nodes).sum()) <= 160
    got = capi.knn(nodes, 16, method="grid")
    assert np.array_equal(got, capi.knn(nodes, 16, method="brute"))


def test_knn_grid_many_scan_blocks():
    """300k nodes: the cell-count scan spans ~70 look-back blocks (more than one 64-block
    window); the grid table equals the all-pairs one."""
    nodes = synth.sample_states(321, [-6, -6, 0], [6, 6, 2], 300_000)
    got = capi.knn(nodes, 8, method="grid_ws")
    assert np.array_equal(got, capi.knn(nodes, 8, method="brute"))


def test_knn_grid_back_to_back_streams():
    """Cached-workspace reuse is ordered on the GPU: grid k-NN launched on two streams and
    repeatedly without host syncs in between gives the synchronous answer every time."""
    import ctypes as C
    L = capi.lib()
    nodes = synth.sample_states(77, [-6, -6, 0], [6, 6, 2], 60000)
    ref = capi.knn(nodes, 16, method="grid")
    d_n = capi.DeviceBuffer.from_array(nodes)
    outs = [capi.DeviceBuffer(4 * 16 * len(nodes)) for _ in range(4)]
    sts = []
    for _ in range(2):
        s = C.c_void_p()
        capi.check(L.epp_stream_create(C.byref(s)))
        sts.append(s.value)
    for r, o in enumerate(outs):
        capi.check(L.epp_knn_grid(d_n.ptr, len(nodes), 16, 0.0, o.ptr, sts[r % 2]))
    for s in sts:
        capi.check(L.epp_stream_sync(s))
        capi.check(L.epp_stream_destroy(s))
    for o in outs:
        assert np.array_equal(o.download(np.int32, 16 * len(nodes)).reshape(-1, 16), ref)


def test_knn_grid_flat_and_radius():
    nodes = synth.sample_states(5, [-3, -3, 0.7], [3, 3, 0.7], 3000)  # all z equal: flat grid
    assert np.array_equal(capi.knn(nodes, 16, method="grid"), _knn_ref(nodes, 16))
    nodes3 = synth.sample_states(6, [-3, -3, 0], [3, 3, 2], 3000)
    assert np.array_equal(capi.knn(nodes3, 8, 0.35, method="grid"), _knn_ref(nodes3, 8, 0.35))
    one = np.array([[0.5, 0.5, 0.5]])
    assert (capi.knn(one, 4, method="grid") == -1).all()


def test_knn_radius_and_small_n():
    nodes = synth.sample_states(3, [-1, -1, 0], [1, 1, 1], 300)
    assert np.array_equal(capi.knn(nodes, 16, 0.3), _knn_ref(nodes, 16, 0.3))
    few = nodes[:5]
    got = capi.knn(few, 8)
    assert np.array_equal(got, _knn_ref(few, 8))
    assert (got[:, 4:] == -1).all()
    with pytest.raises(capi.EppError):
        capi.knn(nodes, 5)


def test_knn_edges():
    nodes = synth.sample_states(11, [-1, -1, 0], [1, 1, 1], 40)
    nbr = capi.knn(nodes[:6], 8)          # ragged: -1 entries become degenerate edges
    s1, s2 = capi.knn_edges(nodes[:6], nbr)
    i = np.repeat(np.arange(6), 8)
    j = nbr.reshape(-1)
    assert np.array_equal(s1, nodes[i])
    assert np.array_equal(s2, nodes[np.where(j < 0, i, j)])


# ---------------------------------------------------------------------------- PathPlanner
@pytest.fixture(scope="module")
def c1(cfg, geom):
    g, o, start, goal = synth.c1_world()
    rg, ro = config.inflate_radii(cfg)
    w = O.world_build(geom, g, o, rg, ro)
    return g, o, start, goal, w, rg, ro


def _path_valid(path, w, rg, ro, can_pass):
    assert O.check_states(w, rg, ro, path, can_pass).all()
    assert O.check_motions(w, rg, ro, path[:-1], path[1:], can_pass, 0).all()


@pytest.mark.parametrize("planner", ["fmt", "rrt"])
def test_plan_path_valid(tmp_path, c1, planner):
    g, o, start, goal, w, rg, ro = c1
    path_cfg, _ = _write_config(tmp_path, path_planner_properties__planner=planner)
    pp = _ot().PathPlanner(g, o, path_cfg)
    path = pp.plan_path(start, goal, 2.0)
    assert path is not None and len(path) >= 2
    assert np.array_equal(path[0], start) and np.array_equal(path[-1], goal)
    _path_valid(path, w, rg, ro, False)
    st = pp.last_stats()
    assert st["states_sampled"] >= 4096 and st["edges_checked"] > 0


def test_plan_path_seeded_is_deterministic(c1):
    g, o, start, goal, *_ = c1
    a = _ot().PathPlanner(g, o, CONFIG)
    b = _ot().PathPlanner(g, o, CONFIG)
    pa, pb = a.plan_path(start, goal, 2.0), b.plan_path(start, goal, 2.0)
    assert np.array_equal(pa, pb)


def test_plan_paths_concurrent_matches_sequential(c1):
    """planPaths (one host thread + stream per problem) gives problem i exactly what the
    i-th of consecutive planPath calls gives, failures included, whatever the timing."""
    g, o, start, goal, w, rg, ro = c1
    blocked = np.array([1.0, 0.5, 0.5])  # inside an obstacle
    problems = [(start, goal), (goal, start), (start, blocked), (start, (start + goal) / 2), (goal, start)]
    a = _ot().PathPlanner(g, o, CONFIG)
    seq = [a.plan_path(s, t, 0.5) for s, t in problems]
    for rep in range(2):
        b = _ot().PathPlanner(g, o, CONFIG)
        con = b.plan_paths(problems, 0.5)
        assert len(con) == len(problems)
        for (ok, path), ref in zip(con, seq):
            assert ok == (ref is not None)
            if ok:
                assert np.array_equal(path, ref)
                _path_valid(path, w, rg, ro, False)


def test_plan_path_blocked_goal(c1):
    g, o, start, _, *_ = c1
    pp = _ot().PathPlanner(g, o, CONFIG)
    assert pp.plan_path(start, np.array([1.0, 0.5, 0.5]), 0.2) is None  # inside an obstacle


def test_unknown_planner(tmp_path, c1):
    g, o, start, goal, *_ = c1
    path_cfg, _ = _write_config(tmp_path, path_planner_properties__planner="prm")
    pp = _ot().PathPlanner(g, o, path_cfg)
    with pytest.raises(RuntimeError, match="Unknown planner"):
        pp.plan_path(start, goal, 1.0)


def _prune_ref(seg, w, rg, ro):
    """pruneWaypoints (src/PathPlanner.cpp:232-265) on the oracle's checkRayValid(.., true)."""
    if len(seg) < 3:
        return list(seg)
    out = [seg[0]]
    ref = 0
    for cur in range(2, len(seg)):
        ok = O.check_motions(w, rg, ro, seg[ref][None], seg[cur][None], True, 0)[0]
        if not ok:
            out.append(seg[cur - 1])
            ref = cur - 1
    out.append(seg[-1])
    return out


def _include_gates2_ref(segs, w, rg, ro, method):
    segs = [list(map(np.asarray, s)) for s in segs]
    centers = [(segs[i][-1] + segs[i + 1][0]) / 2 for i in range(len(segs) - 1)]
    for i, c in enumerate(centers):
        segs[i].append(c)
        segs[i + 1].insert(0, c)
    flat = []
    for s in segs:
        pr = s if method == "none" else _prune_ref(s, w, rg, ro)
        for p in pr:
            if flat:
                d = flat[-1] - p
                if np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) < 0.05:
                    continue
            flat.append(p)
    return np.array(flat)


@pytest.mark.parametrize("method", ["custom", "none", "ompl"])
def test_include_gates2_matches_restatement(tmp_path, c1, method):
    """includeGates2 with each pruning method against the restatement: "custom" and
    "none" above, "ompl" (OMPL's smoothBSpline, src/PathPlanner.cpp:282-313) against
    oracle/track_planner.py smooth_bspline -- the segments' states bit for bit."""
    import track_planner as TP
    g, o, _, _, w, rg, ro = c1
    path_cfg, _ = _write_config(tmp_path, path_planner_properties__path_simplification=method)
    pp = _ot().PathPlanner(g, o, path_cfg)
    rs = np.random.RandomState(5)
    segs = []
    for s in range(3):
        n = 3 + 4 * s
        segs.append(np.cumsum(rs.uniform(-0.3, 0.3, (n, 3)), 0) + [0, 0, 1.0])
    segs[1][0] = segs[0][-1] + 0.01  # a gate centre within the 0.05 de-duplication radius
    got = pp.include_gates2(segs)
    if method == "ompl":
        ref = TP.include_gates2(segs, w, rg, ro, "ompl", False)
        assert len(got) > sum(len(x) for x in segs)  # subdivided
    else:
        ref = _include_gates2_ref(segs, w, rg, ro, method)
    assert np.array_equal(got, ref)


def test_precompute_traj_ompl_simplification_equals_cpu(track, geom, tmp_path):
    """A whole track with path_simplification "ompl": the 9 plans, smoothBSpline on every
    segment (batched steps on the GPU), the min-snap fit -- equal to the CPU restatement
    (waypoints bit for bit, trajectory within 1e-6, time column exact)."""
    import track_planner as TP
    _, c, gates, obstacles, start, goal = track
    c = json.loads(json.dumps(c))
    c["path_planner_properties"]["path_simplification"] = "ompl"
    p = tmp_path / "config_ompl.json"
    p.write_text(json.dumps(c))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, str(p))
    otg.pre_compute_traj(0.0)
    rg, ro = config.inflate_radii(c)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    lo, hi = np.array(c["world_properties"]["lower_bound"], float), np.array(c["world_properties"]["upper_bound"], float)
    tg, pp = c["trajectory_generator_properties"], c["path_planner_properties"]
    wp, rows = TP.plan_track(w, rg, ro, lo, hi, otg.get_checkpoints(), pp["samples_fmt"], tg["max_velocity"],
                             tg["max_acceleration"], tg["sampling_interval"], threads=8, method="ompl",
                             can_pass=bool(pp["can_pass_gate"]))
    assert np.array_equal(otg.get_waypoints(), wp)
    traj = otg.get_planned_traj()
    assert traj.shape == rows.shape and np.array_equal(traj[:, 9], rows[:, 9])
    assert np.abs(traj[:, :9] - rows[:, :9]).max() < 1e-6


FILLING_CONFIG = os.path.join(ROOT, "configs", "config_filling.json")


@pytest.mark.parametrize("n", [700, 3000])
def test_check_rays_both(n):
    """World::checkRaysBoth (the shortcut's batch in planPathsIncludeGates2): bit 0 = the
    oracle's checkRayValid(.., false), bit 1 = (.., true), in a world with filling OBBs
    (configs/config_filling.json) where the two differ -- rays through the gate openings
    and random rays; 700 rays take the small path (one launch for both answers), 3,000 the
    two launches past it."""
    cfg = config.load(FILLING_CONFIG)
    fgeom = config.geometry(cfg)
    g, o, _, _ = synth.c1_world()
    rg, ro = config.inflate_radii(cfg)
    w = O.world_build(fgeom, g, o, rg, ro)
    pp = _ot().PathPlanner(g, o, FILLING_CONFIG)
    rs = np.random.RandomState(n)
    m = n // 2  # through the openings: either side of the portal, along its normal
    loc = rs.uniform([-0.3, -0.6, -0.3], [0.3, -0.3, 0.3], size=(m, 3))
    loc2 = loc + np.c_[rs.uniform(-0.1, 0.1, m), rs.uniform(0.6, 1.2, m), rs.uniform(-0.1, 0.1, m)]
    gt = g[0]
    h = fgeom.gate_height[int(gt[6])]
    c, sn = np.cos(gt[5]), np.sin(gt[5])

    def world(l):
        return np.stack([gt[0] + c * l[:, 0] - sn * l[:, 1], gt[1] + sn * l[:, 0] + c * l[:, 1], h + l[:, 2]], 1)

    s1 = np.vstack([world(loc), synth.sample_states(5, [-2, -2, 0], [2, 2, 2], n - m)])
    s2 = np.vstack([world(loc2), s1[m:] + rs.uniform(-0.8, 0.8, (n - m, 3))])
    got = pp.check_rays_both(s1, s2)
    e0 = O.check_motions(w, rg, ro, s1, s2, False, 0)
    e1 = O.check_motions(w, rg, ro, s1, s2, True, 0)
    assert (e1 > e0).sum() >= 20 and e0.min() == 0 and e1.max() == 1
    assert np.array_equal(got, e0.astype(np.uint8) | (e1.astype(np.uint8) << 1))


@pytest.mark.parametrize("filling", [False, True])
@pytest.mark.parametrize("can_pass", [False, True])
def test_plan_paths_include_gates2_equals_two_calls(track, tmp_path, can_pass, filling):
    """planPathsIncludeGates2 (preComputeTraj's call: the pruning's rays in the shortcut's
    batch) gives what planPaths followed by includeGates2 gives, on two planners with the
    same call numbers: the same segments and the same pruned waypoints, for can_pass_gate
    false and true (the shortcut reading the other answer bit), in the track world and in
    the same world with filling OBBs (configs/config_filling.json), where the two answers
    differ at the portals."""
    _, c, gates, obstacles, start, goal = track
    c = json.loads(json.dumps(c))
    if filling:
        f = json.load(open(FILLING_CONFIG))
        f["world_properties"]["lower_bound"] = c["world_properties"]["lower_bound"]
        f["world_properties"]["upper_bound"] = c["world_properties"]["upper_bound"]
        c = f
    c["path_planner_properties"]["can_pass_gate"] = can_pass
    p = tmp_path / "config.json"
    p.write_text(json.dumps(c))
    cps = synth.gate_checkpoints(gates, np.array([1.0, 0.525]), 0.55)
    problems = [(cps[i], cps[i + 1]) for i in range(0, len(cps) - 1, 2)]
    a, b = _ot().PathPlanner(gates, obstacles, str(p)), _ot().PathPlanner(gates, obstacles, str(p))
    for _ in range(2):  # (the second call: the next call numbers)
        segs = a.plan_paths(problems, 2.0)
        assert all(ok for ok, _ in segs)
        exp = a.include_gates2([x for _, x in segs])
        segs2, got = b.plan_paths_include_gates2(problems, 2.0)
        assert all(np.array_equal(x, y) and o1 == o2 for (o1, x), (o2, y) in zip(segs, segs2))
        assert got is not None and np.array_equal(got, exp)


def test_plan_paths_include_gates2_edges(c1):
    """planPathsIncludeGates2 at the edges: one problem (no gate centres), a chain with a
    problem that fails (pruned is None, the segments as plan_paths gives them, failures
    included), and a chain whose second problem starts where the first ends (a gate
    centre equal to both ends) -- each against plan_paths + include_gates2 on a planner
    with the same call numbers."""
    g, o, start, goal, *_ = c1
    blocked = np.array([1.0, 0.5, 0.5])  # inside an obstacle
    mid = (start + goal) / 2
    for problems in ([(start, goal)], [(start, mid), (mid, blocked), (mid, goal)], [(start, mid), (mid, goal)]):
        a, b = _ot().PathPlanner(g, o, CONFIG), _ot().PathPlanner(g, o, CONFIG)
        segs = a.plan_paths(problems, 0.5)
        segs2, got = b.plan_paths_include_gates2(problems, 0.5)
        assert all(o1 == o2 and np.array_equal(x, y) for (o1, x), (o2, y) in zip(segs, segs2))
        if all(ok for ok, _ in segs):
            assert got is not None and np.array_equal(got, a.include_gates2([x for _, x in segs]))
        else:
            assert got is None


def test_include_gates2_unknown_method(tmp_path, c1):
    g, o, *_ = c1
    path_cfg, _ = _write_config(tmp_path, path_planner_properties__path_simplification="bogus")
    pp = _ot().PathPlanner(g, o, path_cfg)
    with pytest.raises(RuntimeError, match="Unknown pruning method"):
        pp.include_gates2([np.zeros((2, 3)), np.ones((2, 3))])


def test_check_trajectory_validity(c1):
    g, o, start, goal, w, rg, ro = c1
    pp = _ot().PathPlanner(g, o, CONFIG)
    pts = synth.sample_states(77, [-2, -2, 0], [2, 2, 2], 400)
    ok = O.check_states_mindist(w, pts, 0.1)
    traj = np.zeros((len(pts), 10))
    traj[:, 0], traj[:, 3], traj[:, 6] = pts[:, 0], pts[:, 1], pts[:, 2]
    good = traj[ok == 1]
    assert pp.check_trajectory_validity(good, 0.1)
    assert pp.check_trajectory_validity(traj, 0.1) == bool(ok.all())
    for i in np.nonzero(ok == 0)[0][:5]:
        assert not pp.check_trajectory_validity(traj[i:i + 1], 0.1)
    assert pp.check_trajectory_validity(np.zeros((0, 10)), 0.1)


# ---------------------------------------------------------------------------- OnlineTrajGenerator
@pytest.fixture(scope="module")
def track(tmp_path_factory, cfg):
    tmp = tmp_path_factory.mktemp("track")
    c = json.load(open(CONFIG))
    c["world_properties"]["lower_bound"] = [-6, -6, 0]
    c["world_properties"]["upper_bound"] = [6, 6, 2]
    p = tmp / "config.json"
    p.write_text(json.dumps(c))
    gates, obstacles = synth.track_world(42)
    # start 0.55 m before gate 0, goal 0.55 m after gate 7 (obstacles keep >= 0.95 m from
    # every gate centre, so both are free)
    cps = synth.gate_checkpoints(gates, np.array([1.0, 0.525]), 0.55)
    start, goal = cps[0], cps[-1]
    return str(p), c, gates, obstacles, start, goal


def _lateral(gate, d):
    """Gate pose shifted by d metres inside its own plane (perpendicular to the normal)."""
    pose = np.array(gate[:6], float)
    pose[0] += d * np.cos(gate[5])
    pose[1] += d * np.sin(gate[5])
    return list(pose)


def test_online_checkpoints(track, geom):
    path, c, gates, obstacles, start, goal = track
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, path)
    cps = otg.get_checkpoints()
    ref = synth.gate_checkpoints(gates, geom.gate_height, c["path_planner_properties"]["checkpoint_gate_offset"])
    assert np.array_equal(cps[0], start) and np.array_equal(cps[-1], goal)
    np.testing.assert_allclose(cps[1:-1], ref, rtol=0, atol=1e-15)


def test_online_no_traj_errors(track):
    path, c, gates, obstacles, start, goal = track
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, path)
    for f in (otg.get_planned_traj, otg.get_traj_end_time):
        with pytest.raises(RuntimeError, match="No trajectory data available."):
            f()
    with pytest.raises(RuntimeError, match="No trajectory data available."):
        otg.sample_traj(0.0)


@pytest.fixture(scope="module")
def planned(track):
    path, c, gates, obstacles, start, goal = track
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, path)
    otg.pre_compute_traj(1.5)
    return otg


def test_online_precompute(track, planned, geom):
    path, c, gates, obstacles, start, goal = track
    traj = planned.get_planned_traj()
    assert traj.shape[1] == 10 and len(traj) > 100
    dt = c["trajectory_generator_properties"]["sampling_interval"]
    assert traj[0, 9] == 1.5
    assert np.allclose(np.diff(traj[:, 9]), dt, atol=1e-9)
    np.testing.assert_allclose(traj[0, [0, 3, 6]], start, atol=1e-12)
    np.testing.assert_allclose(traj[0, [1, 4, 7, 2, 5, 8]], 0, atol=1e-9)
    assert np.linalg.norm(traj[-1, [0, 3, 6]] - goal) < 0.1
    assert planned.get_traj_end_time() == traj[-1, 9]
    # the trajectory passes every gate centre (includeGates2 inserts them as waypoints)
    pos = traj[:, [0, 3, 6]]
    for gt in gates:
        centre = gt[:3] + [0, 0, geom.gate_height[int(gt[6])]]
        assert np.min(np.linalg.norm(pos - centre, axis=1)) < 0.1
    # continuity of position and velocity between rows
    v = traj[:, [1, 4, 7]]
    assert np.abs(np.diff(pos, axis=0)).max() < 0.5
    assert np.abs(np.diff(v, axis=0)).max() < 0.6


def test_online_sample_traj(planned):
    traj = planned.get_planned_traj()
    for t in (0.0, 1.5, 1.54, 1.56, 7.77, 1e6):
        row = planned.sample_traj(t)
        i = int(np.argmin(np.abs(traj[:, 9] - t)))
        assert np.array_equal(row, traj[i])


def test_online_update_gate_pos(track, geom):
    path, c, gates, obstacles, start, goal = track
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, path)
    otg.pre_compute_traj(0.0)
    before = otg.get_planned_traj()
    gid = 2
    # 0.3 m sideways: the old path still crosses the gate plane within the 0.425 m
    # opening test but runs 0.1 m from a bar, so the lookahead check fails -> replan
    pose = _lateral(gates[gid], 0.3)
    # early outs (src/OnlineTrajGenerator.cpp:125-140)
    assert otg.update_gate_pos(gid, pose, start, False, 1.0) is False
    inside = obstacles[0, :3] + [0, 0, 0.5]  # drone inside an obstacle
    assert otg.update_gate_pos(gid, pose, inside, True, 1.0) is False
    t_fly = 2.0
    i = int(np.argmin(np.abs(before[:, 9] - t_fly)))
    drone = before[i, [0, 3, 6]]
    assert otg.update_gate_pos(gid, pose, drone, True, t_fly) is True
    after = otg.get_planned_traj()
    # the prefix up to the advanced time is kept, the rest is replanned
    adv = t_fly + c["path_planner_properties"]["time_limit_online"] + 0.01
    k = int(np.argmax(before[:, 9] > adv))
    assert np.array_equal(after[:k], before[:k])
    assert not np.array_equal(after, before)
    moved = np.array(pose[:3]) + [0, 0, geom.gate_height[int(gates[gid, 6])]]
    assert np.min(np.linalg.norm(after[:, [0, 3, 6]] - moved, axis=1)) < 0.1
    # already observed gate: no second update
    assert otg.update_gate_pos(gid, pose, drone, True, t_fly) is False


def test_online_async_update(track):
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    c2["path_planner_properties"]["recalculate_online"] = True
    p2 = os.path.join(os.path.dirname(path), "config_async.json")
    open(p2, "w").write(json.dumps(c2))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, p2)
    otg.pre_compute_traj(0.0)
    before = otg.get_planned_traj()
    pose = _lateral(gates[4], 0.3)
    i = int(np.argmin(np.abs(before[:, 9] - 5.0)))
    assert otg.update_gate_pos(4, pose, before[i, [0, 3, 6]], True, 5.0) is True
    otg.wait_for_update()
    assert not np.array_equal(otg.get_planned_traj(), before)


def test_online_optimal_type(tmp_path, track):
    """type "optimal" (src/OnlineTrajGenerator.cpp:108-114, :385-406): 11 columns, the
    planned rows equal the oracle's time-optimal parametrisation of the same waypoints,
    and a gate update re-simulates the lead-in and keeps the prefix."""
    import timeopt  # oracle/ (test infrastructure)
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    tg = c2["trajectory_generator_properties"]
    tg["type"] = "optimal"
    p2 = tmp_path / "c_opt.json"
    p2.write_text(json.dumps(c2))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, str(p2))
    otg.pre_compute_traj(1.5)
    traj = otg.get_planned_traj()
    assert traj.shape[1] == 11 and len(traj) > 50
    exp = np.array(timeopt.calculate_trajectory(np.asarray(otg.get_waypoints()), [], tg["max_velocity"],
                                                tg["max_acceleration"], 1.5, tg["sampling_interval"],
                                                tg["max_traj_divergence"]))
    assert np.array_equal(traj, exp)
    assert len(otg.sample_traj(2.0)) == 11 and otg.get_traj_end_time() == traj[-1, 10]
    np.testing.assert_allclose(traj[0, [0, 3, 6]], start, atol=1e-12)
    before = traj
    gid = 2
    t_fly = 2.0
    i = int(np.argmin(np.abs(before[:, 10] - t_fly)))
    replanned = otg.update_gate_pos(gid, _lateral(gates[gid], 0.3), before[i, [0, 3, 6]], True, t_fly)
    after = otg.get_planned_traj()
    assert after.shape[1] == 11
    adv = t_fly + c["path_planner_properties"]["time_limit_online"] + 0.01
    k = int(np.argmax(before[:, 10] > adv))
    assert np.array_equal(after[:k], before[:k])
    assert replanned == (not np.array_equal(after, before))


def test_online_spline_type_and_path_writer(tmp_path, track, monkeypatch):
    """type "spline" (src/OnlineTrajGenerator.cpp:102-107: TrajInterpolation through the
    waypoints, sampled up to max_time) and the PathWriter dumps the reference writes to
    ./path_segments (src/PathWriter.cpp, src/OnlineTrajGenerator.cpp:20-47, :90)."""
    import spline_np  # oracle/ (test infrastructure)
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    tg = c2["trajectory_generator_properties"]
    tg["type"] = "spline"
    p2 = tmp_path / "c_spline.json"
    p2.write_text(json.dumps(c2))
    monkeypatch.chdir(tmp_path)
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, str(p2))
    otg.pre_compute_traj(1.5)
    traj = otg.get_planned_traj()
    wp = np.asarray(otg.get_waypoints())
    exp = spline_np.interpolate_traj(wp, tg["max_time"], 1.5, tg["sampling_interval"])
    assert traj.shape == exp.shape and traj.shape[1] == 10
    np.testing.assert_allclose(traj, exp, rtol=0, atol=1e-9)
    out = tmp_path / "path_segments"
    assert sorted(os.listdir(out)) == ["checkpoints.txt", "gates.txt", "obstacles.txt", "path_0.txt"]
    assert len((out / "gates.txt").read_text().splitlines()) == len(gates)
    assert len((out / "obstacles.txt").read_text().splitlines()) == len(obstacles)
    pts = np.loadtxt(out / "path_0.txt")
    np.testing.assert_allclose(pts, wp, rtol=1e-5, atol=1e-5)  # default stream precision (6 digits)
    assert (out / "gates.txt").read_text().splitlines()[0].startswith("id: 0 info: ")


def test_trajectory_type_not_supported(tmp_path, track):
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    c2["trajectory_generator_properties"]["type"] = "linear"
    p2 = tmp_path / "c.json"
    p2.write_text(json.dumps(c2))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, str(p2))
    with pytest.raises(RuntimeError, match="Trajectory type not supported"):
        otg.pre_compute_traj(0.0)


def test_vector_and_matrix_helpers():
    ot = _ot()
    v = ot.Vector3d(np.array([1.0, 2.0, 3.0]))
    assert np.array_equal(np.asarray(v), [1, 2, 3])
    m = ot.MatrixXd(np.arange(6.0).reshape(2, 3))
    assert m.shape == (2, 3) and np.array_equal(np.asarray(m), np.arange(6.0).reshape(2, 3))


@pytest.mark.parametrize("n", [1, 15, 4095, 4096, 65536, 100_003, 1_000_003])
def test_compact_states_ordered(n):
    """Ordered compaction (the planner's node list): same rows, same order as numpy.  The
    single-pass kernel's look-back crosses several 64-block windows at 1M states."""
    xyz = synth.sample_states(12, [-6, -6, 0], [6, 6, 2], n)
    valid = (np.random.RandomState(n).rand(n) < 0.9).astype(np.uint8)
    assert np.array_equal(capi.compact_states(xyz, valid), xyz[valid.astype(bool)])
    assert np.array_equal(capi.compact_states(xyz, valid, ws=True), xyz[valid.astype(bool)])
    assert len(capi.compact_states(xyz, np.zeros(n, np.uint8))) == 0


def _scan_tag_now() -> int:
    """The launch tag of the last look-back scan, read back from a compaction's caller
    workspace (its word 0 = [tag:24 | inclusive:1 | value:39])."""
    n = 5000
    xyz = synth.sample_states(1, [0, 0, 0], [1, 1, 1], n)
    d_x, d_v = capi.DeviceBuffer.from_array(xyz), capi.DeviceBuffer.from_array(np.ones(n, np.uint8))
    d_o, d_c = capi.DeviceBuffer(24 * n), capi.DeviceBuffer(8)
    nb = int(capi.lib().epp_compact_workspace_size(n))
    d_w = capi.DeviceBuffer(nb)
    capi.check(capi.lib().epp_compact_states_ws(d_x.ptr, d_v.ptr, n, d_o.ptr, d_c.ptr, d_w.ptr, nb, None))
    capi.sync()
    return int(d_w.download(np.uint64, 1)[0]) >> 40


def _stale_word(tag: int, value: int = 5) -> int:
    """A status word that reads as an inclusive prefix published by launch `tag`."""
    return (tag << 40) | (1 << 39) | value


def _next_tag(t: int) -> int:
    t = (t + 1) & 0xFFFFFF
    return t if t else 1


@pytest.mark.parametrize("n", [5000, 300_000])
def test_scans_ignore_stale_workspace_words(n):
    """a caller workspace that holds words carrying the NEXT launch's tag (stale
    data of a moved carve, or a wrapped tag) must not be taken for published look-back
    status words: the k-NN cell scan and the ordered compaction stay exact."""
    nodes = synth.sample_states(900 + n, [-6, -6, 0], [6, 6, 2], n)
    ref = capi.knn(nodes, 16, method="grid_ws")
    t = _scan_tag_now()
    got = capi.knn(nodes, 16, method="grid_ws", ws_fill=_stale_word(_next_tag(t)))
    assert np.array_equal(got, ref)
    lo, hi = nodes.min(0), nodes.max(0)
    t = _scan_tag_now()
    got = capi.knn(nodes, 16, method="grid_ws", box=(lo, hi), ws_fill=_stale_word(_next_tag(t)))
    assert np.array_equal(got, ref)
    valid = (np.random.RandomState(n).rand(n) < 0.7).astype(np.uint8)
    t = _scan_tag_now()
    out = capi.compact_states(nodes, valid, ws=True, ws_fill=_stale_word(_next_tag(t), 123))
    assert np.array_equal(out, nodes[valid.astype(bool)])


def test_mask_edges():
    rs = np.random.RandomState(3)
    nbr = rs.randint(-1, 1000, (777, 16)).astype(np.int32)
    valid = (rs.rand(777, 16) < 0.7).astype(np.uint8)
    assert np.array_equal(capi.mask_edges(nbr, valid), np.where(valid.astype(bool), nbr, -1))
    for n in (777, 1, 64, 65537):  # ragged, single, one wave, several blocks
        nb = rs.randint(-1, 1000, (n, 16)).astype(np.int32)
        va = (rs.rand(n, 16) < 0.7).astype(np.uint8)
        want = np.where(va.astype(bool), nb, -1)
        got, cnt, into = capi.mask_edges_count(nb, va, 7)
        assert np.array_equal(got, want) and cnt == int((want >= 0).sum()) and into == int((want == 7).sum())


def test_online_update_while_replanning_throws(track):
    """An update arriving while the online recomputation (recalculate_online) still runs
    and needing a recomputation itself gets the reference's runtime_error
    (src/OnlineTrajGenerator.cpp:208-212); the running worker's world is not touched;
    wait_for_update() then completes the first one."""
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    c2["path_planner_properties"]["recalculate_online"] = True
    c2["path_planner_properties"]["samples_fmt"] = 1 << 20  # a replan of ~10 ms
    p2 = os.path.join(os.path.dirname(path), "config_async_busy.json")
    open(p2, "w").write(json.dumps(c2))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, p2)
    otg.pre_compute_traj(0.0)
    before = otg.get_planned_traj()
    i = int(np.argmin(np.abs(before[:, 9] - 5.0)))
    drone = before[i, [0, 3, 6]]
    assert otg.update_gate_pos(4, _lateral(gates[4], 0.3), drone, True, 5.0) is True
    with pytest.raises(RuntimeError, match="while previous update is still going on"):
        otg.update_gate_pos(5, _lateral(gates[5], 0.3), drone, True, 5.0)
    otg.wait_for_update()
    assert not np.array_equal(otg.get_planned_traj(), before)


def test_c1_plumbing_end_to_end(tmp_path, c1, geom):
    """BASELINE config 1 (single gate + 4 obstacles, bounds [-2,2]^2 x [0,2]) end to end:
    OnlineTrajGenerator plans start -> gate -> goal, its waypoints are valid under the
    oracle's validators, and its trajectory equals polynomial_trajectory's
    generate_trajectory of those waypoints and the oracle's within 1e-6 (time column
    exact)."""
    import polynomial_trajectory as pt
    g, o, start, goal, w, rg, ro = c1
    otg = _ot().OnlineTrajGenerator(start, goal, g, o, CONFIG)
    otg.pre_compute_traj(0.0)
    wp = otg.get_waypoints()
    traj = otg.get_planned_traj()
    centre = g[0, :3] + [0, 0, geom.gate_height[0]]
    assert min(np.linalg.norm(wp - centre, axis=1)) < 1e-12  # includeGates2 inserts the gate centre
    _path_valid(wp, w, rg, ro, False)
    rows = pt.generate_trajectory(wp, 1.0, 2.0, 0.1)
    assert np.array_equal(rows, traj)
    exp = O.generate_trajectory(wp, 1.0, 2.0, 0.1)
    assert rows.shape == exp.shape and np.array_equal(rows[:, 9], exp[:, 9])
    assert np.abs(rows[:, :9] - exp[:, :9]).max() < 1e-6


# ---- the planner against its CPU restatement (oracle/epp_oracle.cpp or_plan_once) ------
# Same counter-RNG samples, exact k-NN with the same tie rule, the same A* and shortcut:
# the GPU pipeline must give the SAME path, not just a valid one.
# EPP_PLAN_ELLIPSE: the row-restricted table download (default factor 1.25), a bound the
# paths exceed (1.0: the search falls back to the whole table) and the whole table only (0)
ELLIPSE = ["", "1.0", "0"]


@pytest.mark.parametrize("ellipse", ELLIPSE)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_plan_once_equals_cpu_restatement(c1, seed, ellipse, monkeypatch):
    if ellipse:
        monkeypatch.setenv("EPP_PLAN_ELLIPSE", ellipse)
    g, o, start, goal, w, rg, ro = c1
    pp = _ot().PathPlanner(g, o, CONFIG)
    lo, hi = synth.C1_BOUNDS
    for samples in (1000, 4096, 20_000):
        got = pp.plan_once(start, goal, samples, seed)
        exp, st = O.plan_once(w, rg, ro, lo, hi, start, goal, samples, seed, 16, False, 8)
        assert (got is None) == (exp is None)
        if got is not None:
            assert np.array_equal(got, exp), (samples, got, exp)
    blocked = np.array([1.0, 0.5, 0.5])
    assert pp.plan_once(start, blocked, 4096, seed) is None
    assert O.plan_once(w, rg, ro, lo, hi, start, blocked, 4096, seed, 16, False, 4)[0] is None


@pytest.mark.parametrize("world", ["empty", "1100_obbs"])
def test_plan_worlds_without_tile_tables(c1, geom, cfg, world):
    """Worlds the rows' fused motion check does not take (no OBBs: no tile tables; 1,104
    OBBs: records past the LDS budget) plan through the whole table with the default row
    restriction on, in planPath and the batched planPaths alike (these threw),
    and equal the CPU restatement."""
    g0, o0, start, goal, *_ = c1
    if world == "empty":
        g, o = np.zeros((0, 7)), np.zeros((0, 6))
    else:
        rng = np.random.default_rng(3)
        o = np.zeros((1100, 6))
        o[:, 0] = rng.uniform(20, 60, 1100)  # (far outside the sampling box: they count, never hit)
        o[:, 1] = rng.uniform(-20, 20, 1100)
        o[:4] = o0
        g = g0
    rg, ro = config.inflate_radii(cfg)
    w = O.world_build(geom, g, o, rg, ro)
    pp = _ot().PathPlanner(g, o, CONFIG)
    lo, hi = synth.C1_BOUNDS
    for seed in (1, 2):
        got = pp.plan_once(start, goal, 4096, seed)
        exp, _ = O.plan_once(w, rg, ro, lo, hi, start, goal, 4096, seed, 16, False, 8)
        assert got is not None and np.array_equal(got, exp), (world, seed)
    st = pp.last_stats()
    assert st["restricted_rows"] == 0 and st["fallbacks"] == 0
    res = pp.plan_paths([(start, goal), (goal, start)], 0.5)
    assert all(ok for ok, _ in res)
    for ok, path in res:
        _path_valid(path, w, rg, ro, False)


def test_plan_once_symmetrised_on_rows_equals_cpu(bench_track_config, geom):
    """Goals outside the sampling box (the C4 box, track world 100, 65,536 samples): no
    sample keeps the goal among its 16 neighbours, so the forward search fails and the
    symmetrised graph (the goal's own row, reversed) decides.  The planner runs that search
    on the downloaded rows (host_planner.cpp solve, `restricted_symmetrised`) instead of the
    whole table -- here after the whole table's masked k-NN showed no kept edge into the
    goal (the forward search popped above the bound: `symmetrised_after_census`); the path
    equals the CPU restatement's, whose stats say its symmetrised search ran."""
    path, c = bench_track_config
    gates, obstacles = synth.track_world(100)
    pp = _ot().PathPlanner(gates, obstacles, path)
    rg, ro = config.inflate_radii(c)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    lo, hi = np.array(c["world_properties"]["lower_bound"], float), np.array(c["world_properties"]["upper_bound"], float)
    cases = [((0, 5.0, 1.0), (0, 6.4, 1.0)), ((5.0, 0, 1.0), (6.4, 0.5, 1.0)), ((0, -5, 1.0), (0.5, -6.5, 1.0)),
             ((2, 2, 1.2), (2.5, 2.5, 2.5)), ((-5, -5, 1.0), (-6.4, -6.4, 1.0))]
    sym = ran = cen = 0
    for s, g in cases:
        s, g = np.array(s, float), np.array(g, float)
        for seed in (0, 1):
            s0 = pp.last_stats().get("restricted_symmetrised", 0)
            c0 = pp.last_stats().get("symmetrised_after_census", 0)
            got = pp.plan_once(s, g, 65536, seed)
            exp, st = O.plan_once(w, rg, ro, lo, hi, s, g, 65536, seed, 16, False, 16)
            assert exp is not None and got is not None and np.array_equal(got, exp), (s, g, seed)
            ran += int(st[4])
            sym += pp.last_stats()["restricted_symmetrised"] - s0
            cen += pp.last_stats()["symmetrised_after_census"] - c0
    st = pp.last_stats()
    assert ran == 10 and sym == ran and cen >= 1 and st["fallbacks"] == 0, (ran, sym, cen, st.get("fallback_why"), st.get("fallbacks"),
                                      st.get("restricted_rows"), st.get("rows_downloaded"))


@pytest.mark.parametrize("ellipse", ELLIPSE)
def test_plan_once_equals_cpu_restatement_track(track, geom, ellipse, monkeypatch):
    """Every gate-to-gate segment of the C2 track (65,536 samples, the C4 size) equal on
    GPU and CPU, with the row-restricted table download and without."""
    if ellipse:
        monkeypatch.setenv("EPP_PLAN_ELLIPSE", ellipse)
    path, c, gates, obstacles, start, goal = track
    pp = _ot().PathPlanner(gates, obstacles, path)
    rg, ro = config.inflate_radii(c)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    lo, hi = np.array(c["world_properties"]["lower_bound"], float), np.array(c["world_properties"]["upper_bound"], float)
    cps = synth.gate_checkpoints(gates, geom.gate_height, c["path_planner_properties"]["checkpoint_gate_offset"])
    cps = np.vstack([start, cps, goal])
    rows = []
    for s in range(0, len(cps) - 1, 2):
        r0 = pp.last_stats()["rows_downloaded"]  # (plan_once accumulates the stats)
        got = pp.plan_once(cps[s], cps[s + 1], 65536, 1000 + s)
        exp, st = O.plan_once(w, rg, ro, lo, hi, cps[s], cps[s + 1], 65536, 1000 + s, 16, False, 16)
        assert got is not None and np.array_equal(got, exp), s
        rows.append((pp.last_stats()["rows_downloaded"] - r0, st[1] + 2))
    if ellipse == "0":
        assert all(r == n for r, n in rows)
    elif ellipse == "":  # most segments' searches stay inside the ellipsoid
        assert sum(r < n for r, n in rows) >= len(rows) // 2, rows
    # one segment past 65,535 nodes: the k-NN table goes down as int32 instead of u16
    got = pp.plan_once(cps[1], cps[2], 80_000, 77)
    exp, st = O.plan_once(w, rg, ro, lo, hi, cps[1], cps[2], 80_000, 77, 16, False, 16)
    assert st[1] + 2 > 65535
    assert got is not None and np.array_equal(got, exp)


def test_precompute_traj_equals_cpu_track(track, geom):
    """OnlineTrajGenerator::preComputeTraj (9 concurrent GPU plans + includeGates2 +
    min-snap) equals the CPU restatement of the whole track (oracle/track_planner.py):
    identical waypoints, trajectory within 1e-6 with the time column exact."""
    import track_planner as TP
    path, c, gates, obstacles, start, goal = track
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, path)
    otg.pre_compute_traj(0.0)
    rg, ro = config.inflate_radii(c)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    lo, hi = np.array(c["world_properties"]["lower_bound"], float), np.array(c["world_properties"]["upper_bound"], float)
    tg, pp = c["trajectory_generator_properties"], c["path_planner_properties"]
    wp, rows = TP.plan_track(w, rg, ro, lo, hi, otg.get_checkpoints(), pp["samples_fmt"], tg["max_velocity"],
                             tg["max_acceleration"], tg["sampling_interval"], threads=8)
    assert np.array_equal(otg.get_waypoints(), wp)
    traj = otg.get_planned_traj()
    assert traj.shape == rows.shape and np.array_equal(traj[:, 9], rows[:, 9])
    assert np.abs(traj[:, :9] - rows[:, :9]).max() < 1e-6


@pytest.fixture(scope="module")
def bench_track_config(tmp_path_factory):
    """bench.py's C4 configuration (_track_config): the shipped config with the track
    bounds [-6,6]^2 x [0,2] and 65,536 samples per segment."""
    c = json.load(open(CONFIG))
    c["world_properties"]["lower_bound"] = [-6, -6, 0]
    c["world_properties"]["upper_bound"] = [6, 6, 2]
    c["path_planner_properties"]["samples_fmt"] = 65536
    p = tmp_path_factory.mktemp("c4") / "config.json"
    p.write_text(json.dumps(c))
    return str(p), c


@pytest.mark.parametrize("world_seed", range(100, 108))
def test_precompute_traj_bench_tracks_equal_cpu(bench_track_config, geom, world_seed):
    """The bench's own C4 tracks (world seeds 100..107: rank r plans seed 100 + r, bench.py
    full_plan) through OnlineTrajGenerator::preComputeTraj with the default row-restricted
    search, against the CPU restatement of the whole track (oracle/track_planner.py):
    identical waypoints, trajectory within 1e-6, the time column exact.  Two calls: the
    first (planner call numbers 0..8) and the second (9..17), as the bench repeats it."""
    import track_planner as TP
    path, c = bench_track_config
    gates, obstacles = synth.track_world(world_seed)
    cps0 = synth.gate_checkpoints(gates, geom.gate_height, 0.55)
    otg = _ot().OnlineTrajGenerator(cps0[0], cps0[-1], gates, obstacles, path)
    rg, ro = config.inflate_radii(c)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    lo, hi = np.array(c["world_properties"]["lower_bound"], float), np.array(c["world_properties"]["upper_bound"], float)
    tg = c["trajectory_generator_properties"]
    for first_call in (0, 9):
        otg.pre_compute_traj(0.0)
        wp, rows = TP.plan_track(w, rg, ro, lo, hi, otg.get_checkpoints(), 65536, tg["max_velocity"],
                                 tg["max_acceleration"], tg["sampling_interval"], threads=16, first_call=first_call)
        assert np.array_equal(otg.get_waypoints(), wp), (world_seed, first_call)
        traj = otg.get_planned_traj()
        assert traj.shape == rows.shape and np.array_equal(traj[:, 9], rows[:, 9])
        assert np.abs(traj[:, :9] - rows[:, :9]).max() < 1e-6


# ---- multi-GPU: the exchange step (RCCL) and planTracks -----------------------------
def test_comm_single_rank_allgather():
    """epp_comm_* on one rank (the box has one GPU): the all-gather returns the rank's own
    ragged set, an empty set, and EPP_ERR_CAPACITY with the counts when a set exceeds cap."""
    uid = capi.Comm.unique_id()
    assert len(uid) == 128
    c = capi.Comm(uid, 1, 0)
    assert (c.rank, c.n_ranks) == (0, 1)
    wp = synth.sample_states(3, [-6, -6, 0], [6, 6, 2], 37)
    sets = c.allgather_waypoints(wp, cap=64)
    assert len(sets) == 1 and np.array_equal(sets[0], wp)
    assert c.allgather_waypoints(np.zeros((0, 3)), cap=8)[0].shape == (0, 3)
    with pytest.raises(capi.EppError) as e:
        c.allgather_waypoints(wp, cap=10)
    assert e.value.code == capi.EPP_ERR_CAPACITY
    c.close()
    (ca,) = capi.Comm.init_all([0])
    assert np.array_equal(ca.allgather_waypoints(wp[:5])[0], wp[:5])
    ca.close()


@pytest.mark.parametrize("order", ["no-torch", "epp-first", "torch-first"])
def test_comm_any_import_order(order):
    """The exchange step works whichever HIP runtime the process loaded first: libepp.so
    before PyTorch leaves two runtimes (and two RCCLs) in the process, and epp_comm must
    use the RCCL of its own runtime (scripts/rccl_probe.py, one process per order)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_probe.py"), order],
                       capture_output=True, text=True, timeout=120)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith(order)]
    assert r.returncode == 0 and line and line[-1].split()[1] == "ok", (r.stdout[-2000:], r.stderr[-2000:])


def test_plan_tracks_across_devices(track, geom):
    """planTracks (include/epp/MultiTrackPlanner.h) over this box's GPU: every track's
    all-gathered waypoints and trajectory equal a standalone OnlineTrajGenerator's."""
    path, c, gates, obstacles, start, goal = track
    g2, o2 = synth.track_world(101)
    cps2 = synth.gate_checkpoints(g2, geom.gate_height, 0.55)
    problems = [(start, goal, gates, obstacles), (cps2[0], cps2[-1], g2, o2), (start, goal, gates, obstacles)]
    res = _ot().plan_tracks(problems, path, [0])
    assert len(res) == 3
    for (wp, traj, dev), (s, gl, g, o) in zip(res, problems):
        otg = _ot().OnlineTrajGenerator(s, gl, g, o, path)
        otg.pre_compute_traj(0.0)
        assert dev == 0
        assert np.array_equal(wp, otg.get_waypoints())
        assert np.array_equal(traj, otg.get_planned_traj())


# ---- the online replan against its CPU restatement (oracle/track_planner.py) ----------
def _online_pair(track, geom, tmp_path, recalc):
    import track_planner as TP
    path, c, gates, obstacles, start, goal = track
    c2 = json.loads(json.dumps(c))
    c2["path_planner_properties"]["recalculate_online"] = recalc
    p2 = tmp_path / f"c_online_{int(recalc)}.json"
    p2.write_text(json.dumps(c2))
    otg = _ot().OnlineTrajGenerator(start, goal, gates, obstacles, str(p2))
    otg.pre_compute_traj(0.0)
    cpu = TP.OnlineTrajGeneratorCPU(geom, c2, start, goal, gates, obstacles, threads=8)
    cpu.pre_compute_traj(0.0)
    assert np.array_equal(otg.get_waypoints(), cpu.waypoints)
    return otg, cpu, c2, gates


def _assert_same_state(otg, cpu, tol=1e-6):
    assert np.array_equal(otg.get_checkpoints(), np.array(cpu.checkpoints))
    assert np.array_equal(otg.get_waypoints(), cpu.waypoints)
    traj = otg.get_planned_traj()
    assert traj.shape == cpu.traj.shape and np.array_equal(traj[:, 9], cpu.traj[:, 9])
    assert np.abs(traj[:, :9] - cpu.traj[:, :9]).max() < tol


@pytest.mark.parametrize("recalc", [False, True])
def test_online_replan_equals_cpu_restatement(tmp_path, track, geom, recalc):
    """OnlineTrajGenerator::updateGatePos -> recomputeTraj (src/OnlineTrajGenerator.cpp:
    123-226, :258-421) pinned to the CPU restatement: the same decision, the two segment
    plans (seeded by the planner's call index), includeGates2 on the slice, the refit from
    the advanced state and the merge give identical checkpoints and waypoints and a
    trajectory within 1e-6 with the time column exact -- for a sequence of updates (two
    replans and a gate already observed), inline and on the online worker.

    The replan starts from a row of the current trajectory, whose bits seed the planner:
    the CPU copy continues from the product's rows (equal to its own within 1e-6, checked),
    so both replan from the same state."""
    otg, cpu, c2, gates = _online_pair(track, geom, tmp_path, recalc)
    before = otg.get_planned_traj()
    assert np.array_equal(before[:, 9], cpu.traj[:, 9]) and np.abs(before[:, :9] - cpu.traj[:, :9]).max() < 1e-6
    replans = 0
    for gid, shift, t_fly in ((2, 0.3, 2.0), (5, 0.3, 6.5), (2, 0.3, 6.6)):
        cur = otg.get_planned_traj()
        cpu.traj = cur.copy()
        i = int(np.argmin(np.abs(cur[:, 9] - t_fly)))
        drone = cur[i, [0, 3, 6]]
        pose = _lateral(gates[gid], shift)
        r = otg.update_gate_pos(gid, pose, drone, True, t_fly)
        if recalc:
            otg.wait_for_update()
        rc = cpu.update_gate_pos(gid, np.array(pose), drone, True, t_fly)
        assert r == rc, (gid, r, rc)
        replans += int(r)
        _assert_same_state(otg, cpu)
    assert replans >= 1 and cpu.calls == 9 + 2 * replans  # each replan took two planner calls
    cnt = otg.recompute_counts()  # every True return here ran the two plans (no degraded exit)
    assert cnt == {"planned": replans, "skipped_invalid_start": 0, "failed": 0}, cnt


def test_online_update_during_replan_keeps_reference_returns(tmp_path):
    """While an online recomputation runs (recalculate_online), another gate's update gets
    the reference's answer (src/OnlineTrajGenerator.cpp:141-212), pinned to the CPU
    restatement -- see tests/online_busy_case.py.  The case holds the online worker with a
    test hook that exists only in the -DEPP_TEST_HOOKS build (efficient-path-planner_amd/
    testhooks/), so it runs in a subprocess that loads that build instead of the product."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "online_busy_case.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "online busy case ok" in r.stdout


# ---- multi-GPU error protocol ------------------------------------------------------------
def test_comm_failure_protocol_single_rank():
    """A rank with no set (its own work failed) joins the all-gather with count -1: every
    rank gets EPP_ERR_PEER with the counts naming it; the all-reduce and barrier the bench
    uses for its max-over-ranks timing and collective error flags."""
    c = capi.Comm(capi.Comm.unique_id(), 1, 0)
    with pytest.raises(capi.EppError) as e:
        c.allgather_waypoints(None, cap=16)
    assert e.value.code == capi.EPP_ERR_PEER and list(e.value.counts) == [-1]
    wp = synth.sample_states(4, [-6, -6, 0], [6, 6, 2], 9)
    assert np.array_equal(c.allgather_waypoints(wp, cap=16)[0], wp)  # usable afterwards
    x = np.array([1.5, -2.0, 7.25])
    for op in (capi.EPP_REDUCE_SUM, capi.EPP_REDUCE_MAX, capi.EPP_REDUCE_MIN):
        assert np.array_equal(c.allreduce(x, op), x)
    c.barrier()
    c.close()


def test_comm_abort_and_timeout_single_rank():
    """The collectives' failure safety (epp.h): an abort requested from any thread makes the
    collective in flight or the next one abort the communicator and fail with EPP_ERR_PEER
    instead of waiting in RCCL; every later call fails at once; destroy still works.  The
    deadline setter validates its argument."""
    c = capi.Comm(capi.Comm.unique_id(), 1, 0)
    c.set_timeout(5.0)
    with pytest.raises(capi.EppError) as e:
        c.set_timeout(0.0)
    assert e.value.code == capi.EPP_ERR_INVALID_ARGUMENT
    wp = synth.sample_states(6, [-6, -6, 0], [6, 6, 2], 5)
    assert np.array_equal(c.allgather_waypoints(wp, cap=8)[0], wp)
    c.abort()
    with pytest.raises(capi.EppError) as e:
        c.allgather_waypoints(wp, cap=8)
    assert e.value.code == capi.EPP_ERR_PEER and "aborted" in str(e.value)
    with pytest.raises(capi.EppError) as e:
        c.barrier()
    assert e.value.code == capi.EPP_ERR_PEER
    c.close()
    c2 = capi.Comm(capi.Comm.unique_id(), 1, 0)  # a new communicator works
    c2.barrier()
    c2.close()


def test_rccl_group_single_rank():
    """eppamd.dist.RcclGroup (the bench's torch-free process group) on one rank."""
    from eppamd.dist import LegFailed, RcclGroup
    g = RcclGroup(1, 0)
    g.barrier()
    assert g.max(3.0) == 3.0 and g.sum(2.0) == 2.0
    wp = synth.sample_states(5, [-6, -6, 0], [6, 6, 2], 4)
    assert np.array_equal(g.all_gather_waypoints(wp)[0], wp)
    with pytest.raises(LegFailed) as e:
        g.all_gather_waypoints(None)
    assert e.value.failed == [0]
    with pytest.raises(LegFailed):
        g.check(RuntimeError("Path not found"))
    g.check(None)
    g.close()


def test_plan_tracks_failure_raises_not_hangs(track, geom):
    """planTracks with an unplannable track (its goal inside an obstacle) raises that
    track's "Path not found" instead of stranding the other rounds in the all-gather;
    a later call on the same device still works."""
    path, c, gates, obstacles, start, goal = track
    blocked_goal = obstacles[0, :3] + [0.0, 0.0, 0.5]
    problems = [(start, goal, gates, obstacles), (start, blocked_goal, gates, obstacles),
                (start, goal, gates, obstacles)]
    with pytest.raises(RuntimeError, match="Path not found"):
        _ot().plan_tracks(problems, path, [0])
    res = _ot().plan_tracks(problems[:1], path, [0])
    assert len(res) == 1 and len(res[0][0]) > 2


def test_comm_deadline_and_abort_in_flight():
    """The exchange's failure safety with a collective in flight: the deadline
    and an abort from another thread end the call while the collective is still queued,
    and nothing is copied into the caller's buffers afterwards -- see
    tests/comm_stall_case.py.  The in-flight collective is held by a bounded stall that
    exists only in the -DEPP_TEST_HOOKS build (efficient-path-planner_amd/testhooks/), so
    the case runs in a subprocess that loads that build instead of the product."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-u", os.path.join(here, "comm_stall_case.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "comm stall case ok" in r.stdout

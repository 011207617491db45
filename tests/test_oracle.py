"""CPU tests: pin the oracle against the reference's own known answers and invariants.

Reference tests mirrored here: external/poly_traj/test/test_polynomial_optimization.cpp
(TwoVerticesSetup :743-787, AMatrixInversion :731-741, checkPath :113-174,
ConstraintPacking :505-564, TimeAllocation :566-606) and the hand-derived World/OBB
known answers in tests/golden/obb_boundary.json.
"""
import json
import os

import numpy as np
import pytest

import minsnap_np
import oracle as O
import pyref_obb
from eppamd import config, synth
from eppamd.config import OBB_DESC_DTYPE, Geometry

from conftest import GOLDEN

REF = json.load(open(os.path.join(GOLDEN, "reference_minsnap.json")))


def _vertex_constraints(wp, max_derivative=4):
    """createRandomVertices vertex set: ends fixed up to max_derivative (p, then 0), inner p."""
    W, D = wp.shape
    mask = np.zeros((W, 5), np.uint8)
    val = np.zeros((W, 5, D))
    for v in range(W):
        mask[v, 0] = 1
        val[v, 0] = wp[v]
    for v in (0, W - 1):
        mask[v, : max_derivative + 1] = 1
    return mask, val


def test_two_vertices_setup_golden():
    c = REF["two_vertices_setup"]
    mask = np.ones((2, 5), np.uint8)
    val = np.zeros((2, 5, 1))
    val[0, 0, 0], val[1, 0, 0] = c["start_x"], c["goal_x"]
    coeffs = O.minsnap_solve(mask, val, [c["segment_time"]], 1, c["derivative"])[0, 0]
    np.testing.assert_allclose(coeffs, c["matlab_coeffs"], rtol=0, atol=c["tolerance"])


def test_a_matrix_inversion():
    c = REF["a_matrix_inversion"]
    for t in range(c["t_min"], c["t_max"] + 1):
        A = O.mapping_matrix(float(t))
        Ai = O.invert_mapping(A)
        assert np.abs(Ai - np.linalg.inv(A)).max() < c["tolerance"], t


def _check_path(wp, times, coeffs, mask, val, tol):
    """checkPath: fixed constraints met, C0..C4 continuity at every vertex (tol 1e-6)."""
    M = len(times)
    D = wp.shape[1]
    for i in range(M):
        for k in range(5):
            for d in range(D):
                beg = O.poly_eval(coeffs[i, d], 0.0, k)
                end = O.poly_eval(coeffs[i, d], times[i], k)
                if mask[i, k]:
                    assert abs(beg - val[i, k, d]) < tol
                if mask[i + 1, k]:
                    assert abs(end - val[i + 1, k, d]) < tol
                if i > 0:
                    prev = O.poly_eval(coeffs[i - 1, d], times[i - 1], k)
                    assert abs(prev - beg) < tol


@pytest.mark.parametrize("ps", REF["parameter_sets"], ids=lambda p: p["name"])
def test_unconstrained_linear_estimate_segment_times(ps):
    D = ps["D"]
    wp = O.random_vertices(ps["segments"], D, -ps["pos"], ps["pos"], ps["seed"])
    assert wp.shape == (ps["segments"] + 1, D)
    assert (wp <= ps["pos"]).all() and (wp >= -ps["pos"]).all()  # VertexGeneration
    times = O.segment_times(wp, ps["v_max"], ps["a_max"])
    assert ((times > 0) & (times < REF["time_allocation"]["upper"])).all()  # TimeAllocation
    mask, val = _vertex_constraints(wp)
    coeffs = O.minsnap_solve(mask, val, times, D, ps["deriv"])
    _check_path(wp, times, coeffs, mask, val, REF["check_path_tolerance"]["tol"])
    # v/a within 2.5x limits (numerical maximum, test_utils.h getMaximumMagnitude)
    if ps["deriv"] == 4:
        vm = am = 0.0
        for i in range(len(times)):
            for t in np.arange(0, times[i], 0.01):
                v = [O.poly_eval(coeffs[i, d], t, 1) for d in range(D)]
                a = [O.poly_eval(coeffs[i, d], t, 2) for d in range(D)]
                vm, am = max(vm, np.linalg.norm(v)), max(am, np.linalg.norm(a))
        assert vm < 2.5 * ps["v_max"] and am < 2.5 * ps["a_max"]


@pytest.mark.parametrize("D", [1, 3])
def test_constraint_packing(D):
    c = REF["constraint_packing"]
    for k in range(c["setups"]):
        wp = O.random_vertices(10, D, -c["pos"], c["pos"], c["seed"] + k)
        times = O.segment_times(wp, c["v_max"], c["a_max"])
        mask, val = _vertex_constraints(wp)
        coeffs = O.minsnap_solve(mask, val, times, D, 4)
        # p -> d: A_i p_i reproduces [d(vertex i); d(vertex i+1)] and is continuous
        for i, T in enumerate(times):
            A = O.mapping_matrix(T)
            for d in range(D):
                dd = A @ coeffs[i, d]
                if i > 0:
                    prev = O.mapping_matrix(times[i - 1]) @ coeffs[i - 1, d]
                    np.testing.assert_allclose(dd[:5], prev[5:], atol=c["tol"])
                np.testing.assert_allclose(dd[0], wp[i, d], atol=c["tol"])
                np.testing.assert_allclose(dd[5], wp[i + 1, d], atol=c["tol"])


def test_oracle_vs_numpy_kkt():
    """Independent formulation (KKT in normalised time) agrees with the oracle."""
    for s in range(6):
        wp = synth.random_track_waypoints(50 + s, 12)
        T, Cf = O.minsnap_track(wp, 1.0, 2.0)
        Cn = minsnap_np.track(wp, T)
        assert np.abs(Cf - Cn).max() < 1e-7


def test_oracle_vs_high_precision():
    """30-digit KKT solve (mpmath) on a small track pins the absolute accuracy."""
    mp = pytest.importorskip("mpmath")
    from math import factorial
    mp.mp.dps = 30
    wp = synth.random_track_waypoints(7, 4)
    T, Cf = O.minsnap_track(wp, 1.0, 2.0)
    N, K, M = 10, 4, len(T)
    ff = lambda j, k: mp.mpf(factorial(j)) / factorial(j - k) if j >= k else mp.mpf(0)  # noqa: E731
    Tm = [mp.mpf(float(t)) for t in T]
    nv = N * M
    fixed = {(0, k): (wp[0] if k == 0 else np.zeros(3)) for k in range(5)}
    fixed.update({(M, k): (wp[M] if k == 0 else np.zeros(3)) for k in range(5)})
    fixed.update({(v, 0): wp[v] for v in range(1, M)})
    rows, rhs = [], []

    def drow(k, tau, seg):
        r = [mp.mpf(0)] * nv
        for j in range(k, N):
            r[N * seg + j] = ff(j, k) * (mp.mpf(tau) ** (j - k) if j > k else 1) / Tm[seg] ** k
        return r
    for v in range(M + 1):
        for k in range(5):
            if (v, k) in fixed:
                for seg, tau in ((v - 1, 1), (v, 0)):
                    if 0 <= seg < M:
                        rows.append(drow(k, tau, seg))
                        rhs.append([mp.mpf(float(x)) for x in fixed[(v, k)]])
            elif 0 < v < M:
                a, b = drow(k, 1, v - 1), drow(k, 0, v)
                rows.append([x - y for x, y in zip(a, b)])
                rhs.append([mp.mpf(0)] * 3)
    nc = len(rows)
    A = mp.zeros(nv + nc, nv + nc)
    for i in range(M):
        for a in range(K, N):
            for b in range(K, N):
                A[N * i + a, N * i + b] = 2 * ff(a, K) * ff(b, K) / (a + b - 2 * K + 1) / Tm[i] ** (2 * K - 1)
    for r in range(nc):
        for c in range(nv):
            if rows[r][c] != 0:
                A[nv + r, c] = rows[r][c]
                A[c, nv + r] = rows[r][c]
    for d in range(3):
        x = mp.lu_solve(A, mp.matrix([0] * nv + [rhs[r][d] for r in range(nc)]))
        exact = np.array([[float(x[N * i + j] / Tm[i] ** j) for j in range(N)] for i in range(M)])
        assert np.abs(Cf[:, d, :] - exact).max() < 1e-7  # well inside the 1e-6 parity budget


def _mp_reduced_track(wp, T, dps=40):
    """The reference's own formulation (impl/polynomial_optimization_linear_impl.h:111-379:
    A_i, Q_i, H_i = A_i^-T Q_i A_i^-1, R = C^T H C, R_pp d_p = -R_pf d_f, p_i = A_i^-1 d_i)
    carried out in `dps`-digit arithmetic (mpmath), where the cancellation in H that costs
    the double-precision formulation ~7 digits does not matter."""
    mp = pytest.importorskip("mpmath")
    from math import factorial
    mp.mp.dps = dps
    N, H5, M = 10, 5, len(T)
    ff = lambda j, k: mp.mpf(factorial(j)) / factorial(j - k) if j >= k else mp.mpf(0)  # noqa: E731
    fixed = lambda v, k: v == 0 or v == M or k == 0  # noqa: E731  (generateTrajectory's vertices)
    col, nf = {}, 0
    for v in range(M + 1):
        for k in range(H5):
            if fixed(v, k):
                col[(v, k)], nf = nf, nf + 1
    n_all = nf
    for v in range(M + 1):
        for k in range(H5):
            if not fixed(v, k):
                col[(v, k)], n_all = n_all, n_all + 1
    R = mp.zeros(n_all, n_all)
    Ainv = []
    for i in range(M):
        t = mp.mpf(float(T[i]))
        A = mp.zeros(N, N)
        for k in range(H5):
            A[k, k] = ff(k, k)
            for j in range(k, N):
                A[H5 + k, j] = ff(j, k) * t ** (j - k)
        Ai = mp.inverse(A)
        Ainv.append(Ai)
        Q = mp.zeros(N, N)
        for a in range(4, N):
            for b in range(4, N):
                Q[a, b] = ff(a, 4) * ff(b, 4) * t ** (a + b - 7) / (a + b - 7)
        H = Ai.T * Q * Ai
        idx = [col[(i + r // H5, r % H5)] for r in range(N)]
        for r in range(N):
            for c in range(N):
                R[idx[r], idx[c]] += H[r, c]
    npf = n_all - nf
    Rpp = mp.matrix([[R[nf + r, nf + c] for c in range(npf)] for r in range(npf)])
    out = np.zeros((M, 3, N))
    for d in range(3):
        df = [mp.mpf(0)] * nf
        for v in range(M + 1):
            df[col[(v, 0)]] = mp.mpf(float(wp[v][d]))
        dp = mp.lu_solve(Rpp, mp.matrix([-mp.fsum(R[nf + r, c] * df[c] for c in range(nf)) for r in range(npf)]))
        dall = df + [dp[r] for r in range(npf)]
        for i in range(M):
            p = Ainv[i] * mp.matrix([dall[col[(i + r // H5, r % H5)]] for r in range(N)])
            out[i, d] = [float(p[j]) for j in range(N)]
    return out


@pytest.mark.parametrize("problem", [184, 1540, 1742, 2942])
def test_truth_pinned_to_high_precision(problem):
    """The accuracy reference ("truth") is minsnap_np.track_batch_refined: the reference's
    formulation in long double from exact rational constants, refined against the
    long-double residual.  Pinned here against the same formulation carried out at 40
    digits (an independent implementation in mpmath), on the bench's C5 problems (seeds
    10000 + problem) the verdict and this round's probes singled out: within 2e-13.  The
    double-precision KKT (`track`, a different formulation) is within 4e-9 (problem 1742:
    3.4e-9 -- why it is a cross-check, not the truth); the oracle -- the reference's
    formulation in doubles, as the reference computes it, H = A^-T Q A^-1 by products whose
    terms cancel -- is off by up to 9.5e-7 (problem 2942)."""
    wp = synth.random_track_waypoints(10_000 + problem, 12)
    T, Cf = O.minsnap_track(wp, 1.0, 2.0)
    exact = _mp_reduced_track(wp, T)
    assert np.abs(minsnap_np.track_batch_refined(wp[None], T[None])[0] - exact).max() < 2e-13
    assert np.abs(minsnap_np.track(wp, T) - exact).max() < 4e-9
    assert np.abs(Cf - exact).max() < 1e-6  # (the reference formulation's own rounding)


def test_truth_short_segments_pinned():
    """The truth on short and mixed-length segments (coefficients up to ~1e7): within
    1e-13 of the 40-digit solve relative to the track's largest coefficient."""
    rng = np.random.default_rng(1)
    steps = rng.uniform(0.02, 3.0, (2, 12, 1)) * rng.normal(size=(2, 12, 3))
    mixed = np.concatenate([np.zeros((2, 1, 3)), np.cumsum(steps, axis=1)], axis=1)
    small = np.array([synth.random_track_waypoints(50_000 + k, 12) for k in range(2)]) * 0.03
    for wps in (mixed, small):
        Ts = np.array([O.segment_times(w, 1.0, 2.0) for w in wps])
        got = minsnap_np.track_batch_refined(wps, Ts)
        for j in range(len(wps)):
            exact = _mp_reduced_track(wps[j], Ts[j])
            assert np.abs(got[j] - exact).max() <= 1e-13 * np.abs(exact).max()


def test_truth_batch_equals_single():
    """track_batch (batched assembly + LU) equals track problem by problem, and the refined
    truth agrees with both to the KKT's accuracy."""
    tracks = np.array([synth.random_track_waypoints(300 + s, 7) for s in range(20)])
    Ts = np.array([O.minsnap_track(w, 1.0, 2.0)[0] for w in tracks])
    got = minsnap_np.track_batch(tracks, Ts, chunk=7)
    ref = minsnap_np.track_batch_refined(tracks, Ts)
    for k in range(len(tracks)):
        assert np.abs(got[k] - minsnap_np.track(tracks[k], Ts[k])).max() < 1e-10
        assert np.abs(ref[k] - got[k]).max() < 1e-8


def test_evaluate_range_recurrence():
    """Sample count/time column follow Trajectory::evaluateRange (src/trajectory.cpp:81-141)."""
    wp = synth.random_track_waypoints(3, 5)
    T, Cf = O.minsnap_track(wp, 1.0, 2.0)
    rows = O.sample_traj(T, Cf, 0.1, t0=2.0)
    acc, i, tis, times = 0.0, 0, 0.0, []
    t_end = 0.0
    for t in T:
        t_end += t
    while acc < t_end:
        if tis > T[i]:
            tis -= T[i]
            i += 1
            if i >= len(T):
                break
            continue
        times.append(acc + 2.0)
        tis += 0.1
        acc += 0.1
    assert len(rows) == len(times)
    assert (rows[:, 9] == np.array(times)).all()
    assert abs(rows[0, 0] - wp[0, 0]) < 1e-12 and abs(rows[0, 1]) < 1e-12


def test_golden_tracks_oracle():
    g = json.load(open(os.path.join(GOLDEN, "minsnap_tracks.json")))
    for tr in g["tracks"][:6]:
        T, Cf = O.minsnap_track(np.array(tr["wp"]), tr["v_max"], tr["a_max"], tr["v0"], tr["a0"])
        assert np.array_equal(T, np.array(tr["times"]))
        assert np.abs(Cf - np.array(tr["coeffs"])).max() < 1e-12


def _boundary_world():
    f = json.load(open(os.path.join(GOLDEN, "obb_boundary.json")))

    def descs(lst):
        a = np.zeros(len(lst), OBB_DESC_DTYPE)
        for i, d in enumerate(lst):
            a[i]["pos"], a[i]["size"], a[i]["filling"] = d["pos"], d["size"], d["filling"]
        return a
    g = Geometry(descs(f["gate_desc"]), np.array([0, len(f["gate_desc"])], np.int32), descs(f["obst_desc"]),
                 np.array([1.0]))
    return f, g


def test_obb_boundary_known_answers():
    f, g = _boundary_world()
    w = O.world_build(g, f["gates"], f["obstacles"], f["r_gate"], f["r_obst"])
    for c in f["points"]:
        assert O.check_states(w, f["r_gate"], f["r_obst"], np.array([c["p"]]), c["can_pass"])[0] == c["valid"], c
    for c in f["mindist"]:
        assert O.check_states_mindist(w, np.array([c["p"]]), c["md"])[0] == c["valid"], c
    for c in f["rays"]:
        got = O.check_motions(w, f["r_gate"], f["r_obst"], np.array([c["s"]]), np.array([c["e"]]),
                              c["can_pass"], c["mode"])[0]
        assert got == c["valid"], c


@pytest.mark.parametrize("cfg_name", ["config.json", "config_filling.json"])
def test_oracle_vs_pure_python_track_world(cfg_name):
    """Two independent restatements agree; config_filling.json adds a filling OBB per gate
    (the opening), so the can_pass_gate skips are exercised too."""
    cfg = config.load(os.path.join(os.path.dirname(GOLDEN), "..", "configs", cfg_name))
    geom = config.geometry(cfg)
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    w = O.world_build(geom, gates, obstacles, rg, ro)
    gd = [{"pos": d["pos"].tolist(), "size": d["size"].tolist(), "filling": int(d["filling"])} for d in geom.gate_desc]
    od = [{"pos": d["pos"].tolist(), "size": d["size"].tolist(), "filling": int(d["filling"])} for d in geom.obst_desc]
    pw = pyref_obb.build(gd, geom.gate_desc_off.tolist(), od, gates, obstacles, rg, ro)
    for k, o in enumerate(w):
        assert list(o["aabb_lo"]) == pw[k]["aabb_lo"] and list(o["aabb_hi"]) == pw[k]["aabb_hi"]
        assert list(o["center"]) == pw[k]["center"]
    lo, hi = synth.C2_BOUNDS
    pts = synth.sample_states(11, lo, np.array([6.0, 6.0, 1.6]), 1500)
    # plus states in and around the gate openings (gate frame offsets, rotated by the yaw)
    rs = np.random.RandomState(1)
    loc = rs.uniform([-0.3, -0.05, -0.3], [0.3, 0.05, 0.3], size=(len(gates), 60, 3))
    c, s = np.cos(gates[:, 5])[:, None], np.sin(gates[:, 5])[:, None]
    h = geom.gate_height[gates[:, 6].astype(int)][:, None]
    op = np.stack([gates[:, :1] + c * loc[..., 0] - s * loc[..., 1], gates[:, 1:2] + s * loc[..., 0] + c * loc[..., 1],
                   h + loc[..., 2]], -1).reshape(-1, 3)
    pts = np.vstack([pts, op])
    if cfg_name == "config_filling.json":
        assert (O.check_states(w, rg, ro, op, 1) > O.check_states(w, rg, ro, op, 0)).sum() > 20
    for cp in (0, 1):
        got = O.check_states(w, rg, ro, pts, cp)
        ref = np.array([pyref_obb.point_valid(pw, rg, ro, list(p), cp) for p in pts], np.uint8)
        assert (got == ref).all()
    s1, s2 = synth.edges(12, 13, lo, np.array([6.0, 6.0, 1.6]), 600, max_len=1.5)
    for mode in (0, 1):
        for cp in (0, 1):
            got = O.check_motions(w, rg, ro, s1, s2, cp, mode)
            fn = pyref_obb.ray_valid if mode == 0 else pyref_obb.ray_valid_d32
            ref = np.array([fn(pw, rg, ro, list(a), list(b), cp) for a, b in zip(s1, s2)], np.uint8)
            assert (got == ref).all()
    md = O.check_states_mindist(w, pts, 0.3)
    ref = np.array([pyref_obb.point_valid_mindist(pw, list(p), 0.3) for p in pts], np.uint8)
    assert (md == ref).all()


def test_golden_c1_states_oracle(geom):
    f = json.load(open(os.path.join(GOLDEN, "c1_states.json")))
    w = O.world_build(geom, f["gates"], f["obstacles"], f["r_gate"], f["r_obst"])
    for cp in ("0", "1"):
        got = O.check_states(w, f["r_gate"], f["r_obst"], np.array(f["states"]), int(cp))
        assert got.tolist() == f["valid"][cp]


def test_world_build_errors(geom):
    with pytest.raises(ValueError):
        O.world_build(geom, [[0, 0, 0, 0.1, 0, 0, 0]], np.zeros((0, 6)), 0.2, 0.2)  # roll
    with pytest.raises(ValueError):
        O.world_build(geom, np.zeros((0, 7)), [[0, 0, 0.5, 0, 0, 0]], 0.2, 0.2)  # obstacle z


def test_counter_sampler_matches_oracle():
    lo, hi = synth.C2_BOUNDS
    a = synth.sample_states(7, lo, hi, 5000)
    b = O.sample_states(7, lo, hi, 5000)
    assert np.array_equal(a, b)


def test_cpu_planner_restatement_basic(cfg, geom):
    """or_plan_once (the CPU restatement of the batch planner): deterministic, thread-count
    independent, valid paths under the oracle's validators, None for a blocked goal; the
    k-NN inside matches brute force (ties to the lower index)."""
    rg, ro = config.inflate_radii(cfg)
    g, o, start, goal = synth.c1_world()
    w = O.world_build(geom, g, o, rg, ro)
    lo, hi = synth.C1_BOUNDS
    a, sa = O.plan_once(w, rg, ro, lo, hi, start, goal, 3000, 7, 16, False, 1)
    b, sb = O.plan_once(w, rg, ro, lo, hi, start, goal, 3000, 7, 16, False, 5)
    assert a is not None and np.array_equal(a, b) and np.array_equal(sa, sb)
    assert np.array_equal(a[0], start) and np.array_equal(a[-1], goal)
    assert O.check_motions(w, rg, ro, a[:-1], a[1:]).all()
    assert O.plan_once(w, rg, ro, lo, hi, start, np.array([1.0, 0.5, 0.5]), 3000, 7)[0] is None
    assert sa[4] == 0  # (the forward search found it)
    # a goal 0.8 m outside the sampling box: no sample keeps it among its 16 neighbours, so
    # the forward search fails and the symmetrised graph decides (stats[4] = 1)
    far = np.array([0.0, hi[1] + 0.8, 0.3])
    c, sc = O.plan_once(w, rg, ro, lo, hi, start, far, 1000, 0, 16, False, 4)
    assert c is not None and sc[4] == 1 and np.array_equal(c[-1], far)
    assert O.check_motions(w, rg, ro, c[:-1], c[1:]).all()


def test_track_planner_seed_derivation():
    """track_planner.mix / call_seed restate host_planner.cpp's 64-bit mixing (spot values
    computed with the C++ expression)."""
    import track_planner as TP
    assert TP.mix(0, 0) == 0xE220A8397B1DCDAF
    assert TP.mix(0x5EED, 12345678901234) == 0x15220C2B70B99518

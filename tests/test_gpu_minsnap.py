"""GPU parity: batched min-snap fit + sampling (through the C ABI) vs the CPU oracle.

Reference: poly_traj::generateTrajectory (external/poly_traj/src/trajectory_generator.cpp:12-100).
Tolerances (north_star): coefficients within 1e-6; segment times to 1e-12 relative
(device exp vs glibc exp); sample count and time column exact; sampled values 1e-6.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from eppamd import capi, synth

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

COEF_TOL = 1e-6


def test_golden_tracks():
    g = json.load(open(os.path.join(GOLDEN, "minsnap_tracks.json")))
    tracks = [np.array(t["wp"]) for t in g["tracks"]]
    v0 = np.array([t["v0"] for t in g["tracks"]])
    a0 = np.array([t["a0"] for t in g["tracks"]])
    Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0, v0, a0)
    assert (st == 0).all()
    for t, T, Cf in zip(g["tracks"], Ts, Cs):
        np.testing.assert_allclose(T, t["times"], rtol=1e-12, atol=0)
        assert np.abs(Cf - np.array(t["coeffs"])).max() < COEF_TOL


@pytest.mark.parametrize("n_seg", [1, 2, 5, 12, 24, 25, 40])
def test_batch_vs_oracle(n_seg):
    """12 segments = BASELINE config 5; > 24 segments runs the global-scratch kernel."""
    tracks = [synth.random_track_waypoints(300 + 17 * n_seg + k, n_seg) for k in range(16)]
    rs = np.random.RandomState(n_seg)
    v0 = rs.uniform(-0.5, 0.5, (16, 3))
    a0 = rs.uniform(-0.5, 0.5, (16, 3))
    Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0, v0, a0)
    assert (st == 0).all()
    worst = 0.0
    for k, wp in enumerate(tracks):
        T, Cf = O.minsnap_track(wp, 1.0, 2.0, v0[k], a0[k])
        np.testing.assert_allclose(Ts[k], T, rtol=1e-12)
        worst = max(worst, np.abs(Cs[k] - Cf).max())
    assert worst < COEF_TOL, worst


def test_mixed_track_lengths_and_errors():
    tracks = [synth.random_track_waypoints(900 + k, 1 + (k * 7) % 30) for k in range(40)]
    tracks.insert(5, np.zeros((1, 3)))            # fewer than 2 waypoints
    tracks.insert(9, np.array([[0, 0, 1.0], [0, 0, 1.0]]))  # zero-length segment: T = 0
    Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0)
    assert st[5] == -1 and st[9] == -2
    for k, wp in enumerate(tracks):
        if k in (5, 9):
            continue
        assert st[k] == 0
        T, Cf = O.minsnap_track(wp, 1.0, 2.0)
        assert np.abs(Cs[k] - Cf).max() < COEF_TOL


def test_generate_trajectory_rows():
    g = json.load(open(os.path.join(GOLDEN, "traj_rows.json")))
    for c in g["cases"]:
        got = capi.generate_trajectory(np.array(c["wp"]), c["v_max"], c["a_max"], c["dt"], c["t0"])
        exp = np.array(c["rows"])
        assert got.shape == exp.shape
        assert np.array_equal(got[:, 9], exp[:, 9])       # time column exact
        assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6


@pytest.mark.parametrize("seed", range(6))
def test_generate_trajectory_vs_oracle(seed):
    wp = synth.random_track_waypoints(500 + seed, 3 + 2 * seed)
    v0, a0 = (0.3, -0.2, 0.1), (0.0, 0.5, -0.1)
    got = capi.generate_trajectory(wp, 1.0, 2.0, 0.1, 3.25, v0, a0)
    exp = O.generate_trajectory(wp, 1.0, 2.0, 0.1, 3.25, v0, a0)
    assert got.shape == exp.shape
    assert np.array_equal(got[:, 9], exp[:, 9])
    assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6
    # starts at the first waypoint with the given velocity/acceleration
    np.testing.assert_allclose(got[0, [0, 3, 6]], wp[0], atol=1e-9)
    np.testing.assert_allclose(got[0, [1, 4, 7]], v0, atol=1e-9)
    np.testing.assert_allclose(got[0, [2, 5, 8]], a0, atol=1e-9)


@pytest.mark.parametrize("n,dt", [(40, 0.1), (26, 0.01), (9, 0.003), (60, 0.1), (200, 0.05), (331, 0.1),
                                  (800, 0.1), (2000, 0.2)])
def test_generate_trajectory_long_tracks(n, dt):
    """The single-track latency path: up to 40 segments in LDS; more: the segment scratch
    in global memory; past ~300 segments (e.g. a track smoothed by "ompl" simplification:
    ~330 waypoints) the vertex values and coefficients too ("big" refit); many rows (row
    buffer sized from host-side segment times)."""
    wp = synth.random_track_waypoints(900 + n, n)
    got = capi.generate_trajectory(wp, 1.5, 2.5, dt, 0.5)
    exp = O.generate_trajectory(wp, 1.5, 2.5, dt, 0.5)
    assert got.shape == exp.shape
    assert np.array_equal(got[:, 9], exp[:, 9])
    assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6


def test_generate_trajectory_zero_segment():
    wp = np.array([[0.0, 0.0, 0.5], [1.0, 2.0, 1.5], [1.0, 2.0, 1.5], [2.0, 0.0, 1.0]])
    with pytest.raises(capi.EppError) as e:
        capi.generate_trajectory(wp, 1.0, 2.0, 0.1)
    assert "Segment times need to be greater than zero" in str(e.value)


def test_generate_trajectory_two_waypoints_and_errors():
    wp = np.array([[0.0, 0.0, 0.5], [1.0, 2.0, 1.5]])
    got = capi.generate_trajectory(wp, 1.0, 2.0, 0.05)
    exp = O.generate_trajectory(wp, 1.0, 2.0, 0.05)
    assert got.shape == exp.shape and np.abs(got - exp).max() < 1e-9
    with pytest.raises(capi.EppError) as e:
        capi.generate_trajectory(wp[:1], 1.0, 2.0, 0.1)
    assert e.value.code == capi.EPP_ERR_INVALID_ARGUMENT
    assert "At least two waypoints are required" in str(e.value)


def test_large_batch_property():
    """4096 twelve-segment problems -- the bench's C5 batched launch itself (same seeds,
    bench.py side_measurements): EVERY problem's segment times within 1e-12 relative and
    coefficients within 1e-6 of the oracle (north_star), plus continuity of derivatives
    0..4 at every inner vertex and the end constraints (size-independent)."""
    tracks = [synth.random_track_waypoints(10_000 + k, 12) for k in range(4096)]
    Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0)
    assert (st == 0).all()
    worst_c = worst_t = 0.0
    for k, wp in enumerate(tracks):
        T_ref, C_ref = O.minsnap_track(wp, 1.0, 2.0)
        worst_t = max(worst_t, float(np.max(np.abs(Ts[k] - T_ref) / T_ref)))
        worst_c = max(worst_c, float(np.max(np.abs(Cs[k] - C_ref))))
    assert worst_t <= 1e-12, worst_t
    assert worst_c < 1e-6, worst_c
    for k in range(0, 4096, 97):
        T, Cf = Ts[k], Cs[k]
        for i in range(1, 12):
            for d in range(3):
                for der in range(5):
                    a = O.poly_eval(Cf[i - 1, d], T[i - 1], der)
                    b = O.poly_eval(Cf[i, d], 0.0, der)
                    assert abs(a - b) < 1e-6
        np.testing.assert_allclose([O.poly_eval(Cf[-1, d], T[-1], 0) for d in range(3)], tracks[k][-1],
                                   atol=1e-6)


# ---- accuracy against the truth -----------------------------------------------------
# The truth: minsnap_np.track_batch_refined (the reference's formulation in long double,
# refined; pinned to a 40-digit solve in tests/test_oracle.py).  The oracle restates the
# reference's double-precision arithmetic, whose H = A^-T Q A^-1 products cancel: it is up
# to 9.5e-7 off the truth on the bench's batch, so GPU-vs-oracle at 1e-6 alone measures the
# oracle as much as the GPU.
def _norm_err(C, truth, T):
    """Per problem: the largest error of the time-normalised coefficients c_j T^j (a bound on
    the sampled positions' error, up to the factor 10) over the track's largest normalised
    coefficient."""
    C, truth, T = np.asarray(C), np.asarray(truth), np.asarray(T)
    Tn = T[:, :, None, None] ** np.arange(10)[None, None, None, :]
    d = (np.abs(C - truth) * Tn).reshape(len(T), -1).max(1)
    return d / (np.abs(truth) * Tn).reshape(len(T), -1).max(1)


def test_batch_vs_truth():
    """The bench's C5 batch (4096 x 12 segments): every problem within 1e-9 of the truth
    (absolute, coefficients up to ~100), and never farther from the oracle than the
    oracle is from the truth plus 1e-9."""
    import minsnap_np as MN
    tracks = np.array([synth.random_track_waypoints(10_000 + k, 12) for k in range(4096)])
    Ts, Cs, st = capi.minsnap_batch(list(tracks), 1.0, 2.0)
    assert (np.asarray(st) == 0).all()
    Tr, Cr, _ = O.minsnap_batch(list(tracks), 1.0, 2.0, threads=16)
    truth = MN.track_batch_refined(tracks, Tr)
    eg = np.abs(np.asarray(Cs) - truth).reshape(4096, -1).max(1)
    eo = np.abs(np.asarray(Cr) - truth).reshape(4096, -1).max(1)
    ego = np.abs(np.asarray(Cs) - np.asarray(Cr)).reshape(4096, -1).max(1)
    assert eg.max() <= 1e-9, (eg.max(), eg.argmax())
    assert (ego <= eo + 1e-9).all()


def test_batch_vs_truth_short_segment_sweep():
    """65,536 twelve-segment problems with short and mixed segment lengths (waypoints of
    random tracks scaled by 0.1 and 0.03: segments down to ~13 ms and coefficients up to
    ~1e13; and random walks of 0.02-3 m steps: long and very short segments side by side,
    R_pp's condition up to ~1e12): the time-normalised error (_norm_err) within 1e-6 of the
    track's scale, and within the oracle's own on every problem.  (Measured, round 6: 4e-7
    at worst -- the rounding of the data, H's entries Hc T^e in doubles, times R_pp's
    condition; the refinement step brings the solve to that level -- against the
    reference formulation's own 4e-4.  The absolute error of a short segment's
    c_9 ~ (its length) / T^9 has no meaning at these scales: the reference's own
    formulation is off by up to ~1e5 there.)"""
    import minsnap_np as MN
    rng = np.random.default_rng(66)
    n3 = 65536 // 3
    sets = [np.array([synth.random_track_waypoints(70_000 + k, 12) for k in range(n3)]) * 0.1,
            np.array([synth.random_track_waypoints(90_000 + k, 12) for k in range(n3)]) * 0.03]
    n = 65536 - 2 * n3
    steps = rng.uniform(0.02, 3.0, (n, 12, 1)) * rng.normal(size=(n, 12, 3))
    sets.append(np.concatenate([np.zeros((n, 1, 3)), np.cumsum(steps, axis=1)], axis=1))
    worst = 0.0
    for tracks in sets:
        Ts, Cs, st = capi.minsnap_batch(list(tracks), 1.0, 2.0)
        assert (np.asarray(st) == 0).all()
        Tr, Cr, _ = O.minsnap_batch(list(tracks), 1.0, 2.0, threads=16)
        truth = MN.track_batch_refined(tracks, Tr)
        eg, eo = _norm_err(Cs, truth, Tr), _norm_err(Cr, truth, Tr)
        assert (eg <= np.maximum(eo, 1e-12)).all()
        worst = max(worst, float(eg.max()))
    assert worst <= 1e-6, worst


# ---- pinned directly to the reference's own vectors ---------------------------------
# external/poly_traj/test/test_polynomial_optimization.cpp (fixtures in
# tests/golden/reference_minsnap.json): the GPU is compared with the reference's numbers,
# not only with the oracle.
REF = json.load(open(os.path.join(GOLDEN, "reference_minsnap.json")))


def _embed3(wp):
    wp = np.asarray(wp, np.float64)
    out = np.zeros((len(wp), 3))
    out[:, :wp.shape[1]] = wp
    return out


def test_two_vertices_setup_reference_golden():
    """TwoVerticesSetup (:743-787): rest-to-rest 0 -> 5 m in T = 5 s, snap; the
    reference's MATLAB coefficients at 1e-12, embedded in 3-D (y, z at rest at 0), via
    setupFromVertices(vertices, segment_times) = epp_minsnap_batch_times and the fused
    single-track path."""
    c = REF["two_vertices_setup"]
    wp = np.array([[c["start_x"], 0.0, 0.0], [c["goal_x"], 0.0, 0.0]])
    Cs, st = capi.minsnap_batch_times([wp], [[c["segment_time"]]])
    assert st[0] == 0
    np.testing.assert_allclose(Cs[0][0, 0], c["matlab_coeffs"], rtol=0, atol=c["tolerance"])
    assert np.abs(Cs[0][0, 1:]).max() == 0.0
    rows = capi.generate_trajectory_times(wp, [c["segment_time"]], 0.05)
    t = rows[:, 9]
    x = np.polyval(np.asarray(c["matlab_coeffs"])[::-1], t)
    np.testing.assert_allclose(rows[:, 0], x, rtol=0, atol=1e-9)  # (golden rounded to ~1e-15 per coefficient)
    # sample times follow evaluateRange exactly (they depend on the segment time only)
    assert np.array_equal(t, O.sample_traj([c["segment_time"]], Cs[0], 0.05)[:, 9])


def _check_path(times, coeffs, wp, D, tol):
    """checkPath (:113-174): vertex constraints met (positions; start/end derivatives 1..4
    zero) and C0..C4 continuity at every inner vertex."""
    M = len(times)
    for i in range(M):
        for d in range(3):
            for k in range(5):
                beg = O.poly_eval(coeffs[i, d], 0.0, k)
                end = O.poly_eval(coeffs[i, d], times[i], k)
                if k == 0:
                    assert abs(beg - (wp[i, d] if d < D else 0.0)) < tol
                    assert abs(end - (wp[i + 1, d] if d < D else 0.0)) < tol
                if i == 0 and k > 0:
                    assert abs(beg) < tol
                if i == M - 1 and k > 0:
                    assert abs(end) < tol
                if i > 0:
                    assert abs(O.poly_eval(coeffs[i - 1, d], times[i - 1], k) - beg) < tol


SNAP_SETS = [p for p in REF["parameter_sets"] if p["deriv"] == 4]


@pytest.mark.parametrize("ps", SNAP_SETS, ids=lambda p: p["name"])
def test_reference_parameter_sets(ps):
    """The reference's snap parameter sets segment_{1,10,50}_dim_{1,3} (:790-879):
    createRandomVertices (std::mt19937, src/vertex.cpp:27-82) -> estimateSegmentTimes
    (Nfabian) -> solve, checked with checkPath at the reference's 1e-6, and against the
    oracle's coefficients at 1e-6.  50 segments run the global-scratch kernel."""
    D = ps["D"]
    wp = _embed3(O.random_vertices(ps["segments"], D, -ps["pos"], ps["pos"], ps["seed"]))
    Ts, Cs, st = capi.minsnap_batch([wp], ps["v_max"], ps["a_max"])
    assert st[0] == 0
    T_ref = O.segment_times(wp[:, :D], ps["v_max"], ps["a_max"])
    np.testing.assert_allclose(Ts[0], T_ref, rtol=1e-12)
    _check_path(Ts[0], Cs[0], wp, D, REF["check_path_tolerance"]["tol"])
    mask = np.zeros((len(wp), 5), np.uint8)
    mask[:, 0] = 1
    mask[0, :] = mask[-1, :] = 1
    val = np.zeros((len(wp), 5, D))
    val[:, 0] = wp[:, :D]
    ref = O.minsnap_solve(mask, val, T_ref, D, 4)
    assert np.abs(Cs[0][:, :D] - ref).max() < COEF_TOL
    # the same with the caller's times (setupFromVertices(vertices, times))
    Ct, st2 = capi.minsnap_batch_times([wp], [T_ref])
    assert st2[0] == 0 and np.abs(Ct[0][:, :D] - ref).max() < COEF_TOL


@pytest.mark.parametrize("D", [1, 3])
def test_constraint_packing_reference(D):
    """ConstraintPacking (:505-564): 5 setups of 10 segments (seeds 12345..12349,
    positions +-50): A_i p_i reproduces the vertex values and is continuous (1e-6)."""
    c = REF["constraint_packing"]
    tracks = [_embed3(O.random_vertices(10, D, -c["pos"], c["pos"], c["seed"] + k)) for k in range(c["setups"])]
    Ts, Cs, st = capi.minsnap_batch(tracks, c["v_max"], c["a_max"])
    assert (st == 0).all()
    for wp, T, Cf in zip(tracks, Ts, Cs):
        for i in range(len(T)):
            A = O.mapping_matrix(T[i])
            for d in range(3):
                dd = A @ Cf[i, d]
                if i > 0:  # derivatives 0..4 at the shared vertex
                    prev = O.mapping_matrix(T[i - 1]) @ Cf[i - 1, d]
                    np.testing.assert_allclose(dd[:5], prev[5:], atol=c["tol"])
                np.testing.assert_allclose(dd[0], wp[i, d], atol=c["tol"])
                np.testing.assert_allclose(dd[5], wp[i + 1, d], atol=c["tol"])


@pytest.mark.parametrize("seed", range(4))
def test_generate_trajectory_times_vs_oracle(seed):
    rs = np.random.RandomState(seed)
    wp = synth.random_track_waypoints(700 + seed, 4 + 3 * seed)
    T = O.segment_times(wp, 1.0, 2.0) * rs.uniform(0.7, 1.4, len(wp) - 1)  # caller times near Nfabian's
    got = capi.generate_trajectory_times(wp, T, 0.1, 1.5, (0.2, 0.0, -0.1), (0.0, 0.3, 0.0))
    mask = np.zeros((len(wp), 5), np.uint8)
    mask[:, 0] = 1
    mask[0, :] = mask[-1, :] = 1
    val = np.zeros((len(wp), 5, 3))
    val[:, 0] = wp
    val[0, 1], val[0, 2] = (0.2, 0.0, -0.1), (0.0, 0.3, 0.0)
    exp = O.sample_traj(T, O.minsnap_solve(mask, val, T, 3, 4), 0.1, 1.5)
    assert got.shape == exp.shape
    assert np.array_equal(got[:, 9], exp[:, 9])
    assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6
    with pytest.raises(capi.EppError) as e:
        capi.generate_trajectory_times(wp, np.where(np.arange(len(T)) == 1, 0.0, T), 0.1)
    assert "Segment times need to be greater than zero" in str(e.value)


def test_long_tracks_two_streams_back_to_back():
    """Tracks longer than the LDS limit use the per-device workspace; two streams issuing
    batches back to back must not share it while the first still runs (event-ordered
    reuse), answers equal the oracle's."""
    import ctypes as C
    L = capi.lib()
    batches = [[synth.random_track_waypoints(4000 + 50 * b + k, 45 + k % 7) for k in range(24)] for b in range(2)]
    streams = []
    for _ in batches:
        s = C.c_void_p()
        capi.check(L.epp_stream_create(C.byref(s)))
        streams.append(s.value)
    bufs, outs = [], []
    for tracks, s in zip(batches, streams):
        wp = np.ascontiguousarray(np.concatenate(tracks))
        off = np.zeros(len(tracks) + 1, np.int32)
        off[1:] = np.cumsum([len(t) for t in tracks])
        nseg = int(off[-1]) - len(tracks)
        d = [capi.DeviceBuffer.from_array(wp), capi.DeviceBuffer.from_array(off), capi.DeviceBuffer(8 * nseg),
             capi.DeviceBuffer(240 * nseg), capi.DeviceBuffer(4 * len(tracks))]
        bufs.append(d)
        outs.append((off, nseg))
    for (dwp, doff, dT, dC, dst), tracks, s in zip(bufs, batches, streams):  # back to back, no sync between
        capi.check(L.epp_minsnap_batch(dwp.ptr, doff.ptr, len(tracks), 1.0, 2.0, None, None, dT.ptr, dC.ptr,
                                       dst.ptr, s))
    capi.sync()
    for (dwp, doff, dT, dC, dst), tracks, (off, nseg) in zip(bufs, batches, outs):
        Cf = dC.download(np.float64, nseg * 30).reshape(nseg, 3, 10)
        assert (dst.download(np.int32, len(tracks)) == 0).all()
        for k, wp in enumerate(tracks):
            _, ref = O.minsnap_track(wp, 1.0, 2.0)
            assert np.abs(Cf[int(off[k]) - k:int(off[k + 1]) - k - 1] - ref).max() < COEF_TOL
    for s in streams:
        L.epp_stream_destroy(s)


# ---- the polynomial_trajectory pybind surface (external/poly_traj/README.md:79) -------
@pytest.mark.parametrize("seed", range(3))
def test_polynomial_trajectory_module(seed):
    """polynomial_trajectory.generate_trajectory(waypoints, v_max, a_max,
    sampling_intervall) with the README's arguments vs the oracle: same shape, time
    column exact, 1e-6 elsewhere; start time offset and initial state keywords."""
    import polynomial_trajectory as pt
    wp = synth.random_track_waypoints(800 + seed, 5 + 4 * seed)
    got = pt.generate_trajectory(wp, 1.0, 2.0, 0.1)
    exp = O.generate_trajectory(wp, 1.0, 2.0, 0.1)
    assert got.shape == exp.shape and got.shape[1] == 10
    assert np.array_equal(got[:, 9], exp[:, 9])
    assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6
    got = pt.generate_trajectory(wp, 1.5, 2.5, 0.05, startTimeOffset=2.0, initialVel=[0.1, 0.2, 0.0],
                                 initialAcc=[0.0, 0.0, 0.3])
    exp = O.generate_trajectory(wp, 1.5, 2.5, 0.05, 2.0, (0.1, 0.2, 0.0), (0.0, 0.0, 0.3))
    assert got.shape == exp.shape and np.array_equal(got[:, 9], exp[:, 9])
    assert np.abs(got[:, :9] - exp[:, :9]).max() < 1e-6


def test_polynomial_trajectory_errors():
    import polynomial_trajectory as pt
    with pytest.raises(ValueError, match="At least two waypoints are required"):
        pt.generate_trajectory(np.zeros((1, 3)), 1.0, 2.0, 0.1)
    with pytest.raises(ValueError):
        pt.generate_trajectory(np.zeros((4, 2)), 1.0, 2.0, 0.1)  # not (n, 3)
    with pytest.raises(RuntimeError, match="Segment times need to be greater than zero"):
        pt.generate_trajectory(np.array([[0, 0, 1.0], [0, 0, 1.0], [1, 0, 1.0]]), 1.0, 2.0, 0.1)


# ---- the C5 online step in one launch (epp_check_and_generate_trajectory_host) ---------
def _c5_world(cfg, geom):
    from eppamd import config
    rg, ro = config.inflate_radii(cfg)
    gates, obstacles = synth.track_world(42)
    return gates, obstacles, rg, ro


@pytest.mark.parametrize("n_check", [0, 1, 100, 300, 4096])
def test_check_and_generate_equals_two_calls(cfg, geom, n_check):
    """The fused launch gives the A11 flags of World::checkPointValidity(p, minDistance)
    (src/World.cpp:106-128; the oracle, bit for bit) and the rows of generateTrajectory
    (the separate call, bit for bit; the oracle within 1e-6, time column exact), on the
    current index and after a gate update (records read from pinned host memory)."""
    gates, obstacles, rg, ro = _c5_world(cfg, geom)
    md = float(cfg["path_planner_properties"]["min_dist_check_traj_collision"])
    wp = synth.random_track_waypoints(77, 12)
    for version in range(2):
        g = gates.copy()
        if version:
            g[2, :2] += 0.25
        ref = O.world_build(geom, g, obstacles, rg, ro)
        w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
        if version:
            w.update(capi.build_obbs(geom, g, obstacles))  # index stale: pinned records
        rows0 = O.generate_trajectory(wp, 1.0, 2.0, 0.1, 0.0, (0.3, -0.1, 0.0), (0.0, 0.2, 0.0))
        pts = np.vstack([rows0[:, [0, 3, 6]], synth.sample_states(5 + n_check, [-6, -6, 0], [6, 6, 2], 4096)])[:n_check]
        flags, rows = capi.check_and_generate_trajectory(w, pts, md, wp, 1.0, 2.0, 0.1, 0.0, (0.3, -0.1, 0.0),
                                                         (0.0, 0.2, 0.0))
        assert np.array_equal(flags, O.check_states_mindist(ref, pts, md))
        if n_check:
            assert np.array_equal(flags, w.check_states_mindist(pts, md))
        sep = capi.generate_trajectory(wp, 1.0, 2.0, 0.1, 0.0, (0.3, -0.1, 0.0), (0.0, 0.2, 0.0))
        assert np.array_equal(rows, sep)
        assert rows.shape == rows0.shape and np.array_equal(rows[:, 9], rows0[:, 9])
        assert np.abs(rows[:, :9] - rows0[:, :9]).max() < 1e-6
        w.close()


def test_check_and_generate_large_check_unsupported_and_planner_fallback(cfg, geom, tmp_path):
    """Over the small path's limit (4096 points) the C ABI says EPP_ERR_UNSUPPORTED; the
    C++ / pybind PathPlanner entry then makes the two calls (same answers)."""
    import online_traj_planner as otp
    import polynomial_trajectory as pt
    from conftest import CONFIG
    gates, obstacles, rg, ro = _c5_world(cfg, geom)
    md = float(cfg["path_planner_properties"]["min_dist_check_traj_collision"])
    w = capi.World(capi.build_obbs(geom, gates, obstacles), rg, ro)
    wp = synth.random_track_waypoints(78, 12)
    pts = synth.sample_states(9, [-6, -6, 0], [6, 6, 2], 4097)
    with pytest.raises(capi.EppError) as e:
        capi.check_and_generate_trajectory(w, pts, md, wp, 1.0, 2.0, 0.1)
    assert e.value.code == capi.EPP_ERR_UNSUPPORTED
    w.close()
    pp = otp.PathPlanner(gates, obstacles, CONFIG)
    for n in (100, 4097):
        traj = np.zeros((n, 10))
        traj[:, [0, 3, 6]] = synth.sample_states(10 + n, [-6, -6, 0], [6, 6, 2], n)
        ok, rows = pp.check_trajectory_validity_and_generate(traj, md, wp, 1.0, 2.0, 0.1, 0.5, (0.1, 0, 0), (0, 0, 0))
        assert ok == pp.check_trajectory_validity(traj, md)
        assert np.array_equal(rows, pt.generate_trajectory(wp, 1.0, 2.0, 0.1, 0.5, (0.1, 0, 0), (0, 0, 0)))
    traj = O.generate_trajectory(wp, 1.0, 2.0, 0.1)[:100]  # the trajectory's own lookahead
    ok, _ = pp.check_trajectory_validity_and_generate(traj, md, wp, 1.0, 2.0, 0.1)
    assert ok == pp.check_trajectory_validity(traj, md)

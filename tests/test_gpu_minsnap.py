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


@pytest.mark.parametrize("n,dt", [(40, 0.1), (26, 0.01), (9, 0.003)])
def test_generate_trajectory_long_tracks(n, dt):
    """The single-track latency path: more than 24 segments (global scratch), many rows
    (row buffer sized from host-side segment times)."""
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
    """4096 twelve-segment problems (BASELINE config 5 batched variant): continuity of
    derivatives 0..4 at every inner vertex and the end constraints, size-independent."""
    tracks = [synth.random_track_waypoints(10_000 + k, 12) for k in range(4096)]
    Ts, Cs, st = capi.minsnap_batch(tracks, 1.0, 2.0)
    assert (st == 0).all()
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

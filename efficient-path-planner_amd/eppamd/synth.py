"""Deterministic synthetic worlds and query batches.

Everything here is input data: the same arrays are handed to the HIP path and to the
CPU oracle.  Layouts follow the reference: gates are rows (x, y, z, roll, pitch, yaw,
type) and obstacles rows (x, y, z, roll, pitch, yaw) (src/pybind.cpp:13-14,
src/PathPlanner.cpp:60-78).
"""
from __future__ import annotations

import numpy as np

C2_BOUNDS = (np.array([-6.0, -6.0, 0.0]), np.array([6.0, 6.0, 2.0]))
C1_BOUNDS = (np.array([-2.0, -2.0, 0.0]), np.array([2.0, 2.0, 2.0]))

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + _GOLD).astype(np.uint64)
    x = (x ^ (x >> np.uint64(30))) * _M1
    x = (x ^ (x >> np.uint64(27))) * _M2
    return x ^ (x >> np.uint64(31))


def sample_states(seed: int, lo, hi, n: int, start: int = 0) -> np.ndarray:
    """Counter-based uniform states: u = (splitmix64(seed ^ (3i+d)) >> 11) * 2^-53."""
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    i = np.arange(start, start + n, dtype=np.uint64)[:, None] * np.uint64(3) + np.arange(3, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        r = splitmix64(np.uint64(seed) ^ i)
    u = (r >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return lo + (hi - lo) * u


def c1_world():
    """Config 1: one large portal at the origin + 4 single-OBB obstacles (bounds [-2,2]^2 x [0,2])."""
    gates = np.array([[0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0]], float)
    obstacles = np.array([[1.0, 0.5, 0, 0, 0, 0], [-1.0, 0.5, 0, 0, 0, 0],
                          [0.8, -0.9, 0, 0, 0, 0], [-0.7, -1.1, 0, 0, 0, 0]], float)
    start = np.array([0.0, -1.6, 0.3])
    goal = np.array([0.0, 1.6, 0.3])
    return gates, obstacles, start, goal


def track_world(seed: int, n_gates: int = 8, n_obstacles: int = 24, a: float = 4.0, b: float = 3.0,
                clearance: float = 0.5):
    """Gates on an ellipse (yaw tangent + U(-0.3, 0.3), type U{0,1}) and obstacles uniform in
    [-6,6]^2 with >= `clearance` m from every gate centre."""
    rs = np.random.RandomState(seed)
    gates = np.zeros((n_gates, 7))
    for g in range(n_gates):
        th = 2 * np.pi * g / n_gates
        x, y = a * np.cos(th), b * np.sin(th)
        tx, ty = -a * np.sin(th), b * np.cos(th)      # tangent
        yaw = np.arctan2(ty, tx) - np.pi / 2 + rs.uniform(-0.3, 0.3)  # gate normal ~ tangent
        gates[g] = [x, y, 0.0, 0.0, 0.0, yaw, rs.randint(0, 2)]
    obstacles = np.zeros((n_obstacles, 6))
    k = 0
    while k < n_obstacles:
        p = rs.uniform(-6, 6, size=2)
        if np.min(np.hypot(gates[:, 0] - p[0], gates[:, 1] - p[1])) < clearance + 0.45:
            continue
        obstacles[k, :2] = p
        k += 1
    return gates, obstacles


def edges(seed_start: int, seed_dir: int, lo, hi, n: int, max_len: float = 0.5):
    """Motion edges: s1 ~ counter sampler, s2 = s1 + dir * U(0, max_len), clipped to bounds."""
    s1 = sample_states(seed_start, lo, hi, n)
    rs = np.random.RandomState(seed_dir)
    d = rs.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    s2 = s1 + d * rs.uniform(0, max_len, size=(n, 1))
    s2 = np.clip(s2, lo, hi)
    return s1, s2


def gate_checkpoints(gates: np.ndarray, heights: np.ndarray, offset: float):
    """OnlineTrajGenerator ctor checkpoints (src/OnlineTrajGenerator.cpp:32-70)."""
    out = []
    for g in gates:
        c = np.array([g[0], g[1], g[2] + heights[int(g[6])]])
        n = np.array([-np.sin(g[5]), np.cos(g[5]), 0.0])
        n = n / np.linalg.norm(n)
        out.append(c - offset * n)
        out.append(c + offset * n)
    return np.array(out)


def random_track_waypoints(seed: int, n_segments: int = 12, extent: float = 5.0):
    """A racing-like waypoint list (W = n_segments + 1) for min-snap batches.

    Consecutive waypoints are >= 0.05 m apart, as after PathPlanner::includeGates2's
    de-duplication (src/PathPlanner.cpp:222)."""
    rs = np.random.RandomState(seed)
    while True:
        th = np.sort(rs.uniform(0, 2 * np.pi, n_segments + 1))
        r = extent * (0.6 + 0.4 * rs.uniform(size=n_segments + 1))
        z = rs.uniform(0.3, 1.5, n_segments + 1)
        wp = np.stack([r * np.cos(th), r * np.sin(th), z], 1)
        if np.linalg.norm(np.diff(wp, axis=0), axis=1).min() >= 0.05:
            return wp

"""TEST INFRASTRUCTURE ONLY — numpy restatement of the "spline" trajectory type
(src/TrajInterpolation.cpp:1-68: Eigen::SplineFitting<Spline3d>::Interpolate(points, 3,
chord-length parameters), sampled uniformly in the parameter).

Independent formulation from csrc/host_spline.cpp: B-spline basis by the Cox-de Boor
recursion (not the triangular de Boor scheme), control points by numpy.linalg.solve.
Agreement to ~1e-12 cross-checks both.  Parity UNPINNED against the reference (Eigen's
unsupported Splines module is absent; no reference fixture covers this debug type).
"""
from __future__ import annotations

import numpy as np

DEG = 3


def _basis(i, k, u, knots):
    """N_{i,k}(u) by Cox-de Boor; the last non-empty span is closed at u = knots[-1]."""
    if k == 0:
        lo, hi = knots[i], knots[i + 1]
        if lo <= u < hi:
            return 1.0
        return 1.0 if (u == knots[-1] and hi == knots[-1] and lo < hi) else 0.0
    out = 0.0
    d1 = knots[i + k] - knots[i]
    if d1 > 0:
        out += (u - knots[i]) / d1 * _basis(i, k - 1, u, knots)
    d2 = knots[i + k + 1] - knots[i + 1]
    if d2 > 0:
        out += (knots[i + k + 1] - u) / d2 * _basis(i + 1, k - 1, u, knots)
    return out


def interpolate_traj(path, max_t, t0, dt):
    """rows [x 0 0 y 0 0 z 0 0 t] (TrajInterpolation.cpp:44-68)."""
    p = np.asarray(path, float)
    n = len(p)
    t = np.concatenate([[0.0], np.cumsum(np.linalg.norm(np.diff(p, axis=0), axis=1))])
    t = t / t[-1]
    knots = np.zeros(n + DEG + 1)
    for j in range(1, n - DEG):
        knots[j + DEG] = t[j:j + DEG].mean()
    knots[n:] = 1.0
    A = np.array([[_basis(c, DEG, u, knots) for c in range(n)] for u in t])
    A[0, :] = 0.0
    A[-1, :] = 0.0
    A[0, 0] = A[-1, -1] = 1.0
    ctrl = np.linalg.solve(A, p)
    m = int((max_t - t0) / dt) + 1
    rows = np.zeros((m, 10))
    for i in range(m):
        u = i / (m - 1) if m > 1 else 0.0
        b = np.array([_basis(c, DEG, u, knots) for c in range(n)])
        rows[i, [0, 3, 6]] = b @ ctrl
        rows[i, 9] = i * dt + t0
    return rows

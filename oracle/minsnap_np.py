"""TEST INFRASTRUCTURE ONLY — independent numpy restatement of the min-snap solve.

A different formulation from epp_oracle.cpp (and from the reference's
PolynomialOptimization, which eliminates constraints through the mapping matrix and
solves R_pp d_p = -R_pf d_f): here the per-segment coefficients are solved directly
from the KKT system of

    minimise  sum_i  int_0^{T_i} |p_i''''(t)|^2 dt
    s.t.      fixed derivatives at the end vertices, positions at inner vertices,
              C^0..C^4 continuity at inner vertices,

in time-normalised coordinates (tau = t / T_i) for conditioning.  Agreement of the
two formulations to ~1e-9 cross-checks the oracle (see tests/test_oracle.py).
"""
from __future__ import annotations

from math import factorial

import numpy as np

N = 10
K = 4  # snap


def _ff(j: int, k: int) -> float:
    return factorial(j) / factorial(j - k) if j >= k else 0.0


def _deriv_row(k: int, tau: float) -> np.ndarray:
    """d^k/dtau^k of [1, tau, ..., tau^9] at tau."""
    return np.array([_ff(j, k) * tau ** (j - k) if j >= k else 0.0 for j in range(N)])


def _cost_unit() -> np.ndarray:
    """int_0^1 (q''''(tau))^2 dtau as a quadratic form in the normalised coefficients."""
    Q = np.zeros((N, N))
    for a in range(K, N):
        for b in range(K, N):
            Q[a, b] = _ff(a, K) * _ff(b, K) / (a + b - 2 * K + 1)
    return Q


def solve(fixed: dict, n_vertices: int, times, dim: int) -> np.ndarray:
    """fixed[(v, k)] = value vector (dim,) of derivative k at vertex v.

    Every vertex must fix its position; unfixed derivatives 1..4 of inner vertices
    are continuous.  Returns coefficients (segments, dim, 10) in increasing powers of
    the un-normalised time t."""
    M = n_vertices - 1
    T = np.asarray(times, float)
    nv = N * M
    Qu = _cost_unit()
    H = np.zeros((nv, nv))
    for i in range(M):
        H[N * i:N * i + N, N * i:N * i + N] = Qu / T[i] ** (2 * K - 1)
    rows, rhs = [], []

    def add(row, val):
        rows.append(row)
        rhs.append(val)

    for v in range(n_vertices):
        for k in range(5):
            key = (v, k)
            if v > 0:  # end of segment v-1 (tau = 1): d^k/dt^k = T^-k d^k/dtau^k
                end = np.zeros(nv)
                end[N * (v - 1):N * v] = _deriv_row(k, 1.0) / T[v - 1] ** k
            if v < M:
                beg = np.zeros(nv)
                beg[N * v:N * v + N] = _deriv_row(k, 0.0) / T[v] ** k
            if key in fixed:
                val = np.asarray(fixed[key], float)
                if v > 0:
                    add(end, val)
                if v < M:
                    add(beg, val)
            elif 0 < v < M:
                add(end - beg, np.zeros(dim))
    A = np.array(rows)
    b = np.array(rhs)
    nc = len(rows)
    kkt = np.zeros((nv + nc, nv + nc))
    kkt[:nv, :nv] = 2 * H
    kkt[:nv, nv:] = A.T
    kkt[nv:, :nv] = A
    sol = np.linalg.solve(kkt, np.vstack([np.zeros((nv, dim)), b]))[:nv]
    out = np.zeros((M, dim, N))
    for i in range(M):
        scale = T[i] ** -np.arange(N, dtype=float)
        out[i] = (sol[N * i:N * i + N] * scale[:, None]).T
    return out


def track_batch(wps, times, v0=(0, 0, 0), a0=(0, 0, 0), chunk: int = 256) -> np.ndarray:
    """`track` for B problems of the same waypoint count W at once: wps (B, W, 3), times
    (B, W - 1) -> coefficients (B, W - 1, 3, 10), increasing powers of t.  The same KKT
    system in normalised time as `track`, assembled for the whole batch and solved by
    batched LU (partial pivoting), `chunk` problems at a time.  This is the accuracy
    reference ("truth") the GPU and the oracle are both measured against: 40-digit mpmath
    agrees with it to ~1e-12 on the bench's problems (tests/test_oracle.py), where the
    reference's own formulation (R = C^T A^-T Q A^-1 C in the monomial basis, H formed by
    products whose terms cancel) loses ~7 digits."""
    wps = np.asarray(wps, float)
    B, W, dim = wps.shape
    M = W - 1
    T = np.asarray(times, float).reshape(B, M)
    nv = N * M
    Qu = _cost_unit()
    # constraint structure: (kind, vertex, k) per row; rows are shared by the batch, only
    # the 1/T^k scales and the right-hand sides differ
    fixed = {(0, k) for k in range(5)} | {(v, 0) for v in range(1, M)} | {(M, k) for k in range(5)}
    spec = []  # (seg_end or -1, seg_beg or -1, k, sign_beg, rhs source)
    for v in range(W):
        for k in range(5):
            if (v, k) in fixed:
                if v > 0:
                    spec.append((v - 1, -1, k, (v, k)))
                if v < M:
                    spec.append((-1, v, k, (v, k)))
            elif 0 < v < M:
                spec.append((v - 1, v, k, None))
    nc = len(spec)
    ones, zeros = [_deriv_row(k, 1.0) for k in range(5)], [_deriv_row(k, 0.0) for k in range(5)]
    v0, a0 = np.asarray(v0, float), np.asarray(a0, float)
    out = np.zeros((B, M, dim, N))
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        nb = b1 - b0
        Tb = T[b0:b1]
        kkt = np.zeros((nb, nv + nc, nv + nc))
        for i in range(M):
            kkt[:, N * i:N * i + N, N * i:N * i + N] = 2 * Qu[None] / Tb[:, i, None, None] ** (2 * K - 1)
        rhs = np.zeros((nb, nv + nc, dim))
        for r, (se, sb, k, src) in enumerate(spec):
            row = np.zeros((nb, nv))
            if se >= 0:
                row[:, N * se:N * se + N] += ones[k][None] / Tb[:, se, None] ** k
            if sb >= 0:
                row[:, N * sb:N * sb + N] -= (zeros[k][None] / Tb[:, sb, None] ** k) * (1 if se >= 0 else -1)
            kkt[:, nv + r, :nv] = row
            kkt[:, :nv, nv + r] = row
            if src is not None:
                v, kk = src
                if kk == 0:
                    rhs[:, nv + r] = wps[b0:b1, v]
                elif v == 0 and kk == 1:
                    rhs[:, nv + r] = v0
                elif v == 0 and kk == 2:
                    rhs[:, nv + r] = a0
        sol = np.linalg.solve(kkt, rhs)[:, :nv]
        for i in range(M):
            scale = Tb[:, i, None] ** -np.arange(N, dtype=float)[None]  # (nb, N)
            out[b0:b1, i] = np.transpose(sol[:, N * i:N * i + N] * scale[:, :, None], (0, 2, 1))
    return out


def track(wp, times, v0=(0, 0, 0), a0=(0, 0, 0)) -> np.ndarray:
    """generateTrajectory vertex set: start {p, v0, a0, 0, 0}, inner {p}, end {p, 0, 0, 0, 0}."""
    wp = np.asarray(wp, float)
    W = len(wp)
    fixed = {}
    z = np.zeros(3)
    fixed[(0, 0)], fixed[(0, 1)], fixed[(0, 2)], fixed[(0, 3)], fixed[(0, 4)] = wp[0], v0, a0, z, z
    for v in range(1, W - 1):
        fixed[(v, 0)] = wp[v]
    for k in range(5):
        fixed[(W - 1, k)] = wp[-1] if k == 0 else z
    return solve(fixed, W, times, 3)

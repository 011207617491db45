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

track_batch_refined is the accuracy reference ("truth") the GPU and the oracle are
measured against: the reference's own formulation in long double with iterative
refinement, pinned to 40-digit mpmath.
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
    batched LU (partial pivoting), `chunk` problems at a time.  An independent formulation
    (a cross-check of track_batch_refined, the accuracy reference): 40-digit mpmath agrees
    with it to ~4e-12 on most of the bench's problems, but it is off by up to ~3e-9 on a
    few (its KKT matrix is indefinite and pivoted across scales)."""
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


_LD_CONSTS = None


def _ld_consts():
    """Hc (H = A^-T Q A^-1 at T = 1) and A^-1 at T = 1 in long double, from exact rational
    arithmetic (every entry is a ratio of factorials)."""
    global _LD_CONSTS
    if _LD_CONSTS is None:
        from fractions import Fraction as F
        A = [[F(0)] * N for _ in range(N)]
        for k in range(5):
            A[k][k] = F(factorial(k))
            for j in range(k, N):
                A[5 + k][j] = F(factorial(j), factorial(j - k))
        # exact inverse by Gauss-Jordan over the rationals
        aug = [row[:] + [F(int(i == r)) for i in range(N)] for r, row in enumerate(A)]
        for c in range(N):
            piv = next(r for r in range(c, N) if aug[r][c] != 0)
            aug[c], aug[piv] = aug[piv], aug[c]
            pv = aug[c][c]
            aug[c] = [x / pv for x in aug[c]]
            for r in range(N):
                if r != c and aug[r][c] != 0:
                    f = aug[r][c]
                    aug[r] = [x - f * y for x, y in zip(aug[r], aug[c])]
        Ai = [row[N:] for row in aug]
        Q = [[F(0)] * N for _ in range(N)]
        for a in range(K, N):
            for b in range(K, N):
                Q[a][b] = F(factorial(a) // factorial(a - K) * (factorial(b) // factorial(b - K)), a + b - 7)
        H = [[sum(Ai[a][r] * Q[a][b] * Ai[b][c] for a in range(N) for b in range(N)) for c in range(N)]
             for r in range(N)]

        def ld(x):
            return np.longdouble(x.numerator) / np.longdouble(x.denominator)
        _LD_CONSTS = (np.array([[ld(x) for x in row] for row in H], dtype=np.longdouble),
                      np.array([[ld(x) for x in row] for row in Ai], dtype=np.longdouble))
    return _LD_CONSTS


def track_batch_refined(wps, times, v0=(0, 0, 0), a0=(0, 0, 0), iters: int = 3) -> np.ndarray:
    """The accuracy reference ("truth"): the reference's own formulation
    (impl/polynomial_optimization_linear_impl.h:111-379: H_i = A_i^-T Q_i A_i^-1 with
    H[r][c] = Hc[r][c] T^((r%5)+(c%5)-7), R_pp d_p = -R_pf d_f over the inner vertices'
    derivatives 1..4, p_i = A_i^-1 d_i) with every entry and product in long double (64-bit
    mantissa) from exact rational constants, solved in doubles and refined `iters` times
    against the long-double residual.  Pinned to 40-digit mpmath (tests/test_oracle.py):
    ~1e-13 on the bench's problems, where the double-precision KKT of `track_batch` is off
    by up to ~3e-9 on some of them.  wps (B, W, 3), times (B, W - 1) -> (B, W - 1, 3, 10)."""
    Hc, Ai = _ld_consts()
    wps = np.asarray(wps, np.longdouble)
    B, W, dim = wps.shape
    M = W - 1
    T = np.asarray(times, np.float64).reshape(B, M).astype(np.longdouble)
    nin = M - 1
    # vertex values dv[b, v, k, d]: fixed ones now, the free ones from the solve
    dv = np.zeros((B, W, 5, dim), np.longdouble)
    dv[:, :, 0] = wps
    dv[:, 0, 1] = np.asarray(v0, np.longdouble)
    dv[:, 0, 2] = np.asarray(a0, np.longdouble)
    tp = {e: T ** e for e in range(-9, 2)}  # T^e per segment, (B, M)

    def hs(seg, r, c):  # H_seg[r][c], (B,)
        return Hc[r, c] * tp[(r % 5) + (c % 5) - 7][:, seg]
    if nin > 0:
        n = 4 * nin
        R = np.zeros((B, n, n), np.longdouble)
        rhs = np.zeros((B, n, dim), np.longdouble)
        for v in range(1, M):
            for p in range(4):
                for q in range(4):
                    R[:, 4 * (v - 1) + p, 4 * (v - 1) + q] = hs(v - 1, 6 + p, 6 + q) + hs(v, 1 + p, 1 + q)
                    if v < nin:
                        R[:, 4 * (v - 1) + p, 4 * v + q] = hs(v, 1 + p, 6 + q)
                        R[:, 4 * v + q, 4 * (v - 1) + p] = hs(v, 1 + p, 6 + q)
                s = np.zeros((B, dim), np.longdouble)
                for seg, ro, vb in ((v - 1, 6, v - 1), (v, 1, v)):
                    for r in range(N):
                        vv, k = vb + (1 if r >= 5 else 0), r % 5
                        if k == 0 or vv == 0 or vv == M:
                            s += hs(seg, ro + p, r)[:, None] * dv[:, vv, k]
                rhs[:, 4 * (v - 1) + p] = -s
        R64 = R.astype(np.float64)
        x = np.linalg.solve(R64, rhs.astype(np.float64)).astype(np.longdouble)
        for _ in range(iters):
            res = rhs - np.einsum("bij,bjd->bid", R, x)
            x += np.linalg.solve(R64, res.astype(np.float64)).astype(np.longdouble)
        for v in range(1, M):
            dv[:, v, 1:5] = x[:, 4 * (v - 1):4 * v]
    out = np.zeros((B, M, dim, N), np.longdouble)
    for i in range(M):
        d0 = np.concatenate([dv[:, i], dv[:, i + 1]], axis=1)  # (B, 10, dim)
        for r in range(N):
            if r < 5:
                out[:, i, :, r] = Ai[r, r] * d0[:, r]
            else:
                s = np.zeros((B, dim), np.longdouble)
                for k in range(N):
                    if Ai[r, k] != 0:
                        s += (Ai[r, k] * tp[(k % 5) - r][:, i])[:, None] * d0[:, k]
                out[:, i, :, r] = s
    return out.astype(np.float64)


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

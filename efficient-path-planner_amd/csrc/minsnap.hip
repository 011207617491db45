// minsnap.hip — batched minimum-snap trajectory fitting and sampling for gfx950.
//
// Reference: poly_traj::generateTrajectory (external/poly_traj/src/trajectory_generator.cpp:12-100)
// built on mav_trajectory_generation::PolynomialOptimization<10>
// (include/mav_trajectory_generation/impl/polynomial_optimization_linear_impl.h).
//
// One 64-lane wavefront per track.  The formulation is the reference's:
//   T_i      Nfabian segment times                          src/vertex.cpp:272-289
//   A_i^-1   Schur inverse of the mapping matrix             impl :111-121, :142-179
//   Q_i      snap cost matrix                                impl :567-583
//   H_i      = A_i^-T Q_i A_i^-1                             impl :307-336
//   R_pp d_p = -R_pf d_f                                     impl :338-379
//   p_i      = A_i^-1 [d(vertex i); d(vertex i+1)]           impl :262-283
// The free constraints are derivatives 1..4 of the inner vertices, so R_pp is
// block-tridiagonal with 4x4 blocks (vertex v couples only with v-1 and v+1).  It is
// SPD and solved by block elimination (block Thomas with explicit 4x4 inverses) instead
// of the reference's Eigen SparseQR/COLAMD; the two agree to rounding (parity target 1e-6).
//
// Sampling reproduces Trajectory::evaluateRange (src/trajectory.cpp:81-141) exactly:
// one lane runs the sequential `acc += dt` / segment roll-over recurrence (so sample
// times and counts are bit-identical), and the wavefront evaluates the rows.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cached_ws.h"
#include "epp_internal.h"
#include "minsnap_consts.h"
#include "small_body.h"

namespace epp {
namespace {

constexpr int N = 10;
constexpr int HALF = 5;
constexpr int kWave = 64;

// The kernels' constants, one block (kNC doubles, set once per device by ensure_consts and
// staged into LDS at kernel entry, overlapping the inputs' loads — lane-indexed reads of
// __constant__ memory are vector loads that miss the caches on the latency path):
//   kCB   falling factorials B[k][j] = j! / (j-k)!  (src/polynomial.cpp:145-160), 10 x 10
//   kCB5  B5^-1, kCK  K (the closed-form mapping inverse, ainv_entry), 5 x 5 each
//   kCF   1 / r!, r = 0..4
//   kCH   Hc, the constant part of H = A^-T Q A^-1 (hessian_const below), 10 x 10
constexpr int kCB = 0, kCB5 = 100, kCK = 125, kCF = 150, kCH = 156, kNC = 256;  // (kNC even: 16-byte aligned LDS after it)
__constant__ double cC[kNC];
template <int BLOCK>
__device__ __forceinline__ void stage_consts(double* dst) {
    for (int e = threadIdx.x; e < kNC; e += BLOCK) dst[e] = cC[e];
}

// Phase timeline of the fused refit (diagnostics builds only: -DEPP_REFIT_TL, see
// scripts/refit_timeline.py): thread 0 of each workgroup stamps s_memrealtime (100 MHz).
#ifdef EPP_REFIT_TL
__device__ unsigned long long g_refit_tl[2][16];
#define EPP_TL(k)                                                                         \
    do {                                                                                  \
        if (threadIdx.x == 0) g_refit_tl[blockIdx.x & 1][k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// (per-iteration shader clocks of the block solve's forward / backward loops)
__device__ unsigned long long g_refit_it[2][64];
#define EPP_TLI(k)                                                                           \
    do {                                                                                     \
        if (threadIdx.x == 0 && (k) < 64) g_refit_it[blockIdx.x & 1][k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// (slots 14, 15: the shader clock, s_memtime, around the block solve)
#define EPP_TLC(k)                                                                        \
    do {                                                                                  \
        if (threadIdx.x == 0) g_refit_tl[blockIdx.x & 1][k] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define EPP_TLC(k) \
    do {           \
    } while (0)
#define EPP_TLI(k) \
    do {           \
    } while (0)
#define EPP_TL(k) \
    do {          \
    } while (0)
#endif

__host__ __device__ __forceinline__ double nfabian(const double* p, const double* q, double vmax,
                                          double amax) {
    // estimateSegmentTimesNfabian — src/vertex.cpp:272-289 (magic 6.5)
    const double d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
    const double distance = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    return distance / vmax * 2 * (1.0 + 6.5 * vmax / amax * exp(-distance / vmax * 2));
}

// Reciprocal square root: the hardware estimate (v_rsq_f64: ~5e-8 relative error,
// measured) refined by two Newton steps to ~1e-16, in 6 dependent instructions instead of
// the ~10-20 of an IEEE square root and division.
__device__ __forceinline__ double rsq_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = fma(0.5 * y, fma(-(x * y), y, 1.0), y);
    return fma(0.5 * y, fma(-(x * y), y, 1.0), y);
}

// Workgroup barrier.  SCR_LDS (all the solve's shared data in LDS): waits for this
// wave's LDS operations only, so global loads issued earlier (e.g. the refit's host
// reads of its sample data) stay in flight across it; else a full __syncthreads.
template <bool SCR_LDS>
__device__ __forceinline__ void block_sync() {
    if (SCR_LDS) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else __syncthreads();
}

// Orders one wavefront's LDS accesses across its lanes (LDS operations of a wavefront
// complete in order; this waits for them and stops the compiler moving memory accesses
// across the point).
__device__ __forceinline__ void wave_sync_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


// setupMappingMatrix + invertMappingMatrix (impl :111-121, :142-179) in closed form.  The
// mapping matrix is A = [[diag(k!), 0], [C, D]] with C[k][j] = B[k][j] T^(j-k) and
// D[k][j] = B[k][j+5] T^(j+5-k), i.e. D = diag(T^-k) B5 diag(T^(j+5)) for the constant
// B5[k][j] = B[k][j+5].  So
//   A^-1 = [[diag(1/k!), 0], [-D^-1 C diag(1/k!), D^-1]],
//   D^-1[r][c] = B5^-1[r][c] T^(c-r-5),   (-D^-1 C diag(1/k!))[r][c] = K[r][c] T^(c-r-5)
// with constant B5^-1 and K[r][c] = -sum_{k<=c} B5^-1[r][k] B[k][c] / c!: every entry is
// a constant times a power of 1/T, so the 100 entries are independent (one thread each)
// instead of a 5x5 LU per segment on one lane.  The reference's LU with partial pivoting
// gives the same matrix to rounding (the parity target of the solve is 1e-6).
// ipow: (1/T)^0..(1/T)^9
__device__ __forceinline__ double ainv_entry(const double* kc, const double* ipow, int r, int c) {
    if (r < HALF) return r == c ? kc[kCF + r] : 0.0;
    const int rr = r - HALF;
    const int ex = (c < HALF ? c : c - HALF) - rr - HALF;  // in [-9, -1]
    return (c < HALF ? kc[kCK + rr * HALF + c] : kc[kCB5 + rr * HALF + c - HALF]) * ipow[-ex];
}

// H_i = A_i^-T Q_i A_i^-1 in closed form.  Row a >= 4 of A^-1 is a constant times
// T^(c%5 - a) in column c (ainv_entry), and Q[a][b] (a, b >= 4) a constant times
// T^(a+b-7) (computeQuadraticCostJacobian, impl :567-583), so every term of
//   H[r][c] = sum_{a,b >= 4} A^-1[a][r] Q[a][b] A^-1[b][c]
// carries the same power T^((r%5) + (c%5) - 7): H[r][c] = Hc[r][c] T^((r%5) + (c%5) - 7)
// with the constant Hc (computed once on the host in long double, kCH).  The solve
// reads the H entries it needs straight from Hc and the powers of T: no per-segment
// A^-1 / Q / G / H products and none of their barriers.
// Per-segment scratch (doubles): the R_pp blocks -- W (coupling to the next inner vertex,
// then G = S^-1 E of the block solve) and L (diagonal block) -- and the powers of T.
struct Seg {
    static constexpr int kW = 0, kL = 16, kPow = 32, kX = 44, kSize = 56;  // kX: refinement's saved x (12)
};
// kPow: (1/T)^0..(1/T)^9 (A^-1's and H's negative powers) then T (H's one positive power)
constexpr int kNPow = 11;
__device__ __forceinline__ double seg_pow(const double* pw, int e) { return e > 0 ? pw[10] : pw[-e]; }  // T^e, e in [-9, 1]
__device__ __forceinline__ double hess(const double* kc, const double* pw, int r, int c) {
    return kc[kCH + r * 10 + c] * seg_pow(pw, (r % 5) + (c % 5) - 7);
}
// Per track, besides the segment scratch: (M+1) x 5 x 3 vertex values, (M+1) x 4 x 3
// right-hand sides, M segment times and the block solve's lane exchange (kXch, in LDS).
constexpr int kXch = 144;
__host__ __device__ constexpr size_t vertex_doubles(int M) { return (size_t)(M + 1) * 27 + (size_t)M + kXch; }
// Tracks with up to this many segments keep the segment scratch in LDS (~114 KB at 40).
constexpr int kMaxLdsSeg = 40;

// The min-snap solve of one track by one workgroup of BLOCK threads (every thread calls
// it; it contains barriers).  kc: the constants (LDS).  P: W x 3 waypoints; v0/a0: the start vertex's velocity and
// acceleration (NULL = 0); times_in: caller segment times (NULL = Nfabian).  scr: M x
// Seg::kSize, dv/rhs/Tm/xch: vertex_doubles(M) (LDS).  *s_err must be 0 and
// visible to every thread on entry.  Writes T_out (M, may be NULL) and C_out (M x 3 x 10,
// increasing powers).  Returns 0, -2 (a segment time <= 0: the reference's
// CHECK_GT(segment_time, 0), impl :297) or -3 (R_pp not SPD).
template <int BLOCK, bool SCR_LDS>
__device__ __forceinline__ int solve_track(const double* __restrict__ kc, const double* __restrict__ P, int M, double vmax, double amax,
                                           const double* v0, const double* a0, const double* times_in,
                                           double* scr, double* dv, double* rhs, double* Tm, double* xch,
                                           int* s_err, double* T_out, double* C_out, bool refine) {
    const int tid = threadIdx.x;
    // ---- phase 1: segment times, powers of T, fixed vertex values ---------------
    // (one barrier: every thread of a segment's powers takes its time itself -- the
    // caller's, or Nfabian of the same two waypoints, the same arithmetic each time)
    for (int e = tid; e < M * kNPow; e += BLOCK) {  // (1/T)^k, k = 0..9, and T
        const int i = e / kNPow, k = e % kNPow;
        const double T = times_in ? times_in[i] : nfabian(P + 3 * i, P + 3 * (i + 1), vmax, amax);
        if (k == 0) {
            Tm[i] = T;
            if (T_out) T_out[i] = T;
            if (!(T > 0)) atomicOr(s_err, 1);  // CHECK_GT(segment_time, 0)  impl :297
        }
        // 1/T: the hardware reciprocal refined by two Newton steps (~1e-16; a division
        // would cost ~10 dependent instructions)
        double it = __builtin_amdgcn_rcp(T);
        it = fma(it, fma(-T, it, 1.0), it);
        it = fma(it, fma(-T, it, 1.0), it);
        double p = k == 10 ? T : 1.0;
        for (int q = 0; q < k && k < 10; ++q) p = p * it;
        scr[(size_t)i * Seg::kSize + Seg::kPow + k] = p;
    }
    // start vertex {p0, v0, a0, 0, 0}, inner {p}, end {p, 0, 0, 0, 0}: makeStartOrEnd
    // (src/vertex.cpp:146-170) and trajectory_generator.cpp:28-50
    for (int e = tid; e < (M + 1) * 15; e += BLOCK) {
        const int v = e / 15, k = (e % 15) / 3, d = e % 3;
        double val = 0.0;  // free values are overwritten by the solve
        if (k == 0) val = P[3 * v + d];
        else if (v == 0 && k == 1) val = v0 ? v0[d] : 0.0;
        else if (v == 0 && k == 2) val = a0 ? a0[d] : 0.0;
        dv[e] = val;
    }
    block_sync<SCR_LDS>();
    EPP_TL(1);
    if (*s_err) return -2;
    // ---- phase 2: block-tridiagonal system over the inner vertices ----------------
    // free variable (v, p): vertex v in 1..M-1, derivative p+1.  Diagonal block D_v is
    // kept in the L slot of segment v-1, the coupling E_v (v -> v+1) in the W slot.
    // Segment i's H (closed form, hess) couples vertex i (rows 0..4) and i+1 (rows 5..9).
    const int nin = M - 1;
    auto build_blocks = [&]() {
        for (int e = tid; e < nin * 16; e += BLOCK) {
            const int v = 1 + e / 16, p = (e % 16) / 4, q = e % 4;
            const double* pm = scr + (size_t)(v - 1) * Seg::kSize + Seg::kPow;
            const double* pp = scr + (size_t)v * Seg::kSize + Seg::kPow;
            scr[(size_t)(v - 1) * Seg::kSize + Seg::kL + p * 4 + q] = hess(kc, pm, 6 + p, 6 + q) + hess(kc, pp, 1 + p, 1 + q);
            scr[(size_t)(v - 1) * Seg::kSize + Seg::kW + p * 4 + q] = (v < nin) ? hess(kc, pp, 1 + p, 6 + q) : 0.0;
        }
    };
    // b = -R_pf d_f, entry (v, p+1, d).  The two position columns of a segment enter as one
    // difference: H x u = 0 for u = e_0 + e_5 (moving both ends' positions together moves the
    // polynomial without changing its snap), so H[r][0] p_a + H[r][5] p_b = H[r][0] (p_a - p_b)
    // -- the same value without the cancellation of two large terms when the positions are
    // large next to their difference (hess(., 5) := -hess(., 0)).
    auto rhs_entry = [&](int v, int p, int d) -> double {
        double s = 0.0;
        // segment v-1: rows 0..4 = vertex v-1, rows 5..9 = vertex v; row of (v,p+1) = 6+p
        {
            const double* pw = scr + (size_t)(v - 1) * Seg::kSize + Seg::kPow;
            s = hess(kc, pw, 6 + p, 0) * (dv[((v - 1) * HALF) * 3 + d] - dv[(v * HALF) * 3 + d]);
            for (int r = 1; r < N; ++r) {
                const int vv = (r < HALF) ? v - 1 : v, k = r % HALF;
                if (k != 0 && (vv == 0 || vv == M)) s = s + hess(kc, pw, 6 + p, r) * dv[(vv * HALF + k) * 3 + d];
            }
        }
        // segment v: rows 0..4 = vertex v (row of (v,p+1) = 1+p), rows 5..9 = vertex v+1
        {
            const double* pw = scr + (size_t)v * Seg::kSize + Seg::kPow;
            s = s + hess(kc, pw, 1 + p, 0) * (dv[(v * HALF) * 3 + d] - dv[((v + 1) * HALF) * 3 + d]);
            for (int r = 1; r < N; ++r) {
                const int vv = (r < HALF) ? v : v + 1, k = r % HALF;
                if (k != 0 && (vv == 0 || vv == M)) s = s + hess(kc, pw, 1 + p, r) * dv[(vv * HALF + k) * 3 + d];
            }
        }
        return -s;
    };
    build_blocks();
    for (int e = tid; e < nin * 12; e += BLOCK) {
        const int v = 1 + e / 12, p = (e % 12) / 3, d = e % 3;
        rhs[(v * 4 + p) * 3 + d] = rhs_entry(v, p, d);
    }
    block_sync<SCR_LDS>();
    EPP_TL(5);
    EPP_TLC(14);
    // ---- phase 3: block-tridiagonal solve (twisted block Thomas, lanes over the block entries)
    // Inner vertices v = 1..nin, diagonal blocks D_v, couplings E_v (v -> v+1), right-hand
    // sides b_v (3 columns).  Two eliminations run at once and meet at m = (nin+1)/2:
    //   top    (v = 1..m-1): S_1 = D_1, y_1 = b_1;  G_v = S_v^-1 E_v, g_v = S_v^-1 y_v;
    //                        S_{v+1} = D_{v+1} - E_v^T G_v,  y_{v+1} = b_{v+1} - E_v^T g_v
    //   bottom (v = nin..m+1): T_nin = D_nin, z_nin = b_nin;  H_v = T_v^-1 E_{v-1}^T,
    //                        h_v = T_v^-1 z_v;  T_{v-1} = D_{v-1} - E_{v-1} H_v, z likewise
    //   middle: x_m = (D_m - E_{m-1}^T G_{m-1} - E_m H_{m+1})^-1 (b_m - ...) -- the full Schur
    //           complement of vertex m: the top's S_m minus the bottom's correction
    //   back:   x_v = g_v - G_v x_{v+1} (v = m-1..1) and x_v = h_v - H_v x_{v-1} (v = m+1..nin),
    //           both directions at once.
    // The same elimination as one sweep from the top, in about half the dependent steps
    // (11 inner vertices: 5 + 1 + 5 instead of 11 + 11).  Lanes 0..27 run the top, lanes
    // 32..59 the bottom (the same instructions: the bottom reads its coupling transposed).
    // In a group, lane L owns one entry: L < 16 the 4x4 block entry (L>>2, L&3), 16..27
    // the 4x3 right-hand-side entry ((L-16)/3, (L-16)%3).  A step is two LDS-exchanged
    // stages: (1) adj(S) (one cofactor per lane); (2) every lane reads all of adj(S) and
    // forms the column t = adj(S) X of its own right-hand side X (coupling column for block
    // lanes, y column for rhs lanes) while det(S) and its reciprocal are computed beside
    // it; its entry of [G g] = t / det (kept for the back substitution) and of
    // [S' y'] = [D b] - E^T t / det (the next step's S, exchanged) follow without another
    // exchange.  S^-1 = adj(S) / det(S): no pivots or square roots; the Schur complements
    // of an SPD R_pp are SPD (det > 0), and the explicit inverse is within ~cond(S) ulp of
    // a factorisation's answer (parity target 1e-6).  Every value a step needs that does
    // not depend on the chain (the coupling, the next D / b entry) is loaded at its start.
    // G_v / H_v are kept in segment v-1's L slot (D_v is consumed by then), g_v / h_v in
    // rhs[v].  xch: per group (base 48 g) S|y [0,28), adj(S) [28,44); x buffers
    // [96 + 24 g, +24).
    auto block_solve = [&]() {
    if (tid < kWave && nin > 0) {
        const int L = tid & 31, grp = tid >> 5;
        const bool mat = L < 16, act = L < 28;
        const int row = mat ? (L >> 2) : (L - 16) / 3;  // block row (S, G) or rhs row (y, g)
        const int col = mat ? (L & 3) : (L - 16) % 3;
        const int ycol = mat ? 0 : col;                   // (block lanes read a dummy y column)
        const bool diag = mat && (L % 5) == 0;            // S[i][i]: must stay > 0 (SPD)
        const int m = (nin + 1) / 2;
        const int nstep = nin - m;                        // the bottom's steps (the top's: m - 1 <= nstep)
        const int gsteps = grp == 0 ? m - 1 : nin - m;
        double* xg = xch + 48 * grp;
        const int vs = grp == 0 ? 1 : nin;
        double cur = act ? (mat ? scr[(size_t)(vs - 1) * Seg::kSize + Seg::kL + L] : rhs[(size_t)vs * 12 + (L - 16)])
                         : 1.0;  // this lane's S / y entry
        if (act) xg[L] = cur;
        bool ok = !act || !diag || cur > 0.0;
        // the cofactor this lane computes: adj(S)[ar][ac] = (-1)^(ar+ac) det(S minus row ac, col ar)
        const int ar = (L >> 2) & 3, ac = L & 3;
        const int r0 = ac == 0 ? 1 : 0, r1 = ac <= 1 ? 2 : 1, r2 = ac <= 2 ? 3 : 2;
        const int c0 = ar == 0 ? 1 : 0, c1 = ar <= 1 ? 2 : 1, c2 = ar <= 2 ? 3 : 2;
        const double sgn = ((ar + ac) & 1) ? -1.0 : 1.0;
        // one elimination step on S|y in xg with coupling rows Ep (E^T row `row`) and
        // columns Ec (block lanes' X); returns t (4) and 1/det; ok updated
        auto step_core = [&](const double (&Ec)[4], double (&t)[4], double& id, bool live) {
            const double a = xg[r0 * 4 + c0], b = xg[r0 * 4 + c1], c = xg[r0 * 4 + c2];
            const double d = xg[r1 * 4 + c0], e = xg[r1 * 4 + c1], f = xg[r1 * 4 + c2];
            const double g = xg[r2 * 4 + c0], h = xg[r2 * 4 + c1], i = xg[r2 * 4 + c2];
            double s0[4], yc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s0[k] = xg[k];
                yc[k] = xg[16 + k * 3 + ycol];
            }
            const double m0 = fma(e, i, -(f * h)), m1 = fma(d, i, -(f * g)), m2 = fma(d, h, -(e * g));
            const double cof = sgn * fma(c, m2, fma(a, m0, -(b * m1)));
            if (mat && live) xg[28 + L] = cof;
            wave_sync_lds();
            double adj[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) adj[k] = xg[28 + k];
            const double det = fma(s0[0], adj[0], s0[1] * adj[4]) + fma(s0[2], adj[8], s0[3] * adj[12]);
            id = __builtin_amdgcn_rcp(det);  // refined by two Newton steps
            id = fma(id, fma(-det, id, 1.0), id);
            id = fma(id, fma(-det, id, 1.0), id);
            ok = ok && (!live || det > 0.0);
            double X[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) X[k] = mat ? Ec[k] : yc[k];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                t[k] = fma(adj[4 * k], X[0], adj[4 * k + 1] * X[1]) + fma(adj[4 * k + 2], X[2], adj[4 * k + 3] * X[3]);
        };
        wave_sync_lds();
        for (int s = 0; s < nstep; ++s) {
            EPP_TLI(1 + s);
            const bool live = s < gsteps;
            const int v = grp == 0 ? 1 + s : nin - s;
            const int vn = grp == 0 ? v + 1 : v - 1;  // the next vertex of this sweep
            // coupling: top E_v (segment v-1's W slot, E[k][q] at 4k + q), bottom E_{v-1}
            // transposed (segment v-2's W slot); E^T row `row`, and column `col`
            const double* Eb = scr + (size_t)(grp == 0 ? v - 1 : max(v - 2, 0)) * Seg::kSize + Seg::kW;
            double Ep[4], Ec[4], nxt = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                Ep[k] = grp == 0 ? Eb[k * 4 + (row & 3)] : Eb[(row & 3) * 4 + k];
                Ec[k] = grp == 0 ? Eb[k * 4 + (col & 3)] : Eb[(col & 3) * 4 + k];
            }
            if (live && act) nxt = mat ? scr[(size_t)(vn - 1) * Seg::kSize + Seg::kL + L] : rhs[(size_t)vn * 12 + (L - 16)];
            double t[4], id;
            step_core(Ec, t, id, live);
            const double tr = row == 0 ? t[0] : row == 1 ? t[1] : row == 2 ? t[2] : t[3];
            const double et = fma(Ep[0], t[0], Ep[1] * t[1]) + fma(Ep[2], t[2], Ep[3] * t[3]);
            if (live && act) {
                if (mat) scr[(size_t)(v - 1) * Seg::kSize + Seg::kL + L] = tr * id;  // G_v / H_v
                else rhs[(size_t)v * 12 + (L - 16)] = tr * id;                       // g_v / h_v
                const double corr = et * id;
                cur = nxt - corr;  // [S' y'] = [D b] - E^T t / det
                // (the bottom's last step publishes its correction instead: the middle block
                // is the top's S_m minus it)
                xg[L] = (grp == 1 && s == nstep - 1) ? corr : cur;
                ok = ok && (!diag || cur > 0.0);
            }
            wave_sync_lds();
        }
        // middle: the top's S_m | y_m minus the bottom's last correction
        if (grp == 0 && act) {
            cur = cur - (nstep > 0 ? xch[48 + L] : 0.0);
            xg[L] = cur;
            ok = ok && (!diag || cur > 0.0);
        }
        wave_sync_lds();
        {
            const double Ec0[4] = {0.0, 0.0, 0.0, 0.0};
            double t[4], id;
            step_core(Ec0, t, id, grp == 0);
            const double tr = row == 0 ? t[0] : row == 1 ? t[1] : row == 2 ? t[2] : t[3];
            if (grp == 0 && act && !mat) {  // x_m = (middle block)^-1 (middle rhs)
                const double x = tr * id;
                rhs[(size_t)m * 12 + (L - 16)] = x;
                dv[((size_t)m * HALF + 1) * 3 + (L - 16)] = x;  // derivatives 1..4 of vertex m
                xch[96 + (L - 16)] = x;
                xch[96 + 24 + (L - 16)] = x;
            }
        }
        // (the G/g stores, LDS or, for long tracks, global scratch: a workgroup-scope fence
        // makes the latter visible to the wave's own later loads)
        if (!SCR_LDS) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        wave_sync_lds();
        if (__ballot(!ok) == 0ull) {  // wave-uniform
            EPP_TLI(32);
            // lanes 0..11 of each group: x_v entry (p, d) = (L/3, L%3); the next step's G / H
            // row and g / h entry are loaded before this step's exchange completes
            const int p = (L / 3) & 3, d = L % 3;
            const int Lr = L < 12 ? L : 0;
            const int bsteps = grp == 0 ? m - 1 : nin - m;
            double* xb = xch + 96 + 24 * grp;
            int buf = 0;
            double Gr[4] = {0.0, 0.0, 0.0, 0.0}, gx = 0.0;
            auto load_step = [&](int v, double (&G)[4], double& gg) {
                const double* Gp = scr + (size_t)(v - 1) * Seg::kSize + Seg::kL + p * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) G[k] = Gp[k];
                gg = rhs[(size_t)v * 12 + Lr];
            };
            if (bsteps > 0) load_step(grp == 0 ? m - 1 : m + 1, Gr, gx);
            for (int s = 0; s < nstep; ++s) {
                EPP_TLI(33 + s);
                const bool live = s < bsteps;
                const int v = grp == 0 ? m - 1 - s : m + 1 + s;
                double Gn[4] = {0.0, 0.0, 0.0, 0.0}, gn = 0.0;
                if (s + 1 < bsteps) load_step(grp == 0 ? v - 1 : v + 1, Gn, gn);
                const double* xn = xb + buf * 12;
                const double x = gx - (fma(Gr[0], xn[d], Gr[1] * xn[3 + d]) + fma(Gr[2], xn[6 + d], Gr[3] * xn[9 + d]));
                if (live && L < 12) {
                    xb[(buf ^ 1) * 12 + L] = x;
                    dv[((size_t)v * HALF + 1) * 3 + L] = x;  // derivatives 1..4 of vertex v
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) Gr[k] = Gn[k];
                gx = gn;
                buf ^= 1;
                wave_sync_lds();
            }
        } else if (tid == 0) {
            *s_err = 1;
        }
        EPP_TLI(63);
    }
    };
    block_solve();
    block_sync<SCR_LDS>();
    EPP_TL(6);
    EPP_TLC(15);
    if (*s_err) return -3;
    // ---- one step of iterative refinement (refine): r = b - R_pp x (the closed-form blocks
    // again: the solve consumed the L slots), R_pp dx = r by the same elimination, x += dx.
    // The elimination's rounding is amplified by R_pp's condition (up to ~1e12 next to very
    // short segments); one step brings the solution to the accuracy of the data.
    if (refine && nin > 0) {
        for (int e = tid; e < nin * 12; e += BLOCK) {
            const int v = 1 + e / 12, p = (e % 12) / 3, d = e % 3;
            const double* pm = scr + (size_t)(v - 1) * Seg::kSize + Seg::kPow;  // segment v-1
            const double* pp = scr + (size_t)v * Seg::kSize + Seg::kPow;        // segment v
            double r = rhs_entry(v, p, d);
            for (int q = 0; q < 4; ++q) {
                r = r - (hess(kc, pm, 6 + p, 6 + q) + hess(kc, pp, 1 + p, 1 + q)) * dv[(v * HALF + 1 + q) * 3 + d];
                if (v < nin) r = r - hess(kc, pp, 1 + p, 6 + q) * dv[((v + 1) * HALF + 1 + q) * 3 + d];
                if (v > 1) r = r - hess(kc, pm, 1 + q, 6 + p) * dv[((v - 1) * HALF + 1 + q) * 3 + d];
            }
            rhs[(v * 4 + p) * 3 + d] = r;
        }
        block_sync<SCR_LDS>();
        for (int e = tid; e < nin * 12; e += BLOCK) {  // x kept in the segments' X slots
            const int v = 1 + e / 12, p = (e % 12) / 3, d = e % 3;
            scr[(size_t)(v - 1) * Seg::kSize + Seg::kX + p * 3 + d] = dv[(v * HALF + 1 + p) * 3 + d];
        }
        build_blocks();
        block_sync<SCR_LDS>();
        block_solve();
        block_sync<SCR_LDS>();
        if (*s_err) return -3;
        for (int e = tid; e < nin * 12; e += BLOCK) {
            const int v = 1 + e / 12, p = (e % 12) / 3, d = e % 3;
            double& x = dv[(v * HALF + 1 + p) * 3 + d];
            x = scr[(size_t)(v - 1) * Seg::kSize + Seg::kX + p * 3 + d] + x;
        }
        block_sync<SCR_LDS>();
    }
    // ---- phase 4: p_i = A_i^-1 [d_i ; d_{i+1}] -------------------------------------
    for (int e = tid; e < M * 30; e += BLOCK) {
        const int i = e / 30, d = (e % 30) / 10, r = e % 10;
        const double* ipow = scr + (size_t)i * Seg::kSize + Seg::kPow;
        const double* d0 = dv + (size_t)i * HALF * 3 + d;  // vertex i's values, then vertex i+1's
        double s;
        if (r < HALF) {  // rows 0..4 of A^-1: diag(1 / r!)
            s = kc[kCF + r] * d0[3 * r];
        } else {  // rows 5..9: [K | B5^-1] row rr, column c scaled by (1/T)^(rr + 5 - c % 5)
            // (the two positions as one difference: K[rr][0] = -B5^-1[rr][0], A^-1 maps equal
            // end positions to a constant polynomial)
            const int rr = r - HALF;
            s = kc[kCK + rr * HALF] * ipow[rr + HALF] * (d0[0] - d0[3 * HALF]);
#pragma unroll
            for (int k = 1; k < N; ++k) {
                if (k == HALF) continue;
                const double a = (k < HALF ? kc[kCK + rr * HALF + k] : kc[kCB5 + rr * HALF + k - HALF]) *
                                 ipow[rr + HALF - k % HALF];
                s = s + a * d0[3 * k];
            }
        }
        C_out[((size_t)i * 3 + d) * N + r] = s;
    }
    return 0;
}

// Batch: one workgroup (BLOCK threads) per track.  Track k owns waypoints
// [wp_off[k], wp_off[k+1]) and segments [wp_off[k]-k, wp_off[k+1]-k-1).  LDS: the segment
// scratch (when LDS) and the vertex values; else the segment scratch lives in gscratch
// at the track's first segment (Σ M x Seg::kSize doubles).
template <int BLOCK, bool LDS>
__global__ __launch_bounds__(BLOCK) void k_minsnap(const double* __restrict__ wp, const int32_t* __restrict__ wp_off,
                                                   int n_tracks, double vmax, double amax, const double* __restrict__ v0,
                                                   const double* __restrict__ a0, const double* __restrict__ times_in,
                                                   double* __restrict__ seg_times, double* __restrict__ coeffs,
                                                   int32_t* __restrict__ status, double* __restrict__ gscratch,
                                                   int refine) {
    // one dynamic LDS array (cdna_hip_programming.md Guideline 17): the error flag (16
    // bytes), the constants, then the solve's scratch
    extern __shared__ __attribute__((aligned(16))) double smem[];
    int* s_err = reinterpret_cast<int*>(smem);
    double* kc = smem + 2;
    double* sm = kc + kNC;
    stage_consts<BLOCK>(kc);
    const int track = blockIdx.x;
    if (track >= n_tracks) return;
    const int w0 = wp_off[track];
    const int W = wp_off[track + 1] - w0;
    const int M = W - 1;
    const int seg0 = w0 - track;
    if (W < 2) {
        if (threadIdx.x == 0 && status) status[track] = -1;  // std::invalid_argument
        return;
    }
    if (threadIdx.x == 0) *s_err = 0;
    double* scr = LDS ? sm : gscratch + (size_t)seg0 * Seg::kSize;
    double* dv = LDS ? sm + (size_t)M * Seg::kSize : sm;
    double* rhs = dv + (size_t)(M + 1) * 15;
    double* Tm = rhs + (size_t)(M + 1) * 12;
    __syncthreads();
    const int st = solve_track<BLOCK, LDS>(kc, wp + (size_t)w0 * 3, M, vmax, amax, v0 ? v0 + 3 * track : nullptr,
                                      a0 ? a0 + 3 * track : nullptr, times_in ? times_in + seg0 : nullptr, scr, dv, rhs,
                                      Tm, Tm + M, s_err, seg_times + seg0, coeffs + (size_t)seg0 * 30, refine != 0);
    if (threadIdx.x == 0 && status) status[track] = st;
}

constexpr int kRowChunk = 512;  // samples per k_sample_rows round

// Trajectory::evaluateRange control flow — src/trajectory.cpp:81-141.
struct RangeIter {
    const double* T;
    int M, i;
    double t_end, acc, tis, Ti;  // Ti = T[i], kept in a register (one LDS read per segment)
    __host__ __device__ void init(const double* T_, int M_) {
        T = T_;
        M = M_;
        t_end = 0.0;  // max_time_ += segment.getTime()  trajectory.h:63-70
        for (int k = 0; k < M; ++k) t_end = t_end + T[k];
        acc = 0.0;
        for (i = 0; i < M; ++i) {  // t_start = 0
            acc = acc + T[i];
            if (acc > 0.0) break;
        }
        if (i >= M) i = M - 1;
        acc = acc - T[i];
        tis = 0.0 - acc;
        Ti = T[i];
    }
    // Advances to the next sample; returns false when the loop ends.
    __host__ __device__ bool next(int& seg, double& t_in, double& t_acc) {
        while (acc < t_end) {
            if (tis > Ti) {
                tis = tis - Ti;
                i++;
                if (i >= M) return false;
                Ti = T[i];
                continue;
            }
            seg = i;
            t_in = tis;
            t_acc = acc;
            return true;
        }
        return false;
    }
    __host__ __device__ void advance(double dt) {
        tis = tis + dt;
        acc = acc + dt;
    }
    // The next 8 samples at once when none of them rolls over into the next segment or
    // reaches the end (the same additions, in the same order, as 8 next/advance steps;
    // acc and tis only grow, so checking the 8th sample covers all).  False: nothing
    // consumed, take single steps.
    __device__ bool fast8(double dt, double (&tin)[8], double (&tac)[8]) {
        double t = tis, a = acc;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            tin[k] = t;
            tac[k] = a;
            t = t + dt;
            a = a + dt;
        }
        if (!(tac[7] < t_end) || tin[7] > Ti) return false;
        tis = t;
        acc = a;
        return true;
    }
};

// One wavefront per track: the lanes stage the segment times in LDS, lane 0 runs the
// recurrence (every step reads T[i] from LDS, not from memory).
__global__ __launch_bounds__(kWave) void k_sample_count(const double* __restrict__ seg_times,
                                                        const int32_t* __restrict__ wp_off,
                                                        int n_tracks, double dt,
                                                        int64_t* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) double sT[];
    const int t = blockIdx.x;
    if (t >= n_tracks) return;
    const int M = wp_off[t + 1] - wp_off[t] - 1;
    if (M < 1 || !(dt > 0)) {
        if (threadIdx.x == 0) counts[t] = 0;
        return;
    }
    const double* T = seg_times + (wp_off[t] - t);
    for (int i = threadIdx.x; i < M; i += kWave) sT[i] = T[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        RangeIter it;
        it.init(sT, M);
        int64_t n = 0;
        int seg;
        double tin, tac, tin8[8], tac8[8];
        for (;;) {
            if (it.fast8(dt, tin8, tac8)) {
                n += 8;
                continue;
            }
            if (!it.next(seg, tin, tac)) break;
            ++n;
            it.advance(dt);
        }
        counts[t] = n;
    }
}

// Polynomial::evaluate(t, k) — polynomial.h:136-149
// (Horner with fused multiply-adds: the sampled values are compared at 1e-6, the time
// column, which does not go through here, exactly)
__device__ __forceinline__ double poly_eval(const double* B, const double* c, double t, int k) {
    double r = B[k * N + N - 1] * c[N - 1];
    for (int j = N - 2; j >= k; --j) r = fma(r, t, B[k * N + j] * c[j]);
    return r;
}

__global__ __launch_bounds__(kWave) void k_sample_rows(const double* __restrict__ seg_times,
                                                       const double* __restrict__ coeffs,
                                                       const int32_t* __restrict__ wp_off,
                                                       int n_tracks, double dt,
                                                       const double* __restrict__ t0,
                                                       const int64_t* __restrict__ row_off,
                                                       double* __restrict__ rows, int64_t cap_rows) {
    // one dynamic LDS array (Guideline 17): [T (M) | tin | tac | seg (kRowChunk each) | cnt, done]
    // lane 0 runs the sequential time recurrence for kRowChunk samples at a time, then the
    // wave evaluates them (fewer barriers / coefficient-load round trips than 64 a round)
    extern __shared__ __attribute__((aligned(16))) double smB[];  // [B (kNC block) | ...]
    const int t = blockIdx.x;
    if (t >= n_tracks) return;
    const int lane = threadIdx.x;
    const int M = wp_off[t + 1] - wp_off[t] - 1;
    if (M < 1 || !(dt > 0)) return;
    stage_consts<kWave>(smB);
    double* sm = smB + kNC;
    const int seg0 = wp_off[t] - t;
    double* sT = sm;
    double* s_tin = sT + ((M + 1) & ~1);
    double* s_tac = s_tin + kRowChunk;
    int* s_seg = reinterpret_cast<int*>(s_tac + kRowChunk);
    int& s_cnt = s_seg[kRowChunk];
    int& s_done = s_seg[kRowChunk + 1];
    for (int i = lane; i < M; i += kWave) sT[i] = seg_times[seg0 + i];
    const double toff = t0 ? t0[t] : 0.0;
    double* out = rows + (row_off ? row_off[t] : 0) * 10;
    RangeIter it;
    __syncthreads();
    if (lane == 0) {
        it.init(sT, M);
        s_done = 0;
    }
    int64_t base = 0;
    while (true) {
        if (lane == 0) {
            int c = 0;
            int seg;
            double tin, tac, tin8[8], tac8[8];
            while (c < kRowChunk) {
                if (c + 8 <= kRowChunk && it.fast8(dt, tin8, tac8)) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        s_seg[c + k] = it.i;
                        s_tin[c + k] = tin8[k];
                        s_tac[c + k] = tac8[k];
                    }
                    c += 8;
                    continue;
                }
                if (!it.next(seg, tin, tac)) {
                    s_done = 1;
                    break;
                }
                s_seg[c] = seg;
                s_tin[c] = tin;
                s_tac[c] = tac;
                ++c;
                it.advance(dt);
            }
            s_cnt = c;
        }
        __syncthreads();
        const int cnt = s_cnt, done = s_done;
        for (int j = lane; j < cnt && base + j < cap_rows; j += kWave) {  // (cap: single-track host path)
            const double* cs = coeffs + (size_t)(seg0 + s_seg[j]) * 30;
            const double tin = s_tin[j];
            double* row = out + (base + j) * 10;
            for (int d = 0; d < 3; ++d)
                for (int k = 0; k < 3; ++k) row[3 * d + k] = poly_eval(smB + kCB, cs + d * N, tin, k);
            row[9] = s_tac[j] + toff;  // sampling_times[i] + startTimeOffset
        }
        base += cnt;
        __syncthreads();
        if (done) break;
    }
}

// ---- single-track fused refit (the 50 Hz latency path) --------------------------------
// poly_traj::generateTrajectory for one track in ONE launch, reading its inputs from and
// writing the rows to pinned host memory (no copies).  The host has already run the two
// sequential parts, which a GPU lane runs slowly (~65 ns per dependent step): the segment
// times (Nfabian with the host's libm, as the reference) and Trajectory::evaluateRange's
// `acc += dt` recurrence (sample times and segments, exact).  G workgroups each own a
// slice of the rows; every one of them solves the (small) min-snap problem itself with
// those times (solve_track — the same arithmetic, so the same coefficients) while its
// slice's sample data arrives from the host, then evaluates its rows
// (Polynomial::evaluate) and writes them to the host: G CUs writing in parallel (one CU's
// PCIe writes are slow) and no hand-off of the coefficients between workgroups.
// Completion is published in host memory (workgroup 0: the status; every workgroup: its
// slot) and polled by the host instead of synchronising the stream.
constexpr int kRefitArgW = 41;  // tracks up to this many waypoints pass wp, v0, a0, T as kernel arguments
constexpr int kRefitMaxWriters = 16;
struct RefitArgs {
    const double* in;  // host-mapped: [wp (W x 3) | v0 (3) | a0 (3) | T (M)] | t_in (R) | t (R) | segment (R, int32)
    int32_t W;
    int32_t R;         // rows
    int32_t writers;   // G (>= 1)
    uint32_t seq;      // this call's number (completion words hold it)
    double t0;         // startTimeOffset
    double* out;       // host-mapped: R x 10 rows
    int64_t* info;     // host-mapped: [status]
    uint32_t* done;    // host-mapped: the workgroups' completion slots
    double* scratch;   // device: G x segment scratch (tracks longer than kMaxLdsSeg)
    int32_t big;       // (!LDS) the vertex values, right-hand sides, times and coefficients
                       // in the global scratch too (tracks whose LDS part would not fit)
    int32_t refine;    // one step of iterative refinement in the solve (solve_track)
    double small[3 * kRefitArgW + 6 + kRefitArgW - 1];  // wp | v0 | a0 | T when W <= kRefitArgW
};
constexpr int kRefitBlock = 256;
constexpr int kRefitRowChunk = 128;  // rows per round (LDS staged)
constexpr size_t kRefitLdsMax = 150 * 1024;  // dynamic LDS of one refit workgroup (of 160 KB per CU)
__host__ __device__ inline size_t refit_in_doubles(int W, int R) {  // (+ 3: row 0 readable when R = 0)
    return (size_t)3 * W + 6 + (W - 1) + 2 * (size_t)R + ((size_t)R + 1) / 2 + 3;
}
__host__ __device__ inline size_t refit_nin_even(int W) { return ((size_t)3 * W + 6 + (W - 1) + 1) & ~size_t(1); }
// LDS doubles: flag (2) | constants | wp, v0, a0, T | solve scratch | coefficients |
// sample chunk (t_in, t, segment) | row chunk.  big: the vertex values, right-hand sides,
// times and coefficients live in the global scratch; LDS keeps the lane exchange (kXch).
__host__ __device__ inline size_t refit_lds_doubles(int M, bool lds, bool big = false) {
    return 2 + kNC + refit_nin_even(M + 1) + (lds ? (size_t)M * Seg::kSize : 0) +
           (big ? (size_t)kXch : vertex_doubles(M) + (size_t)M * 30) + (size_t)kRefitRowChunk * 3 + 2 +
           (size_t)kRefitRowChunk * 10;
}
// global scratch doubles per writer: the segment scratch, and (big) the vertex values,
// right-hand sides, times and coefficients
__host__ __device__ inline size_t refit_scr_doubles(int M, bool big) {
    return (size_t)M * Seg::kSize + (big ? vertex_doubles(M) - kXch + (size_t)M * 30 : 0);
}

template <bool LDS>
__device__ __forceinline__ void refit_body(const RefitArgs& a, int g, double* smem) {
    const int tid = threadIdx.x, W = a.W, M = W - 1, R = a.R;
    const double* h_tin = a.in + 3 * W + 6 + M;
    const double* h_tac = h_tin + R;
    const int32_t* h_seg = reinterpret_cast<const int32_t*>(h_tac + R);
    int* s_err = reinterpret_cast<int*>(smem);
    double* kc = smem + 2;
    double* P = kc + kNC;  // wp | v0 | a0 | T
    double* const after_p = P + refit_nin_even(W);  // (LDS)
    const bool big = !LDS && a.big;
    double* scr = after_p;
    double* dv = LDS ? scr + (size_t)M * Seg::kSize : scr;
    if (!LDS) {
        scr = a.scratch + (size_t)g * refit_scr_doubles(M, big);
        if (big) dv = scr + (size_t)M * Seg::kSize;
    }
    double* rhs = dv + (size_t)(M + 1) * 15;
    double* Tm = rhs + (size_t)(M + 1) * 12;
    double* xch = big ? after_p : Tm + M;  // the solve's lane exchange: always LDS
    double* C = big ? Tm + M : xch + kXch;  // coefficients (M x 3 x 10)
    double* s_tin = big ? xch + kXch : C + (size_t)M * 30;
    double* s_tac = s_tin + kRefitRowChunk;
    int32_t* s_seg = reinterpret_cast<int32_t*>(s_tac + kRefitRowChunk);
    double* rbuf = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(s_tac + 2 * kRefitRowChunk) + 15) &
                                             ~uintptr_t(15));
    const int per = (R + a.writers - 1) / a.writers;
    const int r0 = min(R, g * per), r1 = min(R, r0 + per);
    EPP_TL(0);
    // every input load in flight at once: the constants, the problem (kernel arguments or
    // host memory) and this slice's first sample chunk (host memory)
    // (unconditional loads at clamped addresses: no branches, so the stores below wait
    // with counted vmcnt for their own loads only and the host reads stay in flight)
    const int nin = 3 * W + 6 + M;
    const double* src = W <= kRefitArgW ? a.small : a.in;
    const double cv = cC[min(tid, kNC - 1)];
    double pv[(3 * kRefitArgW + 6 + kRefitArgW - 1 + kRefitBlock - 1) / kRefitBlock];
    constexpr int kPv = sizeof(pv) / sizeof(double);
#pragma unroll
    for (int q = 0; q < kPv; ++q) pv[q] = src[min(tid + q * kRefitBlock, nin - 1)];
    auto fetch = [&](int c0, int cnt) {  // sample data of rows [c0, c0 + cnt) (host reads)
        if (tid < cnt) {
            s_tin[tid] = h_tin[c0 + tid];
            s_tac[tid] = h_tac[c0 + tid];
            s_seg[tid] = h_seg[c0 + tid];
        }
    };
    // the first chunk's sample data is loaded now and kept in registers until the solve
    // is done (the host pads the input so row 0 is readable even when R = 0)
    const int cnt0 = min(kRefitRowChunk, r1 - r0);
    const int fr = r0 + min(tid, max(cnt0 - 1, 0));
    const double f_tin = h_tin[fr], f_tac = h_tac[fr];
    const int32_t f_seg = h_seg[fr];
    if (tid < kNC) kc[tid] = cv;
#pragma unroll
    for (int q = 0; q < kPv; ++q)
        if (tid + q * kRefitBlock < nin) P[tid + q * kRefitBlock] = pv[q];
    for (int e = kPv * kRefitBlock + tid; e < nin; e += kRefitBlock) P[e] = src[e];  // (long tracks)
    if (tid == 0) *s_err = 0;
    block_sync<LDS>();
    EPP_TL(8);
    const int st = solve_track<kRefitBlock, LDS>(kc, P, M, 0.0, 0.0, P + 3 * W, P + 3 * W + 3, P + 3 * W + 6, scr, dv,
                                            rhs, Tm, xch, s_err, nullptr, C, a.refine != 0);
    EPP_TL(7);
    if (tid < cnt0) {
        s_tin[tid] = f_tin;
        s_tac[tid] = f_tac;
        s_seg[tid] = f_seg;
    }
    __syncthreads();  // coefficients complete
    if (st == 0) {
        for (int c0 = r0; c0 < r1; c0 += kRefitRowChunk) {
            const int cnt = min(kRefitRowChunk, r1 - c0);
            if (c0 != r0) {
                __syncthreads();  // the previous chunk copied out
                fetch(c0, cnt);
                __syncthreads();
            }
            if (tid < cnt) {
                const double* cs = C + (size_t)s_seg[tid] * 30;
                const double tin = s_tin[tid];
                double* r = rbuf + (size_t)tid * 10;
#pragma unroll
                for (int d = 0; d < 3; ++d)
#pragma unroll
                    for (int q = 0; q < 3; ++q) r[3 * d + q] = poly_eval(kc + kCB, cs + d * N, tin, q);
                r[9] = s_tac[tid] + a.t0;  // sampling_times[i] + startTimeOffset
            }
            __syncthreads();
            // contiguous 16-byte stores: a wave writes 1 KB runs
            const double2* src2 = reinterpret_cast<const double2*>(rbuf);
            double2* dst2 = reinterpret_cast<double2*>(a.out + (size_t)c0 * 10);
            for (int q = tid; q < cnt * 5; q += kRefitBlock) dst2[q] = src2[q];
        }
    }
    EPP_TL(13);
    // completion: this slice's rows (and workgroup 0's status) are visible system-wide
    // before the slot is
    wg_stores_settled();
    if (tid == 0) {
        if (g == 0) __hip_atomic_store(a.info, (int64_t)st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.done + g, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool LDS>
__global__ __launch_bounds__(kRefitBlock) void k_refit(RefitArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    refit_body<LDS>(a, blockIdx.x, smem);
}

// ---- the C5 online step in one launch: A11 check + refit --------------------------------
// PathPlanner::checkTrajectoryValidity of the lookahead rows against the world
// (World::checkPointValidity(p, minDistance), src/World.cpp:106-128, src/PathPlanner.cpp:
// 267-280) and the refit of the moved waypoints (poly_traj::generateTrajectory) are
// independent: workgroups [0, writers) run the refit (refit_body), workgroups [writers,
// writers + check groups) the brute-force minDistance check of k_states_small
// (states_small_body, small_body.h) over the pinned points, flags into pinned memory.  Every
// workgroup publishes `seq` in its completion slot: one launch, one host poll for both.
static_assert(kRefitBlock == kSmallBlock, "one block size for both parts");
struct CheckArgs {
    const double* recs;  // OBB records (device blob or pinned host copy: SmallWorld)
    int32_t n_obb, per;
    double rg, ro, md;
    const double* xyz;   // host-mapped: n x 3
    int64_t n;
    uint8_t* valid;      // host-mapped: n flags
};

template <bool LDS>
__global__ __launch_bounds__(kRefitBlock) void k_check_refit(RefitArgs a, CheckArgs c) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    if ((int)blockIdx.x < a.writers) {  // (block-uniform)
        refit_body<LDS>(a, blockIdx.x, smem);
        return;
    }
    states_small_body<true, false>(smem, (int)blockIdx.x - a.writers, c.recs, c.n_obb, c.rg, c.ro, c.xyz, c.n, c.per, 0,
                                   c.md, c.valid, nullptr, nullptr);
    wg_stores_settled();
    if (threadIdx.x == 0) __hip_atomic_store(a.done + blockIdx.x, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

bool g_consts_ready[64];
CachedWs g_minsnap_ws[64];

epp_status ensure_consts() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev >= 0 && dev < 64 && g_consts_ready[dev]) return EPP_OK;
    double B[N][N];
    std::memset(B, 0, sizeof(B));
    for (int i = 0; i < N; ++i) B[0][i] = 1.0;
    int order = N - 1;
    for (int n = 1; n < N; ++n) {
        for (int i = N - 1 - order; i < N; ++i) B[n][i] = (order - (N - 1) + i) * B[n - 1][i];
        order--;
    }
    // B5^-1, K (the closed-form mapping inverse, ainv_entry) and Hc (see hess): exact
    // rationals rounded once to double (minsnap_consts.h, scripts/gen_minsnap_consts.py).
    // (Round 5 derived them here in long double; Hc's products cancel, and some entries
    // were ~3e-13 off -- data error the solve amplified to ~1e-9 in the coefficients.)
    double cc[kNC] = {};
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < N; ++j) cc[kCB + k * N + j] = B[k][j];
    for (int r = 0; r < HALF; ++r)
        for (int c = 0; c < HALF; ++c) {
            cc[kCB5 + r * HALF + c] = minsnap_consts::kB5inv[r * HALF + c];
            cc[kCK + r * HALF + c] = minsnap_consts::kK[r * HALF + c];
        }
    const double inv_fact[HALF] = {1.0, 1.0, 1.0 / 2.0, 1.0 / 6.0, 1.0 / 24.0};
    for (int r = 0; r < HALF; ++r) cc[kCF + r] = inv_fact[r];
    for (int i = 0; i < N * N; ++i) cc[kCH + i] = minsnap_consts::kHc[i];
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(cC), cc, sizeof(cc));
    if (e != hipSuccess) {
        set_error(std::string("epp minsnap: constants: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    if (dev >= 0 && dev < 64) g_consts_ready[dev] = true;
    return EPP_OK;
}

// The track offsets of a batch (they live on the device; the launchers need the largest
// segment count to size LDS and the total for the global scratch).
epp_status read_offsets(const int32_t* d_off, int n_tracks, hipStream_t s, const char* what, int* max_m,
                        int64_t* total_m) {
    std::vector<int32_t> off(n_tracks + 1);
    hipError_t e = hipMemcpyAsync(off.data(), d_off, off.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        set_error(std::string(what) + ": reading track offsets: " + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    int m = 1;
    int64_t tot = 0;
    for (int t = 0; t < n_tracks; ++t) {
        const int mt = off[t + 1] - off[t] - 1;
        m = std::max(m, mt);
        tot += std::max(0, mt);
    }
    *max_m = m;
    if (total_m) *total_m = tot;
    return EPP_OK;
}

epp_status minsnap_batch(const double* wp, const int32_t* wp_offsets, int32_t n_tracks, double v_max, double a_max,
                         const double* v0, const double* a0, const double* times_in, double* seg_times, double* coeffs,
                         int32_t* status, void* stream, const char* what) {
    if (n_tracks < 0 || (n_tracks > 0 && (!wp || !wp_offsets || !seg_times || !coeffs))) {
        set_error(std::string(what) + ": invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    epp_status st = ensure_consts();
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    int max_m = 0;
    int64_t total_m = 0;
    if ((st = read_offsets(wp_offsets, n_tracks, s, what, &max_m, &total_m))) return st;
    constexpr int kB = 64;  // one wavefront per track: the batch is throughput-bound
    // one refinement step in every track's solve (solve_track): +50 % kernel time, 10-100x
    // the accuracy on short and mixed segments (scripts/minsnap_truth_probe.py, DESIGN.md
    // section 4); EPP_MINSNAP_REFINE=0 skips it (A/B knob)
    static const int refine = [] {
        const char* e = std::getenv("EPP_MINSNAP_REFINE");
        return e && *e == '0' ? 0 : 1;
    }();
    if (max_m <= kMaxLdsSeg) {
        const size_t shm = ((size_t)max_m * Seg::kSize + vertex_doubles(max_m) + 2 + kNC) * sizeof(double);
        allow_lds(k_minsnap<kB, true>);
        hipLaunchKernelGGL((k_minsnap<kB, true>), dim3(n_tracks), dim3(kB), shm, s, wp, wp_offsets, n_tracks, v_max,
                           a_max, v0, a0, times_in, seg_times, coeffs, status, nullptr, refine);
        return launch_error(what);
    }
    // long tracks: segment scratch in a per-device workspace whose reuse by another stream
    // waits for this launch (CachedWs)
    int dev = 0;
    (void)hipGetDevice(&dev);
    CachedWs& ws = g_minsnap_ws[dev & 63];
    std::lock_guard<std::mutex> lk(ws.mu);
    const hipError_t e = ws.acquire(s, (size_t)std::max<int64_t>(total_m, 1) * Seg::kSize * sizeof(double));
    if (e != hipSuccess) {
        set_error(std::string(what) + ": workspace: " + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    const size_t shm = (vertex_doubles(max_m) + 2 + kNC) * sizeof(double);
    if (shm > kLdsBudget) {
        ws.release(s);
        set_error(std::string(what) + ": a track has too many waypoints for one workgroup's LDS (" +
                  std::to_string(max_m + 1) + ")");
        return EPP_ERR_UNSUPPORTED;
    }
    allow_lds(k_minsnap<kB, false>);
    hipLaunchKernelGGL((k_minsnap<kB, false>), dim3(n_tracks), dim3(kB), shm, s, wp, wp_offsets, n_tracks, v_max, a_max,
                       v0, a0, times_in, seg_times, coeffs, status, static_cast<double*>(ws.buf), refine);
    st = launch_error(what);
    ws.release(s);
    return st;
}

// Per-host-thread state of the single-track latency path: a stream, pinned host buffers
// the kernel reads / writes directly and the device segment scratch of long tracks.
struct RefitCache {
    hipStream_t s = nullptr;
    int dev = -1;
    double* h_in = nullptr;
    size_t in_cap = 0;
    char* h_out = nullptr;  // [status (8 B) | pad | writer slots (64 B) | rows (at +128)]
    size_t out_cap = 0;
    double* d_scr = nullptr;  // segment scratch (one per workgroup) of long tracks
    size_t scr_cap = 0;
    uint32_t seq = 0;
    std::vector<double> T, tin, tac;  // host side of the refit: times and samples
    std::vector<int32_t> seg;
    void release() {
        if (s) (void)hipStreamSynchronize(s);
        if (h_in) (void)hipHostFree(h_in);
        if (h_out) (void)hipHostFree(h_out);
        if (d_scr) (void)hipFree(d_scr);
        if (s) (void)hipStreamDestroy(s);
        h_in = nullptr;
        h_out = nullptr;
        d_scr = nullptr;
        s = nullptr;
        in_cap = out_cap = scr_cap = 0;
        seq = 0;
    }
    ~RefitCache() { release(); }
    epp_status ensure(size_t in_b, size_t out_b, size_t scr_b) {
        int d = 0;
        (void)hipGetDevice(&d);
        if (d != dev) release();  // bound to another device: start over
        dev = d;
        hipError_t e = hipSuccess;
        if (!s) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        auto grow_host = [&](auto*& p, size_t& cap, size_t need) {
            if (e != hipSuccess || need <= cap) return;
            if (s) (void)hipStreamSynchronize(s);  // (the previous call's kernel has ended)
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            e = hipHostMalloc(reinterpret_cast<void**>(&p), need, hipHostMallocDefault);
            if (e == hipSuccess) cap = need;
        };
        grow_host(h_in, in_cap, in_b);
        grow_host(h_out, out_cap, out_b);
        if (e == hipSuccess && scr_b > scr_cap) {
            (void)hipStreamSynchronize(s);
            if (d_scr) (void)hipFree(d_scr);
            d_scr = nullptr;
            scr_cap = 0;
            e = hipMalloc(reinterpret_cast<void**>(&d_scr), scr_b);
            if (e == hipSuccess) scr_cap = scr_b;
        }
        if (e != hipSuccess) {
            set_error(std::string("generateTrajectory: buffers: ") + hipGetErrorString(e));
            return EPP_ERR_HIP;
        }
        return EPP_OK;
    }
};

}  // namespace
}  // namespace epp

using namespace epp;

extern "C" {

epp_status epp_minsnap_batch(const double* wp, const int32_t* wp_offsets, int32_t n_tracks, double v_max,
                             double a_max, const double* v0, const double* a0, double* seg_times, double* coeffs,
                             int32_t* status, void* stream) {
    return minsnap_batch(wp, wp_offsets, n_tracks, v_max, a_max, v0, a0, nullptr, seg_times, coeffs, status, stream,
                         "epp_minsnap_batch");
}

epp_status epp_minsnap_batch_times(const double* wp, const int32_t* wp_offsets, int32_t n_tracks, const double* v0,
                                   const double* a0, const double* seg_times_in, double* coeffs, int32_t* status,
                                   void* stream) {
    if (n_tracks > 0 && !seg_times_in) {
        set_error("epp_minsnap_batch_times: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    // the kernel copies the caller's times to seg_times: in place is fine (same index)
    return minsnap_batch(wp, wp_offsets, n_tracks, 0.0, 0.0, v0, a0, seg_times_in, const_cast<double*>(seg_times_in),
                         coeffs, status, stream, "epp_minsnap_batch_times");
}

epp_status epp_sample_count(const double* seg_times, const int32_t* wp_offsets, int32_t n_tracks, double dt,
                            int64_t* row_counts, void* stream) {
    if (n_tracks < 0 || (n_tracks > 0 && (!seg_times || !wp_offsets || !row_counts))) {
        set_error("epp_sample_count: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    int max_m = 0;
    epp_status st = read_offsets(wp_offsets, n_tracks, (hipStream_t)stream, "epp_sample_count", &max_m, nullptr);
    if (st) return st;
    hipLaunchKernelGGL(k_sample_count, dim3(n_tracks), dim3(kWave), (size_t)(max_m + 2) * 8, (hipStream_t)stream,
                       seg_times, wp_offsets, n_tracks, dt, row_counts);
    return launch_error("epp_sample_count");
}

epp_status epp_sample_batch(const double* seg_times, const double* coeffs, const int32_t* wp_offsets, int32_t n_tracks,
                            double dt, const double* t0, const int64_t* row_offsets, double* rows, void* stream) {
    if (n_tracks < 0 || (n_tracks > 0 && (!seg_times || !coeffs || !wp_offsets || !row_offsets || !rows))) {
        set_error("epp_sample_batch: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    epp_status st = ensure_consts();
    if (st) return st;
    int max_m = 0;
    if ((st = read_offsets(wp_offsets, n_tracks, (hipStream_t)stream, "epp_sample_batch", &max_m, nullptr))) return st;
    const size_t shm = ((size_t)kNC + ((max_m + 1) & ~1) + 3 * kRowChunk + 2) * 8;
    hipLaunchKernelGGL(k_sample_rows, dim3(n_tracks), dim3(kWave), shm, (hipStream_t)stream, seg_times, coeffs,
                       wp_offsets, n_tracks, dt, t0, row_offsets, rows, (int64_t)INT64_MAX);
    return launch_error("epp_sample_batch");
}

// poly_traj::generateTrajectory with host buffers (src/trajectory_generator.cpp:12-100).
// The host computes the segment times (estimateSegmentTimesNfabian with its libm, as the
// reference, or the caller's) and runs Trajectory::evaluateRange's sample recurrence
// (src/trajectory.cpp:81-141: exact count, times and segments); one launch of k_refit then
// solves and writes the rows straight into pinned memory; one stream synchronisation.
// The rows are copied once, from the pinned buffer the kernel wrote into the buffer
// alloc(ctx, R) returns (the C ABI: malloc; the C++ API: the result matrix itself).
}  // extern "C"

epp_status epp::generate_trajectory_into(const double* wp, int32_t n_wp, const double* times, double v_max,
                                         double a_max, double dt, double t0, const double v0[3], const double a0[3],
                                         double* (*alloc)(void*, int64_t), void* ctx, int64_t* n_rows) {
    return check_and_generate_into(nullptr, wp, n_wp, times, v_max, a_max, dt, t0, v0, a0, alloc, ctx, n_rows);
}

epp_status epp::check_and_generate_into(const FusedCheck* chk, const double* wp, int32_t n_wp, const double* times,
                                        double v_max, double a_max, double dt, double t0, const double v0[3],
                                        const double a0[3], double* (*alloc)(void*, int64_t), void* ctx,
                                        int64_t* n_rows) {
    if (!alloc || !n_rows || (n_wp > 0 && !wp) ||
        (chk && (!chk->world || chk->n < 0 || (chk->n > 0 && (!chk->xyz || !chk->valid))))) {
        set_error("generateTrajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *n_rows = 0;
    if (n_wp < 2) {
        set_error("At least two waypoints are required");  // trajectory_generator.cpp:24
        return EPP_ERR_INVALID_ARGUMENT;
    }
    epp_status rc = ensure_consts();
    if (rc) return rc;
    static thread_local RefitCache c;
    const int M = n_wp - 1;
    c.T.resize(M);
    for (int i = 0; i < M; ++i) {
        c.T[i] = times ? times[i] : nfabian(wp + 3 * i, wp + 3 * (i + 1), v_max, a_max);
        if (!(c.T[i] > 0)) {  // CHECK_GT(segment_time, 0)  impl :297
            set_error("Segment times need to be greater than zero");
            return EPP_ERR_RUNTIME;
        }
    }
    c.tin.clear();
    c.tac.clear();
    c.seg.clear();
    if (dt > 0) {
        RangeIter it;
        it.init(c.T.data(), M);
        int sg;
        double ti, ta;
        while (it.next(sg, ti, ta)) {
            c.seg.push_back(sg);
            c.tin.push_back(ti);
            c.tac.push_back(ta);
            it.advance(dt);
        }
    }
    const int R = (int)c.tin.size();
    const bool lds = M <= kMaxLdsSeg;
    // long tracks whose vertex values and coefficients would not fit LDS beside the rest
    // (> ~300 segments: e.g. a track smoothed by "ompl" simplification) keep them in the
    // global scratch too
    const bool big = !lds && refit_lds_doubles(M, false) * sizeof(double) > kRefitLdsMax;
    if (refit_lds_doubles(M, lds, big) * sizeof(double) > kRefitLdsMax) {
        set_error("generateTrajectory: too many waypoints for one workgroup's LDS (" + std::to_string(n_wp) + ")");
        return EPP_ERR_UNSUPPORTED;
    }
    const int G = R ? std::min(kRefitMaxWriters, (R + kRefitRowChunk - 1) / kRefitRowChunk) : 1;
    // the fused check (chk): the lookahead points after the refit's inputs (h_in), their
    // flags after the completion slots (h_out); its workgroups after the refit's.  The
    // records' snapshot (and its lease: no update rewrites them) is held until the poll ends.
    SmallWorld sw{};
    const int64_t nck = chk ? chk->n : 0;
    int per = kSmallBlock, Gc = 0;
    if (nck > 0) {
        sw = small_world(chk->world);
        if (nck > kSmallStates || sw.n_obb > kSmallMaxObbs) {
            set_error("checkAndGenerate: the check is not small (<= 4096 points, <= 256 OBBs)");
            return EPP_ERR_UNSUPPORTED;
        }
        per = small_per(nck);
        Gc = (int)((nck + per - 1) / per);
    }
    const size_t in_refit = (refit_in_doubles(n_wp, R) + 1) & ~size_t(1);  // (16-byte aligned points after it)
    constexpr size_t kRowsAt = 256;  // h_out: [status | pad | slots (<= 48 x 4 B) | flags | rows]
    const size_t rows_at = kRowsAt + (((size_t)nck + 255) & ~size_t(255));
    if ((rc = c.ensure((in_refit + 3 * (size_t)nck) * 8, (size_t)R * 80 + rows_at,
                       lds ? 0 : (size_t)G * refit_scr_doubles(M, big) * 8)))
        return rc;
    double* in = c.h_in;
    std::memcpy(in, wp, (size_t)n_wp * 24);
    for (int k = 0; k < 3; ++k) {
        in[3 * n_wp + k] = v0 ? v0[k] : 0.0;
        in[3 * n_wp + 3 + k] = a0 ? a0[k] : 0.0;
    }
    std::memcpy(in + 3 * n_wp + 6, c.T.data(), (size_t)M * 8);
    double* ins = in + 3 * n_wp + 6 + M;
    if (R) {
        std::memcpy(ins, c.tin.data(), (size_t)R * 8);
        std::memcpy(ins + R, c.tac.data(), (size_t)R * 8);
        std::memcpy(ins + 2 * R, c.seg.data(), (size_t)R * 4);
    }
    RefitArgs a;
    a.in = in;
    a.W = n_wp;
    a.R = R;
    a.writers = G;
    if (++c.seq == 0) c.seq = 1;
    a.seq = c.seq;
    a.t0 = t0;
    if (n_wp <= kRefitArgW) std::memcpy(a.small, in, (size_t)(3 * n_wp + 6 + M) * 8);
    a.info = reinterpret_cast<int64_t*>(c.h_out);
    a.done = reinterpret_cast<uint32_t*>(c.h_out + 64);
    a.out = reinterpret_cast<double*>(c.h_out + rows_at);
    a.scratch = c.d_scr;
    a.big = big ? 1 : 0;
    {  // the latency path solves without the refinement step: it cost 6-7 us of a ~30 us
       // call (scripts/refit_ab.py) for ~1e-10 of accuracy the sampled rows do not need
       // (rows vs the truth 6e-11 either way).  EPP_REFIT_REFINE=1: with it (A/B knob)
        static const int refine = [] {
            const char* e = std::getenv("EPP_REFIT_REFINE");
            return e && *e == '1' ? 1 : 0;
        }();
        a.refine = refine;
    }
    a.info[0] = -100;
    size_t shm = refit_lds_doubles(M, lds, big) * sizeof(double);
    if (Gc > 0) {
        double* pts = in + in_refit;
        std::memcpy(pts, chk->xyz, (size_t)nck * 24);
        CheckArgs ck;
        ck.recs = sw.recs;
        ck.n_obb = sw.n_obb;
        ck.per = per;
        ck.rg = sw.r_gate;
        ck.ro = sw.r_obst;
        ck.md = chk->min_distance;
        ck.xyz = pts;
        ck.n = nck;
        ck.valid = reinterpret_cast<uint8_t*>(c.h_out + kRowsAt);
        shm = std::max(shm, small_shm(sw.n_obb));
        if (lds) {
            allow_lds(k_check_refit<true>);
            hipLaunchKernelGGL(k_check_refit<true>, dim3(G + Gc), dim3(kRefitBlock), shm, c.s, a, ck);
        } else {
            allow_lds(k_check_refit<false>);
            hipLaunchKernelGGL(k_check_refit<false>, dim3(G + Gc), dim3(kRefitBlock), shm, c.s, a, ck);
        }
    } else if (lds) {
        allow_lds(k_refit<true>);
        hipLaunchKernelGGL(k_refit<true>, dim3(G), dim3(kRefitBlock), shm, c.s, a);
    } else {
        allow_lds(k_refit<false>);
        hipLaunchKernelGGL(k_refit<false>, dim3(G), dim3(kRefitBlock), shm, c.s, a);
    }
    hipError_t e = hipGetLastError();
    // wait for the status word and every workgroup's slot (polled; the stream is queried
    // every ~1k polls so a failed launch ends the wait)
    const int slots = G + Gc;
    auto complete = [&]() {
        if (__atomic_load_n(a.info, __ATOMIC_ACQUIRE) == -100) return false;
        for (int g = 0; g < slots; ++g)
            if (__atomic_load_n(a.done + g, __ATOMIC_ACQUIRE) != a.seq) return false;
        return true;
    };
    for (uint64_t spin = 0; e == hipSuccess && !complete(); ++spin) {
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(c.s);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) e = q;
            else if (!complete()) e = hipErrorUnknown;  // finished without its completion words
            break;
        }
        _mm_pause();
    }
    const int64_t info = __atomic_load_n(a.info, __ATOMIC_ACQUIRE);
    if (e != hipSuccess) {
        set_error(std::string("generateTrajectory: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    if (Gc > 0) std::memcpy(chk->valid, c.h_out + kRowsAt, (size_t)nck);
    if (info != 0) {
        set_error(info == -2 ? "Segment times need to be greater than zero" : "min-snap solve failed");
        return EPP_ERR_RUNTIME;
    }
    double* host_rows = alloc(ctx, R);
    if (!host_rows) {
        set_error("generateTrajectory: out of host memory");
        return EPP_ERR_RUNTIME;
    }
    if (R) std::memcpy(host_rows, a.out, (size_t)R * 80);
    *n_rows = R;
    return EPP_OK;
}

namespace epp {
namespace {
double* malloc_rows(void* ctx, int64_t R) {
    double* p = (double*)std::malloc((size_t)std::max<int64_t>(R, 1) * 80);
    *static_cast<double**>(ctx) = p;
    return p;
}
epp_status generate_trajectory(const double* wp, int32_t n_wp, const double* times, double v_max, double a_max,
                               double dt, double t0, const double v0[3], const double a0[3], double** rows_out,
                               int64_t* n_rows) {
    if (!rows_out || !n_rows) {
        set_error("generateTrajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *rows_out = nullptr;
    const epp_status rc = generate_trajectory_into(wp, n_wp, times, v_max, a_max, dt, t0, v0, a0, malloc_rows,
                                                   rows_out, n_rows);
    if (rc != EPP_OK && *rows_out) {
        std::free(*rows_out);
        *rows_out = nullptr;
    }
    return rc;
}
}  // namespace
}  // namespace epp

extern "C" {

epp_status epp_generate_trajectory_host(const double* wp, int32_t n_wp, double v_max, double a_max, double dt,
                                        double t0, const double v0[3], const double a0[3], double** rows_out,
                                        int64_t* n_rows) {
    return generate_trajectory(wp, n_wp, nullptr, v_max, a_max, dt, t0, v0, a0, rows_out, n_rows);
}

epp_status epp_check_and_generate_trajectory_host(const epp_world* world, const double* check_xyz, int64_t n_check,
                                                  double min_distance, uint8_t* check_valid, const double* wp,
                                                  int32_t n_wp, double v_max, double a_max, double dt, double t0,
                                                  const double v0[3], const double a0[3], double** rows_out,
                                                  int64_t* n_rows) {
    if (!rows_out || !n_rows || !world || n_check < 0 || (n_check > 0 && (!check_xyz || !check_valid))) {
        set_error("epp_check_and_generate_trajectory_host: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *rows_out = nullptr;
    const FusedCheck chk{world, check_xyz, n_check, min_distance, check_valid};
    const epp_status rc = check_and_generate_into(&chk, wp, n_wp, nullptr, v_max, a_max, dt, t0, v0, a0, malloc_rows,
                                                  rows_out, n_rows);
    if (rc != EPP_OK && *rows_out) {
        std::free(*rows_out);
        *rows_out = nullptr;
    }
    return rc;
}

epp_status epp_generate_trajectory_times_host(const double* wp, int32_t n_wp, const double* seg_times, double dt,
                                              double t0, const double v0[3], const double a0[3], double** rows_out,
                                              int64_t* n_rows) {
    if (n_wp >= 2 && !seg_times) {
        set_error("generateTrajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    return generate_trajectory(wp, n_wp, seg_times, 0.0, 0.0, dt, t0, v0, a0, rows_out, n_rows);
}

#ifdef EPP_REFIT_TL
// diagnostics builds only: the last refit's phase timeline (2 workgroups x 16 stamps)
epp_status epp_dbg_refit_tl(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_refit_tl), sizeof(g_refit_tl));
    if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(g_refit_it), sizeof(g_refit_it));
    return e == hipSuccess ? EPP_OK : EPP_ERR_HIP;
}
#endif

}  // extern "C"

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
// SPD and solved by a block Cholesky (block Thomas) instead of the reference's
// Eigen SparseQR/COLAMD; the two agree to rounding (parity target 1e-6).
//
// Sampling reproduces Trajectory::evaluateRange (src/trajectory.cpp:81-141) exactly:
// one lane runs the sequential `acc += dt` / segment roll-over recurrence (so sample
// times and counts are bit-identical), and the wavefront evaluates the rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "epp_internal.h"

namespace epp {
namespace {

constexpr int N = 10;
constexpr int HALF = 5;
constexpr int kWave = 64;
constexpr int kMaxLdsSeg = 24;  // tracks with more segments use the global scratch path

// falling factorials: B[k][j] = j! / (j-k)!  (src/polynomial.cpp:145-160)
__constant__ double cB[N][N];

struct SegScratch {  // per-segment scratch: A^-1 (100), H (100), Q 6x6 block (36), W (16), L (16)
    static constexpr int kAinv = 0, kH = 100, kQ = 200, kW = 236, kL = 252, kSize = 268;
};

__host__ __device__ __forceinline__ double nfabian(const double* p, const double* q, double vmax,
                                          double amax) {
    // estimateSegmentTimesNfabian — src/vertex.cpp:272-289 (magic 6.5)
    const double d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
    const double distance = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    return distance / vmax * 2 * (1.0 + 6.5 * vmax / amax * exp(-distance / vmax * 2));
}

// setupMappingMatrix + invertMappingMatrix (Schur complement), one lane per segment.
__device__ void invert_mapping(double T, double* Ai /* 10x10 row-major */) {
    // A rows 5+k = baseCoeffsWithTime(N, k, T): [k] = B[k][k], [j>k] = B[k][j] * T^(j-k)
    // with the power built by repeated multiplication (polynomial.h:213-218).
    double C[HALF][HALF], D[HALF][HALF];
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
        double row[N];
#pragma unroll
        for (int j = 0; j < N; ++j) row[j] = 0.0;
        row[k] = cB[k][k];
        if (fabs(T) >= 2.220446049250313e-16) {
            double tp = T;
#pragma unroll
            for (int j = k + 1; j < N; ++j) {
                row[j] = cB[k][j] * tp;
                tp = tp * T;
            }
        }
#pragma unroll
        for (int j = 0; j < HALF; ++j) {
            C[k][j] = row[j];
            D[k][j] = row[j + HALF];
        }
    }
    // D^-1 by LU with partial pivoting (Eigen's 5x5 inverse path).  Every loop is fully
    // unrolled and the row swap is a select, so all indices are static and the arrays
    // stay in registers (a data-dependent row index would put them in scratch memory).
    int perm[HALF];
#pragma unroll
    for (int i = 0; i < HALF; ++i) perm[i] = i;
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
        int p = k;
        double best = fabs(D[k][k]);
#pragma unroll
        for (int r = k + 1; r < HALF; ++r)
            if (fabs(D[r][k]) > best) {
                best = fabs(D[r][k]);
                p = r;
            }
#pragma unroll
        for (int r = k + 1; r < HALF; ++r) {
            const bool sw = (r == p);
#pragma unroll
            for (int c = 0; c < HALF; ++c) {
                const double t = D[k][c];
                D[k][c] = sw ? D[r][c] : t;
                D[r][c] = sw ? t : D[r][c];
            }
            const int t = perm[k];
            perm[k] = sw ? perm[r] : t;
            perm[r] = sw ? t : perm[r];
        }
#pragma unroll
        for (int r = k + 1; r < HALF; ++r) {
            D[r][k] = D[r][k] / D[k][k];
#pragma unroll
            for (int c = k + 1; c < HALF; ++c) D[r][c] = D[r][c] - D[r][k] * D[k][c];
        }
    }
    double Dinv[HALF][HALF];
#pragma unroll
    for (int col = 0; col < HALF; ++col) {
        double x[HALF];
#pragma unroll
        for (int i = 0; i < HALF; ++i) x[i] = (perm[i] == col) ? 1.0 : 0.0;
#pragma unroll
        for (int i = 0; i < HALF; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) x[i] = x[i] - D[i][j] * x[j];
#pragma unroll
        for (int i = HALF - 1; i >= 0; --i) {
#pragma unroll
            for (int j = i + 1; j < HALF; ++j) x[i] = x[i] - D[i][j] * x[j];
            x[i] = x[i] / D[i][i];
        }
#pragma unroll
        for (int i = 0; i < HALF; ++i) Dinv[i][col] = x[i];
    }
    for (int i = 0; i < N * N; ++i) Ai[i] = 0.0;
    for (int r = 0; r < HALF; ++r) {
        const double adinv = 1.0 / cB[r][r];  // A_diag.cwiseInverse()
        Ai[r * N + r] = adinv;
        for (int c = 0; c < HALF; ++c) Ai[(r + HALF) * N + c + HALF] = Dinv[r][c];
    }
    for (int r = 0; r < HALF; ++r)
        for (int c = 0; c < HALF; ++c) {
            double s = 0.0;
            for (int k = 0; k < HALF; ++k) s = s + Dinv[r][k] * C[k][c];
            Ai[(r + HALF) * N + c] = -s * (1.0 / cB[c][c]);  // -D^-1 C A_diag^-1
        }
}

// 4x4 Cholesky (lower factor in place; false if not SPD) and the two triangular solves
// with MC right-hand sides (b: 4 x MC, row-major), on register arrays: fully unrolled so
// the indices are static.  The serial block solve runs on one lane, where every LDS round
// trip in a dependent chain would be exposed latency.
__device__ __forceinline__ bool chol4r(double (&L)[16]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double d = L[j * 4 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) d = d - L[j * 4 + k] * L[j * 4 + k];
        ok = ok && (d > 0.0);
        d = sqrt(d);
        L[j * 4 + j] = d;
#pragma unroll
        for (int i = j + 1; i < 4; ++i) {
            double s = L[i * 4 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) s = s - L[i * 4 + k] * L[j * 4 + k];
            L[i * 4 + j] = s / d;
        }
#pragma unroll
        for (int i = 0; i < j; ++i) L[i * 4 + j] = 0.0;
    }
    return ok;
}
template <int MC>
__device__ __forceinline__ void lsolve4r(const double (&L)[16], double (&b)[4 * MC]) {
#pragma unroll
    for (int c = 0; c < MC; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double s = b[i * MC + c];
#pragma unroll
            for (int k = 0; k < i; ++k) s = s - L[i * 4 + k] * b[k * MC + c];
            b[i * MC + c] = s / L[i * 4 + i];
        }
}
template <int MC>
__device__ __forceinline__ void ltsolve4r(const double (&L)[16], double (&b)[4 * MC]) {
#pragma unroll
    for (int c = 0; c < MC; ++c)
#pragma unroll
        for (int i = 3; i >= 0; --i) {
            double s = b[i * MC + c];
#pragma unroll
            for (int k = i + 1; k < 4; ++k) s = s - L[k * 4 + i] * b[k * MC + c];
            b[i * MC + c] = s / L[i * 4 + i];
        }
}

// One workgroup (= one wavefront) per track.  scratch: per segment SegScratch::kSize
// doubles (LDS when the track has <= kMaxLdsSeg segments, else the global workspace),
// plus per vertex 5x3 derivative values and 4x3 rhs.
template <bool LDS>
__global__ __launch_bounds__(kWave) void k_minsnap(const double* __restrict__ wp,
                                                   const int32_t* __restrict__ wp_off, int n_tracks,
                                                   double vmax, double amax,
                                                   const double* __restrict__ v0,
                                                   const double* __restrict__ a0,
                                                   double* __restrict__ seg_times,
                                                   double* __restrict__ coeffs,
                                                   int32_t* __restrict__ status,
                                                   double* __restrict__ gscratch,
                                                   const int64_t* __restrict__ gscratch_off) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    // all LDS in the one dynamic array (no static __shared__ in front of it:
    // cdna_hip_programming.md Guideline 17); the first 16 bytes hold the error flag
    int& s_err = *reinterpret_cast<int*>(smem);
    double* sm = smem + 2;
    const int track = blockIdx.x;
    if (track >= n_tracks) return;
    const int lane = threadIdx.x;
    const int w0 = wp_off[track];
    const int W = wp_off[track + 1] - w0;
    const int M = W - 1;
    const int seg0 = w0 - track;
    if (lane == 0) s_err = 0;
    if (W < 2) {
        if (lane == 0 && status) status[track] = -1;  // std::invalid_argument
        return;
    }
    double* scr;   // M * kSize
    double* dv;    // (M+1) * 5 * 3 vertex derivative values
    double* rhs;   // (M+1) * 4 * 3
    double* Tm;    // M
    if (LDS) {
        scr = sm;
        dv = scr + (size_t)M * SegScratch::kSize;
    } else {
        scr = gscratch + gscratch_off[track];
        dv = sm;
    }
    rhs = dv + (size_t)(M + 1) * 15;
    Tm = rhs + (size_t)(M + 1) * 12;
    const double* P = wp + (size_t)w0 * 3;
    __syncthreads();

    // ---- phase 1: segment times, mapping inverses, fixed vertex values ----------
    for (int i = lane; i < M; i += kWave) {
        const double T = nfabian(P + 3 * i, P + 3 * (i + 1), vmax, amax);
        Tm[i] = T;
        seg_times[seg0 + i] = T;
        if (!(T > 0)) atomicOr(&s_err, 1);  // CHECK_GT(segment_time, 0)  impl :297
        else invert_mapping(T, scr + (size_t)i * SegScratch::kSize + SegScratch::kAinv);
    }
    for (int e = lane; e < (M + 1) * 15; e += kWave) {
        const int v = e / 15, k = (e % 15) / 3, d = e % 3;
        double val = 0.0;  // free values are overwritten by the solve
        if (k == 0) val = P[3 * v + d];                       // position, every vertex
        else if (v == 0 && k == 1) val = v0 ? v0[3 * track + d] : 0.0;  // makeStartOrEnd
        else if (v == 0 && k == 2) val = a0 ? a0[3 * track + d] : 0.0;
        dv[e] = val;
    }
    __syncthreads();
    if (s_err) {
        if (lane == 0 && status) status[track] = -2;
        return;
    }
    // ---- phase 2: Q (6x6 snap block) and H = A^-T Q A^-1 --------------------------
    for (int e = lane; e < M * 36; e += kWave) {
        const int i = e / 36, a = 4 + (e % 36) / 6, b = 4 + e % 6;
        const double ex = (double)(a + b - 7);  // (N-1-4)*2+1-row-col with row=9-a, col=9-b
        scr[(size_t)i * SegScratch::kSize + SegScratch::kQ + (a - 4) * 6 + (b - 4)] =
            cB[4][a] * cB[4][b] * pow(Tm[i], ex) * 2.0 / ex;
    }
    __syncthreads();
    // All 100 entries are computed (no mirroring of a triangle): each row then keeps
    // the exact translation invariance H[r][0] == -H[r][5] that the reference's full
    // product has; mirroring breaks it and costs ~1e-6 on long, stiff tracks.
    for (int e = lane; e < M * 100; e += kWave) {
        const int i = e / 100, r = (e % 100) / 10, c = e % 10;
        const double* S = scr + (size_t)i * SegScratch::kSize;
        const double* Ai = S + SegScratch::kAinv;
        const double* Q = S + SegScratch::kQ;
        double h = 0.0;
        for (int a = 4; a < N; ++a) {
            double qa = 0.0;
            for (int b = 4; b < N; ++b) qa = qa + Q[(a - 4) * 6 + (b - 4)] * Ai[b * N + c];
            h = h + Ai[a * N + r] * qa;
        }
        double* H = const_cast<double*>(S) + SegScratch::kH;
        H[r * N + c] = h;
    }
    __syncthreads();
    // ---- phase 3: block-tridiagonal system over the inner vertices ----------------
    // free variable (v, p): vertex v in 1..M-1, derivative p+1.  Diagonal block D_v is
    // kept in the L slot of segment v-1, the coupling E_v (v -> v+1) in the W slot.
    const int nin = M - 1;
    for (int e = lane; e < nin * 16; e += kWave) {
        const int v = 1 + e / 16, p = (e % 16) / 4, q = e % 4;
        const double* Hm = scr + (size_t)(v - 1) * SegScratch::kSize + SegScratch::kH;
        const double* Hp = scr + (size_t)v * SegScratch::kSize + SegScratch::kH;
        scr[(size_t)(v - 1) * SegScratch::kSize + SegScratch::kL + p * 4 + q] =
            Hm[(6 + p) * N + 6 + q] + Hp[(1 + p) * N + 1 + q];
        scr[(size_t)(v - 1) * SegScratch::kSize + SegScratch::kW + p * 4 + q] =
            (v < nin) ? Hp[(1 + p) * N + 6 + q] : 0.0;
    }
    for (int e = lane; e < nin * 12; e += kWave) {
        const int v = 1 + e / 12, p = (e % 12) / 3, d = e % 3;
        double s = 0.0;
        // segment v-1: rows 0..4 = vertex v-1, rows 5..9 = vertex v; row of (v,p+1) = 6+p
        {
            const double* H = scr + (size_t)(v - 1) * SegScratch::kSize + SegScratch::kH;
            for (int r = 0; r < N; ++r) {
                const int vv = (r < HALF) ? v - 1 : v, k = r % HALF;
                const bool fixed = (k == 0) || vv == 0 || vv == M;
                if (fixed) s = s + H[(6 + p) * N + r] * dv[(vv * HALF + k) * 3 + d];
            }
        }
        // segment v: rows 0..4 = vertex v (row of (v,p+1) = 1+p), rows 5..9 = vertex v+1
        {
            const double* H = scr + (size_t)v * SegScratch::kSize + SegScratch::kH;
            for (int r = 0; r < N; ++r) {
                const int vv = (r < HALF) ? v : v + 1, k = r % HALF;
                const bool fixed = (k == 0) || vv == 0 || vv == M;
                if (fixed) s = s + H[(1 + p) * N + r] * dv[(vv * HALF + k) * 3 + d];
            }
        }
        rhs[(v * 4 + p) * 3 + d] = -s;
    }
    __syncthreads();
    // ---- phase 4: block Cholesky solve (one lane; 4x4 blocks, 3 right-hand sides) ---
    if (lane == 0 && nin > 0) {
        // the carried blocks (W_{v-1}, z_{v-1}; x_{v+1} on the way back) stay in registers
        bool ok = true;
        double Wp[16], zp[12];
        for (int v = 1; v <= nin; ++v) {
            double* Ls = scr + (size_t)(v - 1) * SegScratch::kSize + SegScratch::kL;
            double L[16], b[12];
#pragma unroll
            for (int i = 0; i < 16; ++i) L[i] = Ls[i];
#pragma unroll
            for (int i = 0; i < 12; ++i) b[i] = rhs[(size_t)v * 12 + i];
            if (v > 1) {  // S_v = D_v - W_{v-1}^T W_{v-1},  W_{v-1} = L_{v-1}^-1 E_{v-1}
#pragma unroll
                for (int p = 0; p < 4; ++p)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        double s = 0.0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) s = s + Wp[k * 4 + p] * Wp[k * 4 + q];
                        L[p * 4 + q] = L[p * 4 + q] - s;
                    }
                // z_v = b_v - W_{v-1}^T z_{v-1}
#pragma unroll
                for (int p = 0; p < 4; ++p)
#pragma unroll
                    for (int d = 0; d < 3; ++d) {
                        double s = 0.0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) s = s + Wp[k * 4 + p] * zp[k * 3 + d];
                        b[p * 3 + d] = b[p * 3 + d] - s;
                    }
            }
            ok = chol4r(L);
            if (!ok) break;
            lsolve4r<3>(L, b);
#pragma unroll
            for (int i = 0; i < 16; ++i) Ls[i] = L[i];
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                rhs[(size_t)v * 12 + i] = b[i];
                zp[i] = b[i];
            }
            if (v < nin) {
                double* Ws = scr + (size_t)(v - 1) * SegScratch::kSize + SegScratch::kW;
                double W[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) W[i] = Ws[i];
                lsolve4r<4>(L, W);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    Ws[i] = W[i];
                    Wp[i] = W[i];
                }
            }
        }
        if (ok) {
            double xn[12];
            for (int v = nin; v >= 1; --v) {
                double x[12], L[16];
#pragma unroll
                for (int i = 0; i < 12; ++i) x[i] = rhs[(size_t)v * 12 + i];
#pragma unroll
                for (int i = 0; i < 16; ++i) L[i] = scr[(size_t)(v - 1) * SegScratch::kSize + SegScratch::kL + i];
                if (v < nin) {  // z_v - W_v x_{v+1}
                    const double* Wv = scr + (size_t)(v - 1) * SegScratch::kSize + SegScratch::kW;
                    double W[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) W[i] = Wv[i];
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int d = 0; d < 3; ++d) {
                            double s = 0.0;
#pragma unroll
                            for (int k = 0; k < 4; ++k) s = s + W[p * 4 + k] * xn[k * 3 + d];
                            x[p * 3 + d] = x[p * 3 + d] - s;
                        }
                }
                ltsolve4r<3>(L, x);
#pragma unroll
                for (int i = 0; i < 12; ++i) {
                    rhs[(size_t)v * 12 + i] = x[i];
                    xn[i] = x[i];
                }
#pragma unroll
                for (int p = 0; p < 4; ++p)
#pragma unroll
                    for (int d = 0; d < 3; ++d) dv[(v * HALF + 1 + p) * 3 + d] = x[p * 3 + d];
            }
        } else {
            s_err = 1;
        }
    }
    __syncthreads();
    if (s_err) {
        if (lane == 0 && status) status[track] = -3;
        return;
    }
    // ---- phase 5: p_i = A_i^-1 [d_i ; d_{i+1}] -------------------------------------
    for (int e = lane; e < M * 30; e += kWave) {
        const int i = e / 30, d = (e % 30) / 10, r = e % 10;
        const double* Ai = scr + (size_t)i * SegScratch::kSize + SegScratch::kAinv;
        double s = 0.0;
        for (int k = 0; k < N; ++k) {
            const int v = i + (k >= HALF ? 1 : 0);
            s = s + Ai[r * N + k] * dv[(v * HALF + (k % HALF)) * 3 + d];
        }
        coeffs[((size_t)(seg0 + i) * 3 + d) * N + r] = s;
    }
    if (lane == 0 && status) status[track] = 0;
}

constexpr int kRowChunk = 512;  // samples per k_sample_rows round

// Trajectory::evaluateRange control flow — src/trajectory.cpp:81-141.
struct RangeIter {
    const double* T;
    int M, i;
    double t_end, acc, tis, Ti;  // Ti = T[i], kept in a register (one LDS read per segment)
    __device__ void init(const double* T_, int M_) {
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
    __device__ bool next(int& seg, double& t_in, double& t_acc) {
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
    __device__ void advance(double dt) {
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
__device__ __forceinline__ double poly_eval(const double* c, double t, int k) {
    double r = cB[k][N - 1] * c[N - 1];
    for (int j = N - 2; j >= k; --j) {
        r = r * t;
        r = r + cB[k][j] * c[j];
    }
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
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int t = blockIdx.x;
    if (t >= n_tracks) return;
    const int lane = threadIdx.x;
    const int M = wp_off[t + 1] - wp_off[t] - 1;
    if (M < 1 || !(dt > 0)) return;
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
                for (int k = 0; k < 3; ++k) row[3 * d + k] = poly_eval(cs + d * N, tin, k);
            row[9] = s_tac[j] + toff;  // sampling_times[i] + startTimeOffset
        }
        base += cnt;
        __syncthreads();
        if (done) break;
    }
}

struct Workspace {
    double* d = nullptr;
    size_t cap = 0;
    int64_t* off = nullptr;
    size_t off_cap = 0;
};
Workspace g_ws[64];
bool g_consts_ready[64];

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
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(cB), B, sizeof(B));
    if (e != hipSuccess) {
        set_error(std::string("epp minsnap: constants: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    if (dev >= 0 && dev < 64) g_consts_ready[dev] = true;
    return EPP_OK;
}

// Largest segment count of a batch (the offsets live on the device).
int max_segments(const int32_t* d_off, int n_tracks, hipStream_t s, int* out) {
    std::vector<int32_t> off(n_tracks + 1);
    hipError_t e = hipMemcpyAsync(off.data(), d_off, off.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        set_error(std::string("epp: reading track offsets: ") + hipGetErrorString(e));
        return -1;
    }
    int m = 1;
    for (int t = 0; t < n_tracks; ++t) m = std::max(m, off[t + 1] - off[t] - 1);
    *out = m;
    return 0;
}

}  // namespace
}  // namespace epp

using namespace epp;

extern "C" {

epp_status epp_minsnap_batch(const double* wp, const int32_t* wp_offsets, int32_t n_tracks,
                             double v_max, double a_max, const double* v0, const double* a0,
                             double* seg_times, double* coeffs, int32_t* status, void* stream) {
    if (n_tracks < 0 || (n_tracks > 0 && (!wp || !wp_offsets || !seg_times || !coeffs))) {
        set_error("epp_minsnap_batch: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    epp_status st = ensure_consts();
    if (st) return st;
    hipStream_t s = (hipStream_t)stream;
    // The offsets live on the device; the launcher needs the largest segment count to
    // size LDS, so read them back (n_tracks + 1 ints).
    std::vector<int32_t> off(n_tracks + 1);
    hipError_t e = hipMemcpyAsync(off.data(), wp_offsets, off.size() * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        set_error(std::string("epp_minsnap_batch: offsets: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    int max_m = 0;
    for (int t = 0; t < n_tracks; ++t) max_m = std::max(max_m, off[t + 1] - off[t] - 1);
    if (max_m < 1) max_m = 1;
    const size_t vert_doubles = (size_t)(max_m + 1) * (15 + 12) + max_m;
    if (max_m <= kMaxLdsSeg) {
        const size_t shm = ((size_t)max_m * SegScratch::kSize + vert_doubles + 2) * sizeof(double);
        hipLaunchKernelGGL((k_minsnap<true>), dim3(n_tracks), dim3(kWave), shm, s, wp, wp_offsets,
                           n_tracks, v_max, a_max, v0, a0, seg_times, coeffs, status, nullptr,
                           nullptr);
    } else {
        int dev = 0;
        (void)hipGetDevice(&dev);
        Workspace& ws = g_ws[dev & 63];
        std::vector<int64_t> goff(n_tracks);
        size_t total = 0;
        for (int t = 0; t < n_tracks; ++t) {
            goff[t] = (int64_t)total;
            total += (size_t)std::max(1, off[t + 1] - off[t] - 1) * SegScratch::kSize;
        }
        if (total > ws.cap) {
            if (ws.d) (void)hipFree(ws.d);
            ws.d = nullptr;
            ws.cap = 0;
            if (hipMalloc(&ws.d, total * sizeof(double)) != hipSuccess) return EPP_ERR_HIP;
            ws.cap = total;
        }
        if ((size_t)n_tracks > ws.off_cap) {
            if (ws.off) (void)hipFree(ws.off);
            ws.off = nullptr;
            ws.off_cap = 0;
            if (hipMalloc(&ws.off, (size_t)n_tracks * 8) != hipSuccess) return EPP_ERR_HIP;
            ws.off_cap = n_tracks;
        }
        e = hipMemcpyAsync(ws.off, goff.data(), (size_t)n_tracks * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return EPP_ERR_HIP;
        const size_t shm = (vert_doubles + 2) * sizeof(double);
        hipLaunchKernelGGL((k_minsnap<false>), dim3(n_tracks), dim3(kWave), shm, s, wp, wp_offsets,
                           n_tracks, v_max, a_max, v0, a0, seg_times, coeffs, status, ws.d, ws.off);
    }
    e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string("epp_minsnap_batch: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    return EPP_OK;
}

epp_status epp_sample_count(const double* seg_times, const int32_t* wp_offsets, int32_t n_tracks,
                            double dt, int64_t* row_counts, void* stream) {
    if (n_tracks < 0 || (n_tracks > 0 && (!seg_times || !wp_offsets || !row_counts))) {
        set_error("epp_sample_count: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    int max_m = 0;
    if (max_segments(wp_offsets, n_tracks, (hipStream_t)stream, &max_m)) return EPP_ERR_HIP;
    hipLaunchKernelGGL(k_sample_count, dim3(n_tracks), dim3(kWave), (size_t)(max_m + 2) * 8,
                       (hipStream_t)stream, seg_times, wp_offsets, n_tracks, dt, row_counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string("epp_sample_count: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    return EPP_OK;
}

epp_status epp_sample_batch(const double* seg_times, const double* coeffs, const int32_t* wp_offsets,
                            int32_t n_tracks, double dt, const double* t0, const int64_t* row_offsets,
                            double* rows, void* stream) {
    if (n_tracks < 0 ||
        (n_tracks > 0 && (!seg_times || !coeffs || !wp_offsets || !row_offsets || !rows))) {
        set_error("epp_sample_batch: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n_tracks == 0) return EPP_OK;
    epp_status st = ensure_consts();
    if (st) return st;
    int max_m = 0;
    if (max_segments(wp_offsets, n_tracks, (hipStream_t)stream, &max_m)) return EPP_ERR_HIP;
    const size_t shm = ((size_t)((max_m + 1) & ~1) + 3 * kRowChunk + 2) * 8;
    hipLaunchKernelGGL(k_sample_rows, dim3(n_tracks), dim3(kWave), shm, (hipStream_t)stream, seg_times,
                       coeffs, wp_offsets, n_tracks, dt, t0, row_offsets, rows, (int64_t)INT64_MAX);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string("epp_sample_batch: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    return EPP_OK;
}

// poly_traj::generateTrajectory with host buffers (src/trajectory_generator.cpp:12-100).
// Latency path (one track, e.g. the 50 Hz refit): per-thread cached device / pinned
// buffers and stream, one upload, the three kernels back to back (the host knows the
// segment count, so no offset read-backs), one download.  The row buffer is sized from
// the segment times recomputed on the host (+16 rows of slack; the kernel never writes
// past it, and a short buffer is detected and redone).
epp_status epp_generate_trajectory_host(const double* wp, int32_t n_wp, double v_max, double a_max,
                                        double dt, double t0, const double v0[3],
                                        const double a0[3], double** rows_out, int64_t* n_rows) {
    if (!rows_out || !n_rows || (n_wp > 0 && !wp)) {
        set_error("generateTrajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *rows_out = nullptr;
    *n_rows = 0;
    if (n_wp < 2) {
        set_error("At least two waypoints are required");  // trajectory_generator.cpp:24
        return EPP_ERR_INVALID_ARGUMENT;
    }
    epp_status rc = ensure_consts();
    if (rc) return rc;
    const int M = n_wp - 1;
    double t_end = 0.0;  // host estimate of the duration (capacity only)
    for (int i = 0; i < M; ++i) t_end += nfabian(wp + 3 * i, wp + 3 * (i + 1), v_max, a_max);
    int64_t cap = (dt > 0 && std::isfinite(t_end)) ? (int64_t)(t_end / dt) + 16 : 16;
    struct Cache {
        char* d = nullptr;
        size_t dcap = 0;
        char* h = nullptr;
        size_t hcap = 0;
        hipStream_t s = nullptr;
    };
    static thread_local Cache c;
    auto a16 = [](size_t x) { return (x + 15) & ~size_t(15); };
    const bool lds = M <= kMaxLdsSeg;
    for (int pass = 0; pass < 2; ++pass) {
        // device: [in: wp | va | t0 | off(2 i32) | goff | roff] [T | C | scratch] [rows (cap) | cnt | status]
        const size_t in_b = a16((size_t)n_wp * 24 + 48 + 8 + 8 + 8 + 8);
        const size_t mid_b = a16((size_t)M * 8) + a16((size_t)M * 240) + (lds ? 0 : a16((size_t)M * SegScratch::kSize * 8));
        const size_t out_b = (size_t)cap * 80 + 16;
        const size_t need = in_b + mid_b + out_b;
        if (!c.s && hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking) != hipSuccess) {
            set_error("generateTrajectory: stream");
            return EPP_ERR_HIP;
        }
        if (need > c.dcap) {
            if (c.d) (void)hipFree(c.d);
            c.d = nullptr;
            c.dcap = 0;
            if (hipMalloc(&c.d, need) != hipSuccess) {
                set_error("generateTrajectory: hipMalloc failed");
                return EPP_ERR_HIP;
            }
            c.dcap = need;
        }
        const size_t hneed = std::max(in_b, out_b);
        if (hneed > c.hcap) {
            if (c.h) (void)hipHostFree(c.h);
            c.h = nullptr;
            c.hcap = 0;
            if (hipHostMalloc(&c.h, hneed, 0) != hipSuccess) {
                set_error("generateTrajectory: hipHostMalloc failed");
                return EPP_ERR_HIP;
            }
            c.hcap = hneed;
        }
        // inputs, staged in pinned memory
        double* h_wp = (double*)c.h;
        std::memcpy(h_wp, wp, (size_t)n_wp * 24);
        double* h_va = h_wp + (size_t)n_wp * 3;
        for (int k = 0; k < 3; ++k) {
            h_va[k] = v0 ? v0[k] : 0.0;
            h_va[3 + k] = a0 ? a0[k] : 0.0;
        }
        h_va[6] = t0;
        int32_t* h_off = (int32_t*)(h_va + 7);
        h_off[0] = 0;
        h_off[1] = n_wp;
        int64_t* h_goff = (int64_t*)(h_off + 2);
        h_goff[0] = 0;  // global scratch offset of the track
        h_goff[1] = 0;  // row offset
        double* d_wp = (double*)c.d;
        double* d_va = d_wp + (size_t)n_wp * 3;
        double* d_t0 = d_va + 6;
        int32_t* d_off = (int32_t*)(d_va + 7);
        int64_t* d_goff = (int64_t*)(d_off + 2);
        int64_t* d_roff = d_goff + 1;
        double* d_T = (double*)(c.d + in_b);
        double* d_C = (double*)(c.d + in_b + a16((size_t)M * 8));
        double* d_scr = (double*)(c.d + in_b + a16((size_t)M * 8) + a16((size_t)M * 240));
        double* d_rows = (double*)(c.d + in_b + mid_b);
        int64_t* d_cnt = (int64_t*)(d_rows + (size_t)cap * 10);
        int32_t* d_status = (int32_t*)(d_cnt + 1);
        hipStream_t s = c.s;
        hipError_t e = hipMemcpyAsync(c.d, c.h, in_b, hipMemcpyHostToDevice, s);
        const size_t vert_doubles = (size_t)(M + 1) * (15 + 12) + M;
        if (lds) {
            const size_t shm = ((size_t)M * SegScratch::kSize + vert_doubles + 2) * sizeof(double);
            hipLaunchKernelGGL((k_minsnap<true>), dim3(1), dim3(kWave), shm, s, d_wp, d_off, 1, v_max, a_max, d_va,
                               d_va + 3, d_T, d_C, d_status, nullptr, nullptr);
        } else {
            hipLaunchKernelGGL((k_minsnap<false>), dim3(1), dim3(kWave), (vert_doubles + 2) * sizeof(double), s,
                               d_wp, d_off, 1, v_max, a_max, d_va, d_va + 3, d_T, d_C, d_status, d_scr, d_goff);
        }
        hipLaunchKernelGGL(k_sample_count, dim3(1), dim3(kWave), (size_t)(M + 2) * 8, s, d_T, d_off, 1, dt, d_cnt);
        hipLaunchKernelGGL(k_sample_rows, dim3(1), dim3(kWave), ((size_t)((M + 1) & ~1) + 3 * kRowChunk + 2) * 8, s,
                           d_T, d_C, d_off, 1, dt, d_t0, d_roff, d_rows, cap);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(c.h, d_rows, out_b, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            set_error(std::string("generateTrajectory: ") + hipGetErrorString(e));
            return EPP_ERR_HIP;
        }
        const int64_t count = *(const int64_t*)(c.h + (size_t)cap * 80);
        const int32_t status = *(const int32_t*)(c.h + (size_t)cap * 80 + 8);
        if (status != 0) {
            set_error(status == -2 ? "Segment times need to be greater than zero" : "min-snap solve failed");
            return EPP_ERR_RUNTIME;
        }
        if (count > cap) {  // host estimate short: once more with the exact size
            cap = count + 16;
            continue;
        }
        double* host_rows = (double*)std::malloc((size_t)std::max<int64_t>(count, 1) * 80);
        if (!host_rows) {
            set_error("generateTrajectory: out of host memory");
            return EPP_ERR_RUNTIME;
        }
        if (count > 0) std::memcpy(host_rows, c.h, (size_t)count * 80);
        *rows_out = host_rows;
        *n_rows = count;
        return EPP_OK;
    }
    set_error("generateTrajectory: row count");
    return EPP_ERR_RUNTIME;
}

}  // extern "C"

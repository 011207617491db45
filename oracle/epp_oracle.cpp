/*
 * epp_oracle.cpp — TEST INFRASTRUCTURE ONLY (see epp_oracle.h).
 *
 * A plain-C++ (no Eigen / Boost / OMPL) restatement of the reference's hot
 * path.  Every function cites the reference file:line it follows.  Compiled
 * with -O2 -ffp-contract=off so that no multiply-add is fused: the reference is
 * built by g++ for x86-64 without FMA, so every product and sum rounds
 * separately there too.
 *
 * Operation-order notes (the reason boolean results are bit-exact):
 *  - R = Rz(yaw) has exact zeros off the xy block, so every Eigen 3x3 product
 *    R^T (p - c) reduces to c*dx + s*dy, -s*dx + c*dy, dz regardless of Eigen's
 *    summation order (adding an exact +-0 never changes a nonzero sum).
 *  - The unqualified abs() in src/OBB.cpp:34 and src/Object.cpp:38 resolves to
 *    the double overload: Eigen/Core includes <emmintrin.h> on x86-64, whose
 *    mm_malloc.h includes libstdc++'s <stdlib.h> wrapper, which does
 *    `using std::abs;` at global scope (checked with g++ 11 in this container).
 *  - Boost.Geometry rtree `contains(point)` keeps boxes that strictly contain
 *    the point (bg::within point/box: min < p < max on every axis);
 *    `intersects(box)` is closed box overlap.  These are restated literally.
 */
#include "epp_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <queue>
#include <random>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// OBB primitives — src/OBB.cpp
// ---------------------------------------------------------------------------

// R^T (p - c) for R = Rz; rot is row-major R (R(i,k) = rot[3i+k]).
// Eigen: localPoint = rotation.transpose() * (point - center)   src/OBB.cpp:66
inline void to_local(const or_obb& o, const double p[3], double l[3]) {
    const double d0 = p[0] - o.center[0];
    const double d1 = p[1] - o.center[1];
    const double d2 = p[2] - o.center[2];
    // (R^T)(i,k) = R(k,i).  Zero entries of Rz make the third term an exact +-0.
    l[0] = (o.rot[0] * d0 + o.rot[3] * d1) + o.rot[6] * d2;
    l[1] = (o.rot[1] * d0 + o.rot[4] * d1) + o.rot[7] * d2;
    l[2] = (o.rot[2] * d0 + o.rot[5] * d1) + o.rot[8] * d2;
}

// OBB::checkCollisionWithPoint — src/OBB.cpp:63-91
bool obb_point_hit(const or_obb& o, const double p[3], double inflate) {
    double l[3];
    to_local(o, p, l);
    double h[3] = {o.half[0], o.half[1], o.half[2]};
    if (!o.filling) {  // shouldBeInflated(): type == "collision"  include/OBB.h:54-57
        h[0] = h[0] + inflate;
        h[1] = h[1] + inflate;
        h[2] = h[2] + inflate;
    }
    return (std::fabs(l[0]) <= h[0]) && (std::fabs(l[1]) <= h[1]) && (std::fabs(l[2]) <= h[2]);
}

// OBB::checkCollisionWithRay — src/OBB.cpp:10-61
bool obb_ray_hit(const or_obb& o, const double s[3], const double e[3], double inflate) {
    const bool hs = obb_point_hit(o, s, inflate);  // :13
    const bool he = obb_point_hit(o, e, inflate);  // :14
    if (hs || he) return true;
    double ls[3], le[3], ld[3];
    to_local(o, s, ls);  // :21
    to_local(o, e, le);  // :22
    for (int i = 0; i < 3; ++i) ld[i] = le[i] - ls[i];  // :23
    double tMin = 0.0, tMax = 1.0;
    for (int i = 0; i < 3; ++i) {
        const double ih = o.half[i] + inflate;  // :28 always inflated
        const double bmin = -ih, bmax = ih;
        if (std::fabs(ld[i]) < 1e-6) {                    // :34 (double abs, see header)
            if (ls[i] < bmin || ls[i] > bmax) return false;  // :37-40
        } else {
            const double invD = 1.0 / ld[i];  // :44  (1.0f promotes exactly to 1.0)
            const double t1 = (bmin - ls[i]) * invD;
            const double t2 = (bmax - ls[i]) * invD;
            const double tEntry = (t2 < t1) ? t2 : t1;  // std::min(t1,t2)
            const double tExit = (t1 < t2) ? t2 : t1;   // std::max(t1,t2)
            tMin = (tMin < tEntry) ? tEntry : tMin;     // std::max(tMin,tEntry)
            tMax = (tExit < tMax) ? tExit : tMax;       // std::min(tMax,tExit)
            if (tMin > tMax) return false;              // :54-57
        }
    }
    return 0 <= tMin && tMin <= 1 && 0 <= tMax && tMax <= 1;  // :60
}

// Boost rtree contains(point): bg::within(point, box) — strict interior.
inline bool aabb_strictly_contains(const or_obb& o, const double p[3]) {
    return o.aabb_lo[0] < p[0] && p[0] < o.aabb_hi[0] && o.aabb_lo[1] < p[1] &&
           p[1] < o.aabb_hi[1] && o.aabb_lo[2] < p[2] && p[2] < o.aabb_hi[2];
}

// Boost rtree intersects(box): closed overlap (not disjoint).
inline bool aabb_intersects(const or_obb& o, const double lo[3], const double hi[3]) {
    for (int i = 0; i < 3; ++i)
        if (o.aabb_hi[i] < lo[i] || hi[i] < o.aabb_lo[i]) return false;
    return true;
}

// OBB::getAABB — src/OBB.cpp:93-123
void obb_aabb(or_obb& o, double inflate) {
    static const double sx[8] = {-1, 1, 1, -1, -1, 1, 1, -1};  // :100
    static const double sy[8] = {-1, -1, 1, 1, -1, -1, 1, 1};  // :101
    static const double sz[8] = {-1, -1, -1, -1, 1, 1, 1, 1};  // :102
    double mn[3], mx[3];
    for (int j = 0; j < 8; ++j) {
        const double c[3] = {sx[j] * o.half[0], sy[j] * o.half[1], sz[j] * o.half[2]};  // :105
        double g[3];
        for (int i = 0; i < 3; ++i)  // rotation * corners + centerStacked  :110
            g[i] = ((o.rot[3 * i + 0] * c[0] + o.rot[3 * i + 1] * c[1]) + o.rot[3 * i + 2] * c[2]) +
                   o.center[i];
        for (int i = 0; i < 3; ++i) {
            if (j == 0) {
                mn[i] = g[i];
                mx[i] = g[i];
            } else {
                mn[i] = std::min(mn[i], g[i]);
                mx[i] = std::max(mx[i], g[i]);
            }
        }
    }
    if (!o.filling) {  // :117-121
        for (int i = 0; i < 3; ++i) {
            mn[i] = mn[i] - inflate;
            mx[i] = mx[i] + inflate;
        }
    }
    for (int i = 0; i < 3; ++i) {
        o.aabb_lo[i] = mn[i];
        o.aabb_hi[i] = mx[i];
    }
}

// ---------------------------------------------------------------------------
// World queries — src/World.cpp:80-162
// ---------------------------------------------------------------------------
inline double owner_inflate(const or_obb& o, double r_gate, double r_obst) {
    return o.is_gate ? r_gate : r_obst;  // src/World.cpp:89-90, :148,:155
}

bool point_valid(const or_obb* w, int n, double rg, double ro, const double p[3], bool canPass) {
    for (int i = 0; i < n; ++i) {
        const or_obb& o = w[i];
        if (!aabb_strictly_contains(o, p)) continue;  // rtree.query(contains(point))  :83
        if (o.filling && canPass) continue;           // :92-95
        if (obb_point_hit(o, p, owner_inflate(o, rg, ro))) return false;  // :97-100
    }
    return true;
}

bool point_valid_mindist(const or_obb* w, int n, const double p[3], double minDist) {
    for (int i = 0; i < n; ++i) {
        const or_obb& o = w[i];
        if (!aabb_strictly_contains(o, p)) continue;  // world-inflated boxes  :109
        if (o.filling) continue;                      // :116-119
        if (obb_point_hit(o, p, minDist)) return false;  // :121-125
    }
    return true;
}

bool ray_valid(const or_obb* w, int n, double rg, double ro, const double s[3], const double e[3],
               bool canPass) {
    double lo[3], hi[3];
    for (int i = 0; i < 3; ++i) {  // ray.rowwise().minCoeff()/maxCoeff()  :137-138
        lo[i] = std::min(s[i], e[i]);
        hi[i] = std::max(s[i], e[i]);
    }
    for (int i = 0; i < n; ++i) {
        const or_obb& o = w[i];
        if (!aabb_intersects(o, lo, hi)) continue;  // rtree.query(intersects(rayBox))  :143
        if (o.filling && canPass) continue;         // :150-153
        if (obb_ray_hit(o, s, e, owner_inflate(o, rg, ro))) return false;  // :157-160
    }
    return true;
}

// discrete32: OMPL RealVectorStateSpace::interpolate convention x = s + (e - s) * t,
// t = k/32, k = 1..32 (build-defined mode).
bool ray_valid_discrete32(const or_obb* w, int n, double rg, double ro, const double s[3],
                          const double e[3], bool canPass) {
    for (int k = 1; k <= 32; ++k) {
        const double t = (double)k / 32.0;
        double p[3];
        for (int i = 0; i < 3; ++i) p[i] = s[i] + (e[i] - s[i]) * t;
        if (!point_valid(w, n, rg, ro, p, canPass)) return false;
    }
    return true;
}

// ---------------------------------------------------------------------------
// min-snap — external/poly_traj
// ---------------------------------------------------------------------------
constexpr int N = 10;       // polynomial coefficients (trajectory_generator.cpp:17)
constexpr int HALF = N / 2;  // constraints per vertex

// computeBaseCoefficients — src/polynomial.cpp:145-160 (falling factorials, exact)
struct BaseCoeffs {
    double b[N][N];
    BaseCoeffs() {
        std::memset(b, 0, sizeof(b));
        for (int i = 0; i < N; ++i) b[0][i] = 1.0;
        const int DEG = N - 1;
        int order = DEG;
        for (int n = 1; n < N; ++n) {
            for (int i = DEG - order; i < N; ++i) b[n][i] = (order - DEG + i) * b[n - 1][i];
            order--;
        }
    }
};
const BaseCoeffs kB;

// Polynomial::baseCoeffsWithTime — polynomial.h:201-219
void base_coeffs_with_time(int k, double t, double* row) {
    for (int j = 0; j < N; ++j) row[j] = 0.0;
    row[k] = kB.b[k][k];
    if (std::fabs(t) < 2.220446049250313e-16) return;  // numeric_limits<double>::epsilon
    double tp = t;
    for (int j = k + 1; j < N; ++j) {
        row[j] = kB.b[k][j] * tp;
        tp = tp * t;
    }
}

// computeQuadraticCostJacobian — impl/polynomial_optimization_linear_impl.h:567-583
void cost_matrix(int derivative, double t, double* Q) {
    for (int i = 0; i < N * N; ++i) Q[i] = 0.0;
    for (int col = 0; col < N - derivative; ++col) {
        for (int row = 0; row < N - derivative; ++row) {
            const double exponent = (N - 1 - derivative) * 2 + 1 - row - col;
            Q[(N - 1 - row) * N + (N - 1 - col)] = kB.b[derivative][N - 1 - row] *
                                                   kB.b[derivative][N - 1 - col] *
                                                   std::pow(t, exponent) * 2.0 / exponent;
        }
    }
}

// LU with partial pivoting inverse (what Eigen's 5x5 .inverse() does).
bool inverse_lu(const double* M, int n, double* Minv) {
    std::vector<double> a(M, M + n * n);
    std::vector<int> perm(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = std::fabs(a[k * n + k]);
        for (int r = k + 1; r < n; ++r)
            if (std::fabs(a[r * n + k]) > best) {
                best = std::fabs(a[r * n + k]);
                p = r;
            }
        if (best == 0.0) return false;
        if (p != k) {
            for (int c = 0; c < n; ++c) std::swap(a[k * n + c], a[p * n + c]);
            std::swap(perm[k], perm[p]);
        }
        for (int r = k + 1; r < n; ++r) {
            a[r * n + k] /= a[k * n + k];
            for (int c = k + 1; c < n; ++c) a[r * n + c] -= a[r * n + k] * a[k * n + c];
        }
    }
    for (int col = 0; col < n; ++col) {
        std::vector<double> x(n);
        for (int i = 0; i < n; ++i) x[i] = (perm[i] == col) ? 1.0 : 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < i; ++j) x[i] -= a[i * n + j] * x[j];
        for (int i = n - 1; i >= 0; --i) {
            for (int j = i + 1; j < n; ++j) x[i] -= a[i * n + j] * x[j];
            x[i] /= a[i * n + i];
        }
        for (int i = 0; i < n; ++i) Minv[i * n + col] = x[i];
    }
    return true;
}

// Cholesky solve of SPD system A x = B (B: n x m, overwritten with x).
bool chol_solve(std::vector<double>& A, int n, std::vector<double>& B, int m) {
    for (int j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (int c = 0; c < m; ++c) {
        for (int i = 0; i < n; ++i) {
            double s = B[i * m + c];
            for (int k = 0; k < i; ++k) s -= A[i * n + k] * B[k * m + c];
            B[i * m + c] = s / A[i * n + i];
        }
        for (int i = n - 1; i >= 0; --i) {
            double s = B[i * m + c];
            for (int k = i + 1; k < n; ++k) s -= A[k * n + i] * B[k * m + c];
            B[i * m + c] = s / A[i * n + i];
        }
    }
    return true;
}

// splitmix64 (SURVEY §8d counter-based sampler)
inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

}  // namespace

// ===========================================================================
// extern "C"
// ===========================================================================
extern "C" {

// World::addGatePrivateOperation / addObstacle / addObject + Object::createFromDescription,
// translate, rotateZ (src/World.cpp:13-67, src/Object.cpp:11-85, src/PathPlanner.cpp:60-78)
int or_world_build(const or_obb_desc* gate_desc, const int32_t* gate_desc_off, int n_gate_types,
                   const or_obb_desc* obst_desc, int n_obst_desc, const double* gates,
                   int n_gates, const double* obstacles, int n_obstacles, double r_gate,
                   double r_obst, or_obb* out, int max_out) {
    int count = 0;
    auto build_object = [&](const double g_in[3], const double rot_in[3], const or_obb_desc* d,
                            int nd, int is_gate, double inflate) -> int {
        if (std::fabs(rot_in[0]) > 1e-6) return -2;  // Object.cpp:38-42
        if (std::fabs(rot_in[1]) > 1e-6) return -2;  // Object.cpp:43-47
        if (g_in[2] > 1e-6) return -3;               // Object.cpp:16-20
        const double g[3] = {g_in[0], g_in[1], g_in[2]};
        // globalCenter = 0 + translation  (Object.cpp:13, :54)
        const double gc[3] = {0.0 + g[0], 0.0 + g[1], 0.0 + g[2]};
        const double ca = std::cos(rot_in[2]);  // Object.cpp:69-70
        const double sa = std::sin(rot_in[2]);
        const double R[9] = {ca, -sa, 0.0, sa, ca, 0.0, 0.0, 0.0, 1.0};  // :72-75
        for (int k = 0; k < nd; ++k) {
            if (count >= max_out) return -1;
            or_obb& o = out[count++];
            std::memset(&o, 0, sizeof(o));
            for (int i = 0; i < 3; ++i) {
                o.half[i] = d[k].size[i] / 2;        // ConfigParserYAML.cpp:63
                o.center[i] = d[k].pos[i] + g[i];    // translate  Object.cpp:57
            }
            double rel[3];
            for (int i = 0; i < 3; ++i) rel[i] = o.center[i] - gc[i];  // :81
            for (int i = 0; i < 3; ++i)                                 // :82
                o.center[i] = ((R[3 * i + 0] * rel[0] + R[3 * i + 1] * rel[1]) + R[3 * i + 2] * rel[2]) +
                              gc[i];
            // obb.rotation = rotation * Identity (:83) == R exactly
            for (int i = 0; i < 9; ++i) o.rot[i] = R[i];
            o.filling = d[k].filling;
            o.is_gate = is_gate;
            obb_aabb(o, inflate);  // World::addObject -> getAABBs(inflateSize)  World.cpp:59-60
        }
        return 0;
    };
    for (int gi = 0; gi < n_gates; ++gi) {
        const double* row = gates + 7 * gi;
        const double pos[3] = {row[0], row[1], 0.0};  // gate(2) = 0 (PathPlanner.cpp:68, World.cpp:16)
        const double rot[3] = {row[3], row[4], row[5]};
        const int type = (int)row[6];                  // World.cpp:18
        if (type < 0 || type >= n_gate_types) return -4;
        const int rc = build_object(pos, rot, gate_desc + gate_desc_off[type],
                                    gate_desc_off[type + 1] - gate_desc_off[type], 1, r_gate);
        if (rc < 0) return rc;
    }
    for (int oi = 0; oi < n_obstacles; ++oi) {
        const double* row = obstacles + 6 * oi;
        const double pos[3] = {row[0], row[1], row[2]};  // World.cpp:49
        const double rot[3] = {row[3], row[4], row[5]};
        const int rc = build_object(pos, rot, obst_desc, n_obst_desc, 0, r_obst);
        if (rc < 0) return rc;
    }
    return count;
}

int or_point_valid(const or_obb* w, int n, double rg, double ro, const double p[3], int cp) {
    return point_valid(w, n, rg, ro, p, cp != 0) ? 1 : 0;
}
int or_point_valid_mindist(const or_obb* w, int n, const double p[3], double md) {
    return point_valid_mindist(w, n, p, md) ? 1 : 0;
}
int or_ray_valid(const or_obb* w, int n, double rg, double ro, const double s[3], const double e[3],
                 int cp) {
    return ray_valid(w, n, rg, ro, s, e, cp != 0) ? 1 : 0;
}

void or_check_states(const or_obb* w, int n, double rg, double ro, const double* xyz, int64_t ns,
                     int cp, uint8_t* valid) {
    for (int64_t i = 0; i < ns; ++i) valid[i] = point_valid(w, n, rg, ro, xyz + 3 * i, cp != 0);
}

void or_check_states_mindist(const or_obb* w, int n, const double* xyz, int64_t ns, double md,
                             uint8_t* valid) {
    for (int64_t i = 0; i < ns; ++i) valid[i] = point_valid_mindist(w, n, xyz + 3 * i, md);
}

void or_check_motions(const or_obb* w, int n, double rg, double ro, const double* s1,
                      const double* s2, int64_t ne, int cp, int mode, uint8_t* valid) {
    for (int64_t i = 0; i < ne; ++i)
        valid[i] = mode == 0 ? ray_valid(w, n, rg, ro, s1 + 3 * i, s2 + 3 * i, cp != 0)
                             : ray_valid_discrete32(w, n, rg, ro, s1 + 3 * i, s2 + 3 * i, cp != 0);
}

void or_check_states_mt(const or_obb* w, int n, double rg, double ro, const double* xyz,
                        int64_t ns, int cp, uint8_t* valid, int nt) {
    if (nt < 1) nt = 1;
    std::vector<std::thread> th;
    const int64_t chunk = (ns + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t b = t * chunk, e = std::min<int64_t>(ns, b + chunk);
        if (b >= e) break;
        th.emplace_back([=] { or_check_states(w, n, rg, ro, xyz + 3 * b, e - b, cp, valid + b); });
    }
    for (auto& x : th) x.join();
}

void or_check_motions_mt(const or_obb* w, int n, double rg, double ro, const double* s1,
                         const double* s2, int64_t ne, int cp, int mode, uint8_t* valid, int nt) {
    if (nt < 1) nt = 1;
    std::vector<std::thread> th;
    const int64_t chunk = (ne + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t b = t * chunk, e = std::min<int64_t>(ne, b + chunk);
        if (b >= e) break;
        th.emplace_back([=] {
            or_check_motions(w, n, rg, ro, s1 + 3 * b, s2 + 3 * b, e - b, cp, mode, valid + b);
        });
    }
    for (auto& x : th) x.join();
}

void or_sample_states(uint64_t seed, const double lo[3], const double hi[3], int64_t n, double* xyz) {
    for (int64_t i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) {
            const uint64_t r = splitmix64(seed ^ (uint64_t)(3 * i + d));
            const double u = (double)(r >> 11) * 0x1.0p-53;
            xyz[3 * i + d] = lo[d] + (hi[d] - lo[d]) * u;
        }
}

// estimateSegmentTimesNfabian — src/vertex.cpp:272-289 (magic constant 6.5, vertex.h:139-141)
void or_segment_times(const double* wp, int n_wp, int dim, double v_max, double a_max,
                      double* times) {
    const double magic = 6.5;
    for (int i = 0; i + 1 < n_wp; ++i) {
        double sq = 0.0;  // (end - start).norm(): sqrt of sum of squares, left to right
        for (int d = 0; d < dim; ++d) {
            const double df = wp[(i + 1) * dim + d] - wp[i * dim + d];
            sq += df * df;
        }
        const double distance = std::sqrt(sq);
        times[i] = distance / v_max * 2 * (1.0 + magic * v_max / a_max * std::exp(-distance / v_max * 2));
    }
}

void or_mapping_matrix(double t, double* A) {
    // setupMappingMatrix — impl/...linear_impl.h:111-121
    for (int i = 0; i < HALF; ++i) {
        base_coeffs_with_time(i, 0.0, A + i * N);
        base_coeffs_with_time(i, t, A + (i + HALF) * N);
    }
}

void or_invert_mapping(const double* A, double* Ai) {
    // invertMappingMatrix — impl/...linear_impl.h:142-179 (Schur complement)
    double Dm[HALF * HALF], Dinv[HALF * HALF], C[HALF * HALF], Adiag_inv[HALF];
    for (int i = 0; i < HALF; ++i) Adiag_inv[i] = 1.0 / A[i * N + i];  // cwiseInverse
    for (int r = 0; r < HALF; ++r)
        for (int c = 0; c < HALF; ++c) {
            C[r * HALF + c] = A[(r + HALF) * N + c];
            Dm[r * HALF + c] = A[(r + HALF) * N + c + HALF];
        }
    inverse_lu(Dm, HALF, Dinv);
    for (int i = 0; i < N * N; ++i) Ai[i] = 0.0;
    for (int r = 0; r < HALF; ++r) {
        Ai[r * N + r] = Adiag_inv[r];
        for (int c = 0; c < HALF; ++c) Ai[(r + HALF) * N + c + HALF] = Dinv[r * HALF + c];
    }
    // -D_inv * C * A_inv  (A_inv diagonal): (D_inv*C)(r,c) * Ainv(c)
    for (int r = 0; r < HALF; ++r)
        for (int c = 0; c < HALF; ++c) {
            double s = 0.0;
            for (int k = 0; k < HALF; ++k) s += Dinv[r * HALF + k] * C[k * HALF + c];
            Ai[(r + HALF) * N + c] = -s * Adiag_inv[c];
        }
}

double or_poly_eval(const double* c, double t, int k) {
    // Polynomial::evaluate(t, derivative) — polynomial.h:136-149
    if (k >= N) return 0.0;
    double r = kB.b[k][N - 1] * c[N - 1];
    for (int j = N - 2; j >= k; --j) {
        r *= t;
        r += kB.b[k][j] * c[j];
    }
    return r;
}

int or_minsnap_solve(const uint8_t* fixed_mask, const double* fixed_val, int n_vertices, int dim,
                     const double* times, int deriv, double* coeffs) {
    const int M = n_vertices - 1;
    if (M < 1) return -1;
    // updateSegmentTimes — impl :285-305
    std::vector<double> Ainv((size_t)M * N * N), Hs((size_t)M * N * N);
    for (int i = 0; i < M; ++i) {
        if (!(times[i] > 0)) return -1;  // CHECK_GT(segment_time, 0)  :297
        double Q[N * N], A[N * N];
        cost_matrix(deriv, times[i], Q);
        or_mapping_matrix(times[i], A);
        or_invert_mapping(A, &Ainv[(size_t)i * N * N]);
        // constructR: H = Ai^T * Q * Ai  — impl :307-336
        const double* Ai = &Ainv[(size_t)i * N * N];
        double QA[N * N];
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < N; ++c) {
                double s = 0.0;
                for (int k = 0; k < N; ++k) s += Q[r * N + k] * Ai[k * N + c];
                QA[r * N + c] = s;
            }
        for (int r = 0; r < N; ++r)
            for (int c = 0; c < N; ++c) {
                double s = 0.0;
                for (int k = 0; k < N; ++k) s += Ai[k * N + r] * QA[k * N + c];
                Hs[(size_t)i * N * N + r * N + c] = s;
            }
    }
    // setupConstraintReorderingMatrix — impl :181-260.  all_constraints lists
    // vertex 0 once, inner vertices twice, the last vertex once, derivatives 0..4.
    // fixed/free sets are ordered by (vertex_idx, constraint_idx).
    std::vector<int> col_of((size_t)n_vertices * HALF);
    int n_fixed = 0, n_free = 0;
    for (int v = 0; v < n_vertices; ++v)
        for (int k = 0; k < HALF; ++k)
            if (fixed_mask[v * HALF + k]) col_of[v * HALF + k] = n_fixed++;
    for (int v = 0; v < n_vertices; ++v)
        for (int k = 0; k < HALF; ++k)
            if (!fixed_mask[v * HALF + k]) col_of[v * HALF + k] = n_fixed + n_free++;
    const int n_all = n_fixed + n_free;
    // segment i rows: [vertex i derivs 0..4 ; vertex i+1 derivs 0..4]
    auto row_col = [&](int seg, int r) {
        const int v = seg + (r >= HALF ? 1 : 0);
        return col_of[v * HALF + (r % HALF)];
    };
    std::vector<double> dall((size_t)n_all * dim, 0.0);  // [d_f ; d_p] per dim (column-major by dim)
    for (int v = 0; v < n_vertices; ++v)
        for (int k = 0; k < HALF; ++k)
            if (fixed_mask[v * HALF + k])
                for (int d = 0; d < dim; ++d)
                    dall[(size_t)d * n_all + col_of[v * HALF + k]] = fixed_val[(v * HALF + k) * dim + d];
    if (n_free > 0) {
        // R = C^T H C; Rpp d_p = -Rpf d_f   — impl :338-379 (reference: SparseQR/COLAMD;
        // here a dense Cholesky, R_pp is SPD)
        std::vector<double> R((size_t)n_all * n_all, 0.0);
        for (int i = 0; i < M; ++i)
            for (int r = 0; r < N; ++r)
                for (int c = 0; c < N; ++c)
                    R[(size_t)row_col(i, r) * n_all + row_col(i, c)] += Hs[(size_t)i * N * N + r * N + c];
        std::vector<double> Rpp((size_t)n_free * n_free), rhs((size_t)n_free * dim);
        for (int r = 0; r < n_free; ++r)
            for (int c = 0; c < n_free; ++c)
                Rpp[(size_t)r * n_free + c] = R[(size_t)(n_fixed + r) * n_all + n_fixed + c];
        for (int d = 0; d < dim; ++d)
            for (int r = 0; r < n_free; ++r) {
                double s = 0.0;
                for (int c = 0; c < n_fixed; ++c)
                    s += R[(size_t)(n_fixed + r) * n_all + c] * dall[(size_t)d * n_all + c];
                rhs[(size_t)r * dim + d] = -s;
            }
        if (!chol_solve(Rpp, n_free, rhs, dim)) return -2;
        for (int d = 0; d < dim; ++d)
            for (int r = 0; r < n_free; ++r) dall[(size_t)d * n_all + n_fixed + r] = rhs[(size_t)r * dim + d];
    }
    // updateSegmentsFromCompactConstraints — impl :262-283
    for (int i = 0; i < M; ++i)
        for (int d = 0; d < dim; ++d) {
            double nd[N];
            for (int r = 0; r < N; ++r) nd[r] = dall[(size_t)d * n_all + row_col(i, r)];
            const double* Ai = &Ainv[(size_t)i * N * N];
            for (int r = 0; r < N; ++r) {
                double s = 0.0;
                for (int k = 0; k < N; ++k) s += Ai[r * N + k] * nd[k];
                coeffs[((size_t)i * dim + d) * N + r] = s;
            }
        }
    return n_free;
}

int or_minsnap_track(const double* wp, int n_wp, double v_max, double a_max, const double v0[3],
                     const double a0[3], double* seg_times, double* coeffs) {
    if (n_wp < 2) return -3;  // std::invalid_argument  trajectory_generator.cpp:21-25
    const int dim = 3;
    std::vector<uint8_t> mask((size_t)n_wp * HALF, 0);
    std::vector<double> val((size_t)n_wp * HALF * dim, 0.0);
    // start vertex: makeStartOrEnd([p0; v0; a0], SNAP) — src/vertex.cpp:146-170
    for (int k = 0; k < HALF; ++k) mask[k] = 1;
    for (int d = 0; d < dim; ++d) {
        val[(0 * HALF + 0) * dim + d] = wp[d];
        val[(0 * HALF + 1) * dim + d] = v0[d];
        val[(0 * HALF + 2) * dim + d] = a0[d];
    }
    for (int v = 1; v + 1 < n_wp; ++v) {  // middle: POSITION only
        mask[v * HALF + 0] = 1;
        for (int d = 0; d < dim; ++d) val[(v * HALF + 0) * dim + d] = wp[v * dim + d];
    }
    const int last = n_wp - 1;  // end: makeStartOrEnd(p_end, SNAP): vel/acc/jerk/snap 0
    for (int k = 0; k < HALF; ++k) mask[last * HALF + k] = 1;
    for (int d = 0; d < dim; ++d) val[(last * HALF + 0) * dim + d] = wp[last * dim + d];
    or_segment_times(wp, n_wp, dim, v_max, a_max, seg_times);
    return or_minsnap_solve(mask.data(), val.data(), n_wp, dim, seg_times, 4, coeffs);
}

// A batch of independent tracks (the CPU side of BASELINE C5's batched refit): track k is
// wp[off[k] .. off[k+1]) and gets one or_minsnap_track call (v0 = a0 = 0), its segment
// times at T + (off[k] - k) and coefficients at C + (off[k] - k) * 30, on nt threads
// (contiguous ranges of tracks).  status[k] = or_minsnap_track's return value.
void or_minsnap_batch_mt(const double* wp, const int32_t* off, int n_tracks, double v_max, double a_max,
                         double* T, double* C, int32_t* status, int nt) {
    if (nt < 1) nt = 1;
    const double z[3] = {0.0, 0.0, 0.0};
    auto run = [=](int b, int e) {
        for (int k = b; k < e; ++k) {
            const int64_t seg0 = (int64_t)off[k] - k;
            status[k] = or_minsnap_track(wp + 3 * (int64_t)off[k], off[k + 1] - off[k], v_max, a_max, z, z,
                                         T + seg0, C + seg0 * 30);
        }
    };
    std::vector<std::thread> th;
    const int chunk = (n_tracks + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int b = t * chunk, e = std::min(n_tracks, b + chunk);
        if (b >= e) break;
        th.emplace_back(run, b, e);
    }
    for (auto& x : th) x.join();
}

int64_t or_sample_traj(const double* T, const double* coeffs, int M, double dt, double t0,
                       double* rows, int64_t max_rows) {
    // Trajectory::evaluateRange(min_time=0, max_time, dt, k) — src/trajectory.cpp:81-141
    double t_end = 0.0;  // Trajectory::addSegments: max_time_ += segment.getTime()  trajectory.h:63-70
    for (int i = 0; i < M; ++i) t_end += T[i];
    const double t_start = 0.0;
    double acc = 0.0;
    int i = 0;
    for (i = 0; i < M; ++i) {
        acc += T[i];
        if (acc > t_start) break;
    }
    if (t_start > acc) return 0;
    if (i >= M) i = M - 1;  // not reachable for T[0] > 0
    acc -= T[i];
    double tis = t_start - acc;
    int64_t n = 0;
    while (acc < t_end) {
        if (tis > T[i]) {
            tis = tis - T[i];
            i++;
            if (i >= M) break;
            continue;
        }
        if (rows && n < max_rows) {
            double* row = rows + n * 10;
            for (int d = 0; d < 3; ++d) {
                const double* c = coeffs + ((size_t)i * 3 + d) * N;
                row[3 * d + 0] = or_poly_eval(c, tis, 0);
                row[3 * d + 1] = or_poly_eval(c, tis, 1);
                row[3 * d + 2] = or_poly_eval(c, tis, 2);
            }
            row[9] = acc + t0;  // sampling_times[i] + startTimeOffset  trajectory_generator.cpp:95
        }
        n++;
        tis += dt;
        acc += dt;
    }
    return n;
}

int64_t or_generate_trajectory(const double* wp, int n_wp, double v_max, double a_max, double dt,
                               double t0, const double v0[3], const double a0[3], double* rows,
                               int64_t max_rows) {
    if (n_wp < 2) return -3;
    std::vector<double> T(n_wp - 1), C((size_t)(n_wp - 1) * 3 * N);
    const int rc = or_minsnap_track(wp, n_wp, v_max, a_max, v0, a0, T.data(), C.data());
    if (rc < 0) return rc;
    return or_sample_traj(T.data(), C.data(), n_wp - 1, dt, t0, rows, max_rows);
}

void or_random_vertices(int n_segments, int dim, double pos_min, double pos_max, uint64_t seed,
                        double* out) {
    // createRandomVertices — src/vertex.cpp:27-82
    std::mt19937 gen((std::mt19937::result_type)seed);
    std::vector<std::uniform_real_distribution<double>> dist(dim);
    for (int i = 0; i < dim; ++i) dist[i] = std::uniform_real_distribution<double>(pos_min, pos_max);
    const double min_distance = 0.2;
    std::vector<double> last(dim), pos(dim);
    for (int i = 0; i < dim; ++i) last[i] = dist[i](gen);
    for (int i = 0; i < dim; ++i) out[i] = last[i];
    for (int v = 1; v <= n_segments; ++v) {
        while (true) {
            for (int d = 0; d < dim; ++d) pos[d] = dist[d](gen);
            double sq = 0.0;
            for (int d = 0; d < dim; ++d) sq += (pos[d] - last[d]) * (pos[d] - last[d]);
            if (std::sqrt(sq) > min_distance) break;
        }
        for (int d = 0; d < dim; ++d) out[v * dim + d] = pos[d];
        last = pos;
    }
}

}  // extern "C"

// ===== CPU restatement of this build's batch planner ====================================
// TEST INFRASTRUCTURE: the CPU baseline of "full plan ms/track" (the same planner on host
// cores) and the checker of PathPlanner::planOnce (paths must be EQUAL: same
// counter-RNG samples, exact k-NN with the same tie rule, the same A* and shortcut).  It
// restates efficient-path-planner_amd/csrc/host_planner.cpp:planOnce and the k-NN /
// compaction contracts of include/epp.h, not the reference (OMPL's planners are unseeded).
namespace {

struct KnnGridCpu {
    double lo[3], h;
    int n[3];
    std::vector<int> start, idx;
};

// Exact k nearest neighbours (squared distance ((dx*dx + dy*dy) + dz*dz), ties to the
// lower index, self excluded) by expanding cube shells of a uniform grid.
void knn_cpu(const double* p, int n, int k, int32_t* nbr, int threads) {
    KnnGridCpu g;
    double hi[3];
    for (int d = 0; d < 3; ++d) {
        g.lo[d] = hi[d] = n ? p[d] : 0.0;
        for (int i = 1; i < n; ++i) {
            g.lo[d] = std::min(g.lo[d], p[3 * i + d]);
            hi[d] = std::max(hi[d], p[3 * i + d]);
        }
    }
    double vol = 1.0;
    for (int d = 0; d < 3; ++d) vol *= std::max(hi[d] - g.lo[d], 1e-9);
    g.h = std::cbrt(vol * 2.0 / std::max(n, 1));  // ~2 nodes per cell
    if (!(g.h > 0)) g.h = 1.0;
    size_t cells = 1;
    for (int d = 0; d < 3; ++d) {
        g.n[d] = std::max(1, std::min(1024, (int)((hi[d] - g.lo[d]) / g.h) + 1));
        cells *= g.n[d];
    }
    auto cell_of = [&](const double* q, int* c) {
        for (int d = 0; d < 3; ++d) c[d] = std::min(g.n[d] - 1, std::max(0, (int)((q[d] - g.lo[d]) / g.h)));
    };
    g.start.assign(cells + 1, 0);
    std::vector<int> cid(n);
    for (int i = 0; i < n; ++i) {
        int c[3];
        cell_of(p + 3 * i, c);
        cid[i] = (c[2] * g.n[1] + c[1]) * g.n[0] + c[0];
        ++g.start[cid[i] + 1];
    }
    for (size_t c = 0; c < cells; ++c) g.start[c + 1] += g.start[c];
    g.idx.resize(n);
    {
        std::vector<int> fill(g.start.begin(), g.start.end() - 1);
        for (int i = 0; i < n; ++i) g.idx[fill[cid[i]]++] = i;
    }
    auto work = [&](int b, int e) {
        std::vector<std::pair<double, int>> best;
        for (int i = b; i < e; ++i) {
            const double* q = p + 3 * i;
            int c[3];
            cell_of(q, c);
            best.clear();
            const int rmax = std::max(g.n[0], std::max(g.n[1], g.n[2]));
            for (int r = 0; r <= rmax; ++r) {
                for (int z = c[2] - r; z <= c[2] + r; ++z) {
                    if (z < 0 || z >= g.n[2]) continue;
                    for (int y = c[1] - r; y <= c[1] + r; ++y) {
                        if (y < 0 || y >= g.n[1]) continue;
                        for (int x = c[0] - r; x <= c[0] + r; ++x) {
                            if (x < 0 || x >= g.n[0]) continue;
                            if (std::max(std::abs(x - c[0]), std::max(std::abs(y - c[1]), std::abs(z - c[2]))) != r)
                                continue;  // only the shell of radius r
                            const int cell = (z * g.n[1] + y) * g.n[0] + x;
                            for (int t = g.start[cell]; t < g.start[cell + 1]; ++t) {
                                const int j = g.idx[t];
                                if (j == i) continue;
                                const double dx = p[3 * j] - q[0], dy = p[3 * j + 1] - q[1], dz = p[3 * j + 2] - q[2];
                                best.push_back({(dx * dx + dy * dy) + dz * dz, j});
                            }
                        }
                    }
                }
                if ((int)best.size() >= k) {
                    std::nth_element(best.begin(), best.begin() + (k - 1), best.end());
                    const double dk = best[k - 1].first;
                    // a node beyond shell r is at least r cells away along some axis
                    const double reach = (double)r * g.h;
                    if (reach * reach > dk) break;
                }
            }
            std::sort(best.begin(), best.end());  // (distance, index): ties to the lower index
            for (int c2 = 0; c2 < k; ++c2) nbr[(size_t)i * k + c2] = c2 < (int)best.size() ? best[c2].second : -1;
        }
    };
    threads = std::max(1, threads);
    std::vector<std::thread> th;
    const int chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const int b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back(work, b, e);
    }
    for (auto& x : th) x.join();
}

double norm3(double x, double y, double z) { return std::sqrt((x * x + y * y) + z * z); }

}  // namespace

int or_plan_once(const or_obb* w, int nw, double rg, double ro, const double lo[3], const double hi[3],
                 const double start[3], const double goal[3], int64_t samples, uint64_t seed, int k, int can_pass,
                 int threads, double* path, int cap, int64_t* stats) {
    // 1. samples, StateValidator check, ordered compaction; nodes = start, goal, valid samples
    std::vector<double> xyz((size_t)samples * 3);
    or_sample_states(seed, lo, hi, samples, xyz.data());
    std::vector<uint8_t> ok((size_t)samples);
    or_check_states_mt(w, nw, rg, ro, xyz.data(), samples, can_pass, ok.data(), threads);
    std::vector<double> nodes = {start[0], start[1], start[2], goal[0], goal[1], goal[2]};
    for (int64_t i = 0; i < samples; ++i)
        if (ok[i]) nodes.insert(nodes.end(), {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]});
    const int n = (int)(nodes.size() / 3);
    // 2. k-NN edges, MotionValidator check, failed motions -> -1
    std::vector<int32_t> nbr((size_t)n * k);
    knn_cpu(nodes.data(), n, k, nbr.data(), threads);
    const size_t m = (size_t)n * k;
    std::vector<double> e1(m * 3), e2(m * 3);
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < k; ++c) {
            const size_t e = (size_t)i * k + c;
            const int j = nbr[e] >= 0 ? nbr[e] : i;
            for (int d = 0; d < 3; ++d) {
                e1[3 * e + d] = nodes[3 * i + d];
                e2[3 * e + d] = nodes[3 * j + d];
            }
        }
    std::vector<uint8_t> ev(m);
    or_check_motions_mt(w, nw, rg, ro, e1.data(), e2.data(), (int64_t)m, can_pass, 0, ev.data(), threads);
    int64_t n_valid_edges = 0;
    for (size_t e = 0; e < m; ++e) {
        if (!ev[e]) nbr[e] = -1;
        n_valid_edges += nbr[e] >= 0;
    }
    if (stats) {
        stats[0] = samples;
        stats[1] = n - 2;
        stats[2] = (int64_t)m;
        stats[3] = n_valid_edges;
    }
    // 3. A* (forward k-NN edges, then the symmetrised graph), start = 0, goal = 1
    auto nd = [&](int v, int d) { return nodes[3 * v + d]; };
    auto dist_to = [&](int v, const double* q) { return norm3(nd(v, 0) - q[0], nd(v, 1) - q[1], nd(v, 2) - q[2]); };
    const double gp[3] = {nd(1, 0), nd(1, 1), nd(1, 2)};
    std::vector<double> dist(n);
    std::vector<int> prev(n);
    std::vector<uint8_t> closed(n);
    std::vector<int32_t> roff, radj;
    using QE = std::pair<double, int>;
    auto astar = [&](bool with_reverse) {
        std::fill(dist.begin(), dist.end(), std::numeric_limits<double>::infinity());
        std::fill(prev.begin(), prev.end(), -1);
        std::fill(closed.begin(), closed.end(), 0);
        std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
        dist[0] = 0.0;
        q.push({dist_to(0, gp), 0});
        auto relax = [&](int u, const double* pu, int v) {
            if (closed[v]) return;
            const double nd2 = dist[u] + dist_to(v, pu);
            if (nd2 < dist[v]) {
                dist[v] = nd2;
                prev[v] = u;
                q.push({nd2 + dist_to(v, gp), v});
            }
        };
        while (!q.empty()) {
            const int u = q.top().second;
            q.pop();
            if (closed[u]) continue;
            closed[u] = 1;
            if (u == 1) return true;
            const double pu[3] = {nd(u, 0), nd(u, 1), nd(u, 2)};
            for (int c = 0; c < k; ++c) {
                const int v = nbr[(size_t)u * k + c];
                if (v >= 0) relax(u, pu, v);
            }
            if (with_reverse)
                for (int32_t r = roff[u]; r < roff[u + 1]; ++r) relax(u, pu, radj[r]);
        }
        return false;
    };
    const bool forward = astar(false);
    if (stats) stats[4] = forward ? 0 : 1;
    if (!forward) {
        roff.assign(n + 1, 0);
        for (size_t e = 0; e < m; ++e)
            if (nbr[e] >= 0) ++roff[nbr[e] + 1];
        for (int i = 0; i < n; ++i) roff[i + 1] += roff[i];
        radj.resize(roff[n]);
        std::vector<int32_t> fill(roff.begin(), roff.end() - 1);
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < k; ++c) {
                const size_t e = (size_t)i * k + c;
                if (nbr[e] >= 0) radj[fill[nbr[e]]++] = i;
            }
        astar(true);
    }
    if (prev[1] < 0) return 0;
    std::vector<int> chain;
    for (int v = 1; v >= 0; v = prev[v]) chain.push_back(v);
    std::reverse(chain.begin(), chain.end());
    // 4. greedy shortcut over one batch of all vertex-pair ray checks
    const size_t L = chain.size();
    std::vector<std::vector<uint8_t>> vis(L, std::vector<uint8_t>(L, 0));
    for (size_t i = 0; i < L; ++i)
        for (size_t j = i + 2; j < L; ++j) {
            const double a[3] = {nd(chain[i], 0), nd(chain[i], 1), nd(chain[i], 2)};
            const double b[3] = {nd(chain[j], 0), nd(chain[j], 1), nd(chain[j], 2)};
            vis[i][j] = (uint8_t)or_ray_valid(w, nw, rg, ro, a, b, can_pass);
        }
    std::vector<int> out = {chain[0]};
    if (L >= 3) {
        size_t cur = 0;
        while (cur + 1 < L) {
            size_t nxt = cur + 1;
            for (size_t j = L - 1; j > cur + 1; --j)
                if (vis[cur][j]) {
                    nxt = j;
                    break;
                }
            out.push_back(chain[nxt]);
            cur = nxt;
        }
    } else {
        out = chain;
    }
    if ((int)out.size() > cap) return -1;
    for (size_t i = 0; i < out.size(); ++i)
        for (int d = 0; d < 3; ++d) path[3 * i + d] = nd(out[i], d);
    return (int)out.size();
}

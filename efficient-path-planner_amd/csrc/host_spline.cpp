// host_spline.cpp — epp::TrajInterpolation, the "spline" trajectory type
// (src/TrajInterpolation.cpp:1-133).  Restates Eigen's unsupported Splines module for the
// one case the reference uses: degree-3 interpolation of 3-D points at chord-length
// parameters.  Knots by averaging (Eigen KnotAveraging), basis functions by the
// triangular de Boor scheme (Piegl & Tiller A2.2, as Eigen's BasisFunctions), control
// points from the collocation system (Eigen: Householder QR; here LU with partial
// pivoting -- the same solution up to rounding).  Host code: a few dozen points.
#include <algorithm>
#include <array>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "epp/TrajInterpolation.h"

namespace epp {
namespace {

constexpr int kDeg = 3;

struct Spline3 {
    std::vector<double> knots;
    std::vector<std::array<double, 3>> ctrl;

    // Eigen Spline::Span: the knot span holding u
    long span(double u) const {
        if (u <= knots[0]) return kDeg;
        const auto it = std::upper_bound(knots.begin() + kDeg - 1, knots.end() - kDeg - 1, u);
        return (long)(it - knots.begin()) - 1;
    }
    std::array<double, kDeg + 1> basis(double u, long i) const {
        std::array<double, kDeg + 1> left{}, right{}, n{};
        for (int k = 1; k <= kDeg; ++k) {
            left[k] = u - knots[i + 1 - k];
            right[k] = knots[i + k] - u;
        }
        n[0] = 1.0;
        for (int j = 1; j <= kDeg; ++j) {
            double saved = 0.0;
            for (int r = 0; r < j; ++r) {
                const double tmp = n[r] / (right[r + 1] + left[j - r]);
                n[r] = saved + right[r + 1] * tmp;
                saved = left[j - r] * tmp;
            }
            n[j] = saved;
        }
        return n;
    }
    Vec3 operator()(double u) const {
        const long i = span(u);
        const auto n = basis(u, i);
        Vec3 p;
        for (int d = 0; d < 3; ++d) {
            double acc = 0.0;
            for (int k = 0; k <= kDeg; ++k) acc += ctrl[i - kDeg + k][d] * n[k];
            p[d] = acc;
        }
        return p;
    }
};

// chord-length parameters in [0, 1] (TrajInterpolation.cpp:4-16)
std::vector<double> chordParams(const std::vector<Vec3>& path) {
    std::vector<double> t(path.size());
    t[0] = 0;
    for (size_t i = 1; i < path.size(); ++i) t[i] = t[i - 1] + (path[i] - path[i - 1]).norm();
    const double last = t.back();
    for (double& v : t) v /= last;
    return t;
}

// SplineFitting<Spline3d>::Interpolate(points, 3, t)
Spline3 fit(const std::vector<double>& t, const std::vector<Vec3>& pts) {
    const long n = (long)pts.size();
    if (n < kDeg + 1) throw std::invalid_argument("spline trajectory: needs at least 4 waypoints");
    Spline3 s;
    s.knots.assign(n + kDeg + 1, 0.0);
    for (long j = 1; j < n - kDeg; ++j) s.knots[j + kDeg] = ((t[j] + t[j + 1]) + t[j + 2]) / 3.0;
    for (long j = 0; j <= kDeg; ++j) s.knots[n + j] = 1.0;
    // collocation matrix, row-major n x n, and the right-hand sides
    std::vector<double> A((size_t)(n * n), 0.0);
    std::vector<std::array<double, 3>> b(n);
    A[0] = 1.0;
    A[(size_t)(n * n - 1)] = 1.0;
    for (long i = 1; i < n - 1; ++i) {
        const long sp = s.span(t[i]);
        const auto nb = s.basis(t[i], sp);
        for (int k = 0; k <= kDeg; ++k) A[(size_t)(i * n + sp - kDeg + k)] = nb[k];
    }
    for (long i = 0; i < n; ++i) b[i] = {pts[i].x, pts[i].y, pts[i].z};
    // LU with partial pivoting
    for (long c = 0; c < n; ++c) {
        long piv = c;
        for (long r = c + 1; r < n; ++r)
            if (std::abs(A[(size_t)(r * n + c)]) > std::abs(A[(size_t)(piv * n + c)])) piv = r;
        if (A[(size_t)(piv * n + c)] == 0.0) throw std::runtime_error("spline trajectory: singular collocation matrix");
        if (piv != c) {
            for (long k = 0; k < n; ++k) std::swap(A[(size_t)(c * n + k)], A[(size_t)(piv * n + k)]);
            std::swap(b[c], b[piv]);
        }
        for (long r = c + 1; r < n; ++r) {
            const double f = A[(size_t)(r * n + c)] / A[(size_t)(c * n + c)];
            if (f == 0.0) continue;
            for (long k = c; k < n; ++k) A[(size_t)(r * n + k)] -= f * A[(size_t)(c * n + k)];
            for (int d = 0; d < 3; ++d) b[r][d] -= f * b[c][d];
        }
    }
    s.ctrl.assign(n, {0.0, 0.0, 0.0});
    for (long r = n - 1; r >= 0; --r)
        for (int d = 0; d < 3; ++d) {
            double v = b[r][d];
            for (long k = r + 1; k < n; ++k) v -= A[(size_t)(r * n + k)] * s.ctrl[k][d];
            s.ctrl[r][d] = v / A[(size_t)(r * n + r)];
        }
    return s;
}

// numSamples = int(maxT / dt) + 1 points at u = i / (numSamples - 1) (TrajInterpolation.cpp:30-42)
std::vector<Vec3> sample(const Spline3& s, double maxT, double dt) {
    const int m = static_cast<int>(maxT / dt) + 1;
    if (m < 1) return {};
    std::vector<Vec3> out(m);
    for (int i = 0; i < m; ++i) out[i] = s(m > 1 ? static_cast<double>(i) / (m - 1) : 0.0);
    return out;
}

Matrix rows(const std::vector<Vec3>& pts, const std::vector<double>& times, double t0) {
    Matrix m(pts.size(), 10, 0.0);
    for (size_t i = 0; i < pts.size(); ++i) {
        m(i, 0) = pts[i].x;
        m(i, 3) = pts[i].y;
        m(i, 6) = pts[i].z;
        m(i, 9) = times[i] + t0;
    }
    return m;
}

// TrajInterpolation.cpp:71-94
double segmentTime(const Vec3& p1, const Vec3& p2, double v_start, double v_max, double a_max) {
    const double d = (p1 - p2).norm();
    if (d == 0) return 0;
    double t_acc = (v_max - v_start) / a_max;
    const double d_acc = v_start * t_acc + 0.5 * a_max * t_acc * t_acc;
    if (d_acc >= d / 2) {
        t_acc = (-v_start + std::sqrt(v_start * v_start + 2 * a_max * d / 2)) / a_max;
        return 2 * t_acc;
    }
    t_acc = (v_max - v_start) / a_max;
    const double t_dec = (v_max - 0) / a_max;
    const double t_const = (d - 2 * d_acc) / v_max;
    return t_acc + t_const + t_dec;
}

}  // namespace

Matrix TrajInterpolation::interpolateTraj(const std::vector<Vec3>& path, double maxT, double advancedTime,
                                          double dt) const {
    const std::vector<Vec3> pts = sample(fit(chordParams(path), path), maxT - advancedTime, dt);
    std::vector<double> times(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) times[i] = (double)i * dt;
    return rows(pts, times, advancedTime);
}

Matrix TrajInterpolation::interpolateTrajMaxVel(const std::vector<Vec3>& path, double v_start, double v_max,
                                                double a_max, double advancedTime, double dt) const {
    const std::vector<Vec3> pts = sample(fit(chordParams(path), path), 15 - advancedTime, dt);
    std::vector<double> times{0}, vel{v_start};
    for (size_t i = 1; i < pts.size(); ++i) {
        times.push_back(times[i - 1] + segmentTime(pts[i - 1], pts[i], vel[i - 1], v_max, a_max));
        vel.push_back(v_max);
    }
    times.resize(pts.size());
    return rows(pts, times, advancedTime);
}

}  // namespace epp

// C ABI (include/epp.h): the "spline" trajectory with host buffers.
#include <cstdlib>
#include <cstring>

#include "epp.h"
#include "epp_internal.h"

extern "C" epp_status epp_spline_trajectory_host(const double* wp, int32_t n_wp, double max_t, double t0, double dt,
                                                 double** rows_out, int64_t* n_rows) {
    if (!rows_out || !n_rows || n_wp < 0 || (n_wp > 0 && !wp) || !(dt > 0)) {
        epp::set_error("spline trajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *rows_out = nullptr;
    *n_rows = 0;
    std::vector<epp::Vec3> w;
    for (int32_t i = 0; i < n_wp; ++i) w.emplace_back(wp[3 * i], wp[3 * i + 1], wp[3 * i + 2]);
    try {
        const epp::Matrix m = epp::TrajInterpolation().interpolateTraj(w, max_t, t0, dt);
        double* out = (double*)std::malloc(std::max<size_t>(m.data.size(), 1) * sizeof(double));
        if (!out) {
            epp::set_error("spline trajectory: out of host memory");
            return EPP_ERR_RUNTIME;
        }
        if (!m.data.empty()) std::memcpy(out, m.data.data(), m.data.size() * sizeof(double));
        *rows_out = out;
        *n_rows = (int64_t)m.rows;
        return EPP_OK;
    } catch (const std::invalid_argument& e) {
        epp::set_error(e.what());
        return EPP_ERR_INVALID_ARGUMENT;
    } catch (const std::exception& e) {
        epp::set_error(e.what());
        return EPP_ERR_RUNTIME;
    }
}

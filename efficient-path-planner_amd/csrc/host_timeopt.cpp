// host_timeopt.cpp — the "optimal" trajectory type (host path):
// time-optimal parametrisation of a blended waypoint path under per-axis velocity and
// acceleration bounds, after Kunz & Stilman, "Time-Optimal Trajectory Generation for
// Path Following with Bounded Acceleration and Velocity" (RSS 2012), as vendored in
// external/time_parametrization/src/{Path,Trajectory,OptimalTimeParametrizer}.cpp.
//
// It is one sequential phase-plane integration per trajectory (thousands of dependent
// 1 ms steps), so it stays on the host; the GPU path has nothing to batch here.  The
// restatement keeps the reference's constants (integration step 1e-3, eps 1e-6,
// velocity-switch scan 1e-3 refined by bisection to 1e-6) and its floating-point
// operation order, so results match the reference's to the last bit where libm agrees
// (tests/test_timeopt_cpu.py checks against oracle/timeopt.py).
#include <algorithm>
#include <array>
#include <cmath>
#include <limits>
#include <stdexcept>
#include <utility>
#include <vector>

#include "epp/OptimalTimeParametrizer.h"

namespace epp {
namespace {

using P3 = std::array<double, 3>;

// Eigen-order reductions: (x0 op x1) op x2
double sqnorm(const P3& v) { return (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]; }
double len3(const P3& v) { return std::sqrt(sqnorm(v)); }
double dot3(const P3& a, const P3& b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
P3 diff(const P3& a, const P3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
P3 unit(const P3& v) {  // Eigen normalized(): v / sqrt(|v|^2), unchanged when zero
    const double z = sqnorm(v);
    if (!(z > 0.0)) return v;
    const double r = std::sqrt(z);
    return {v[0] / r, v[1] / r, v[2] / r};
}
P3 midpoint(const P3& a, const P3& b) { return {0.5 * (a[0] + b[0]), 0.5 * (a[1] + b[1]), 0.5 * (a[2] + b[2])}; }

// One piece of the blended path: a straight line (Path.cpp:48-87) or a circular blend
// around a corner (Path.cpp:90-186).  `at` is the piece's arc-length offset.
struct Piece {
    bool arc = false;
    double at = 0.0, len = 0.0;
    P3 a{}, b{};                      // line: from a to b
    P3 centre{}, ux{}, uy{};          // arc: centre, in-plane unit axes
    double radius = 1.0;

    static Piece line(const P3& from, const P3& to) {
        Piece p;
        p.a = from;
        p.b = to;
        p.len = len3(diff(to, from));
        return p;
    }
    // blend between the midpoints `from`/`to` of the two edges meeting at `corner`,
    // deviating at most maxDev from the corner
    static Piece blend(const P3& from, const P3& corner, const P3& to, double maxDev) {
        Piece p;
        p.arc = true;
        p.centre = corner;  // degenerate blends: a zero-length point at the corner
        if (len3(diff(corner, from)) < 0.000001 || len3(diff(to, corner)) < 0.000001) return p;
        const P3 din = unit(diff(corner, from)), dout = unit(diff(to, corner));
        if (len3(diff(din, dout)) < 0.000001) return p;
        double dist = std::min(len3(diff(from, corner)), len3(diff(to, corner)));
        const double angle = std::acos(dot3(din, dout));
        dist = std::min(dist, maxDev * std::sin(0.5 * angle) / (1.0 - std::cos(0.5 * angle)));
        p.radius = dist / std::tan(0.5 * angle);
        p.len = angle * p.radius;
        const P3 bis = unit(diff(dout, din));
        const double off = std::cos(0.5 * angle);
        for (int i = 0; i < 3; ++i) p.centre[i] = corner[i] + bis[i] * p.radius / off;
        P3 r0;
        for (int i = 0; i < 3; ++i) r0[i] = (corner[i] - dist * din[i]) - p.centre[i];
        p.ux = unit(r0);
        p.uy = din;
        return p;
    }

    P3 config(double s) const {
        if (!arc) {
            s /= len;
            s = std::max(0.0, std::min(1.0, s));
            return {(1.0 - s) * a[0] + s * b[0], (1.0 - s) * a[1] + s * b[1], (1.0 - s) * a[2] + s * b[2]};
        }
        const double t = s / radius, c = std::cos(t), sn = std::sin(t);
        P3 q;
        for (int i = 0; i < 3; ++i) q[i] = centre[i] + radius * (ux[i] * c + uy[i] * sn);
        return q;
    }
    P3 tangent(double s) const {
        if (!arc) return {(b[0] - a[0]) / len, (b[1] - a[1]) / len, (b[2] - a[2]) / len};
        const double t = s / radius, c = std::cos(t), sn = std::sin(t);
        P3 q;
        for (int i = 0; i < 3; ++i) q[i] = -ux[i] * sn + uy[i] * c;
        return q;
    }
    P3 curvature(double s) const {
        if (!arc) return {0.0, 0.0, 0.0};
        const double t = s / radius, c = std::cos(t), sn = std::sin(t), k = -1.0 / radius;
        P3 q;
        for (int i = 0; i < 3; ++i) q[i] = k * (ux[i] * c + uy[i] * sn);
        return q;
    }
    // arc lengths (local, sorted) where one axis' tangent component crosses zero
    std::vector<double> axisTurns() const {
        std::vector<double> out;
        if (!arc) return out;
        for (int i = 0; i < 3; ++i) {
            double ang = std::atan2(uy[i], ux[i]);
            if (ang < 0.0) ang += M_PI;
            const double s = ang * radius;
            if (s < len) out.push_back(s);
        }
        std::sort(out.begin(), out.end());
        return out;
    }
};

// Waypoint polyline with circular corner blends (Path.cpp:191-238) and its switching
// points: (arc length, is a curvature discontinuity).
class BlendedPath {
public:
    BlendedPath(const std::vector<P3>& pts, double maxDev) {
        if (pts.size() < 2) throw std::invalid_argument("optimal trajectory: need at least 2 waypoints");
        P3 from = pts[0];
        for (size_t k = 1; k < pts.size(); ++k) {
            if (maxDev > 0.0 && k + 1 < pts.size()) {
                const Piece bl = Piece::blend(midpoint(pts[k - 1], pts[k]), pts[k], midpoint(pts[k], pts[k + 1]), maxDev);
                const P3 bstart = bl.config(0.0);
                if (len3(diff(bstart, from)) > 0.000001) pieces_.push_back(Piece::line(from, bstart));
                pieces_.push_back(bl);
                from = bl.config(bl.len);
            } else {
                pieces_.push_back(Piece::line(from, pts[k]));
                from = pts[k];
            }
        }
        total_ = 0.0;
        for (Piece& p : pieces_) {
            p.at = total_;
            for (double s : p.axisTurns()) switches_.emplace_back(total_ + s, false);
            total_ += p.len;
            while (!switches_.empty() && switches_.back().first >= total_) switches_.pop_back();
            switches_.emplace_back(total_, true);
        }
        switches_.pop_back();  // the path end is not a switching point
        starts_.reserve(pieces_.size());
        for (const Piece& p : pieces_) starts_.push_back(p.at);
    }

    double length() const { return total_; }
    const std::vector<std::pair<double, bool>>& switches() const { return switches_; }
    // the last piece starting at or before s (Path.cpp:240-250); s becomes local
    const Piece& piece(double& s) const {
        const size_t k = std::upper_bound(starts_.begin() + 1, starts_.end(), s) - starts_.begin() - 1;
        s -= pieces_[k].at;
        return pieces_[k];
    }
    P3 config(double s) const { const Piece& p = piece(s); return p.config(s); }
    P3 tangent(double s) const { const Piece& p = piece(s); return p.tangent(s); }
    P3 curvature(double s) const { const Piece& p = piece(s); return p.curvature(s); }
    // first switching point beyond s; the path end (a discontinuity) if none
    double nextSwitch(double s, bool& disc) const {
        for (const auto& sw : switches_)
            if (sw.first > s) {
                disc = sw.second;
                return sw.first;
            }
        disc = true;
        return total_;
    }

private:
    std::vector<Piece> pieces_;
    std::vector<double> starts_;
    std::vector<std::pair<double, bool>> switches_;
    double total_ = 0.0;
};

// Phase-plane (s, s-dot) integration (Trajectory.cpp:53-96 and the methods it calls).
class PhasePlane {
public:
    PhasePlane(const BlendedPath& path, double vmax, double amax) : path_(path), vmax_(vmax), amax_(amax) {
        curve_.push_back({0.0, 0.0, 0.0});
        double after = accBound(0.0, 0.0, true);
        while (ok_ && !forward(after) && ok_) {
            Step sw;
            double before;
            if (nextSwitchingPoint(curve_.back().s, sw, before, after)) break;
            backward(sw.s, sw.sd, before);
        }
        if (ok_) backward(path_.length(), 0.0, accBound(path_.length(), 0.0, false));
        if (ok_) {
            curve_[0].t = 0.0;
            for (size_t k = 1; k < curve_.size(); ++k)
                curve_[k].t = curve_[k - 1].t + (curve_[k].s - curve_[k - 1].s) / ((curve_[k].sd + curve_[k - 1].sd) / 2.0);
        }
    }

    bool valid() const { return ok_; }
    double duration() const { return curve_.back().t; }

    // s, s-dot at time t: constant path acceleration between steps (Trajectory.cpp:459-503)
    void state(double t, double& s, double& sd) const {
        size_t k;
        if (t >= curve_.back().t) {
            k = curve_.size() - 1;
        } else {
            k = std::upper_bound(curve_.begin(), curve_.end(), t, [](double v, const Step& st) { return v < st.t; }) -
                curve_.begin();
        }
        const Step& p = curve_[k - 1];
        const Step& c = curve_[k];
        double h = c.t - p.t;
        const double acc = 2.0 * (c.s - p.s - h * p.sd) / (h * h);
        h = t - p.t;
        s = p.s + h * p.sd + 0.5 * h * h * acc;
        sd = p.sd + h * acc;
    }

private:
    struct Step {
        double s, sd, t;
    };
    static constexpr double kEps = 0.000001;
    static constexpr double kStep = 0.001;  // integration time step

    // extreme path acceleration at (s, sd): upper (max) or lower bound
    double accBound(double s, double sd, bool upper) const {
        const P3 d1 = path_.tangent(s), d2 = path_.curvature(s);
        const double f = upper ? 1.0 : -1.0;
        double m = std::numeric_limits<double>::max();
        for (int i = 0; i < 3; ++i)
            if (d1[i] != 0.0) m = std::min(m, amax_ / std::abs(d1[i]) - f * d2[i] * sd * sd / d1[i]);
        return f * m;
    }
    double slopeBound(double s, double sd, bool upper) const { return accBound(s, sd, upper) / sd; }
    // maximum s-dot the acceleration bounds allow (Trajectory.cpp:387-410)
    double accLimit(double s) const {
        double m = std::numeric_limits<double>::infinity();
        const P3 d1 = path_.tangent(s), d2 = path_.curvature(s);
        for (int i = 0; i < 3; ++i) {
            if (d1[i] != 0.0) {
                for (int j = i + 1; j < 3; ++j) {
                    if (d1[j] != 0.0) {
                        const double aij = d2[i] / d1[i] - d2[j] / d1[j];
                        if (aij != 0.0)
                            m = std::min(m, std::sqrt((amax_ / std::abs(d1[i]) + amax_ / std::abs(d1[j])) / std::abs(aij)));
                    }
                }
            } else if (d2[i] != 0.0) {
                m = std::min(m, std::sqrt(amax_ / std::abs(d2[i])));
            }
        }
        return m;
    }
    // maximum s-dot the velocity bounds allow
    double velLimit(double s) const {
        const P3 d1 = path_.tangent(s);
        double m = std::numeric_limits<double>::max();
        for (int i = 0; i < 3; ++i) m = std::min(m, vmax_ / std::abs(d1[i]));
        return m;
    }
    double accLimitDeriv(double s) const { return (accLimit(s + kEps) - accLimit(s - kEps)) / (2.0 * kEps); }
    double velLimitDeriv(double s) const {
        const P3 d1 = path_.tangent(s);
        double m = std::numeric_limits<double>::max();
        int active = 0;
        for (int i = 0; i < 3; ++i) {
            const double v = vmax_ / std::abs(d1[i]);
            if (v < m) {
                m = v;
                active = i;
            }
        }
        return -(vmax_ * path_.curvature(s)[active]) / (d1[active] * std::abs(d1[active]));
    }

    // Trajectory.cpp:124-158; true when the path end is reached
    bool nextSwitchingPoint(double s, Step& sw, double& before, double& after) const {
        Step accSw{s, 0.0, 0.0};
        double accBefore = 0.0, accAfter = 0.0;
        bool accEnd;
        do {
            accEnd = nextAccSwitch(accSw.s, accSw, accBefore, accAfter);
        } while (!accEnd && accSw.sd > velLimit(accSw.s));
        Step velSw{s, 0.0, 0.0};
        double velBefore = 0.0, velAfter = 0.0;
        bool velEnd;
        do {
            velEnd = nextVelSwitch(velSw.s, velSw, velBefore, velAfter);
        } while (!velEnd && velSw.s <= accSw.s &&
                 (velSw.sd > accLimit(velSw.s - kEps) || velSw.sd > accLimit(velSw.s + kEps)));
        if (accEnd && velEnd) return true;
        if (!accEnd && (velEnd || accSw.s <= velSw.s)) {
            sw = accSw;
            before = accBefore;
            after = accAfter;
        } else {
            sw = velSw;
            before = velBefore;
            after = velAfter;
        }
        return false;
    }

    // Trajectory.cpp:160-199: next point where the acceleration limit curve is touched
    bool nextAccSwitch(double s, Step& sw, double& before, double& after) const {
        double ss = s, sd = 0.0;
        for (;;) {
            bool disc;
            ss = path_.nextSwitch(ss, disc);
            if (ss > path_.length() - kEps) return true;
            if (disc) {
                const double vb = accLimit(ss - kEps), va = accLimit(ss + kEps);
                sd = std::min(vb, va);
                before = accBound(ss - kEps, sd, false);
                after = accBound(ss + kEps, sd, true);
                if ((vb > va || slopeBound(ss - kEps, sd, false) > accLimitDeriv(ss - 2.0 * kEps)) &&
                    (vb < va || slopeBound(ss + kEps, sd, true) < accLimitDeriv(ss + 2.0 * kEps)))
                    break;
            } else {
                sd = accLimit(ss);
                before = 0.0;
                after = 0.0;
                if (accLimitDeriv(ss - kEps) < 0.0 && accLimitDeriv(ss + kEps) > 0.0) break;
            }
        }
        sw = {ss, sd, 0.0};
        return false;
    }

    // Trajectory.cpp:201-237: next point where the velocity limit curve is touched
    bool nextVelSwitch(double s, Step& sw, double& before, double& after) const {
        const double scan = 0.001, accuracy = 0.000001;
        bool started = false;
        s -= scan;
        do {
            s += scan;
            if (slopeBound(s, velLimit(s), false) >= velLimitDeriv(s)) started = true;
        } while ((!started || slopeBound(s, velLimit(s), false) > velLimitDeriv(s)) && s < path_.length());
        if (s >= path_.length()) return true;
        double lo = s - scan, hi = s;
        while (hi - lo > accuracy) {
            s = (lo + hi) / 2.0;
            if (slopeBound(s, velLimit(s), false) > velLimitDeriv(s)) lo = s;
            else hi = s;
        }
        before = accBound(lo, velLimit(lo), false);
        after = accBound(hi, velLimit(hi), true);
        sw = {hi, velLimit(hi), 0.0};
        return false;
    }

    // Trajectory.cpp:240-329: forward integration at maximum acceleration until the path
    // end (true) or a limit curve is hit (false)
    bool forward(double acc) {
        double s = curve_.back().s, sd = curve_.back().sd;
        const auto& sws = path_.switches();
        size_t nd = 0;  // next discontinuity
        for (;;) {
            while (nd < sws.size() && (sws[nd].first <= s || !sws[nd].second)) ++nd;
            const double s0 = s, sd0 = sd;
            sd += kStep * acc;
            s += kStep * 0.5 * (sd0 + sd);
            if (nd < sws.size() && s > sws[nd].first) {
                sd = sd0 + (sws[nd].first - s0) * (sd - sd0) / (s - s0);
                s = sws[nd].first;
            }
            if (s > path_.length()) {
                curve_.push_back({s, sd, 0.0});
                return true;
            } else if (sd < 0.0) {
                ok_ = false;
                return true;
            }
            if (sd > velLimit(s) && slopeBound(s0, velLimit(s0), false) <= velLimitDeriv(s0)) sd = velLimit(s);
            curve_.push_back({s, sd, 0.0});
            acc = accBound(s, sd, true);
            if (sd > accLimit(s) || sd > velLimit(s)) {
                // bisect the crossing of the limit curve
                const Step over = curve_.back();
                curve_.pop_back();
                double lo = curve_.back().s, vlo = curve_.back().sd;
                double hi = over.s, vhi = over.sd;
                while (hi - lo > kEps) {
                    const double mid = 0.5 * (lo + hi);
                    double vmid = 0.5 * (vlo + vhi);
                    if (vmid > velLimit(mid) && slopeBound(lo, velLimit(lo), false) <= velLimitDeriv(lo)) vmid = velLimit(mid);
                    if (vmid > accLimit(mid) || vmid > velLimit(mid)) {
                        hi = mid;
                        vhi = vmid;
                    } else {
                        lo = mid;
                        vlo = vmid;
                    }
                }
                curve_.push_back({lo, vlo, 0.0});
                if (accLimit(hi) < velLimit(hi)) {
                    // (the reference reads past its switching-point list when no
                    // discontinuity is left; no discontinuity ahead means "not beyond")
                    if (nd < sws.size() && hi > sws[nd].first) return false;
                    if (slopeBound(curve_.back().s, curve_.back().sd, true) > accLimitDeriv(curve_.back().s)) return false;
                } else {
                    if (slopeBound(curve_.back().s, curve_.back().sd, false) > velLimitDeriv(curve_.back().s)) return false;
                }
            }
        }
    }

    // Trajectory.cpp:331-377: backward integration at minimum acceleration from (s, sd)
    // until it meets the forward curve, which is then cut there and continued by it
    void backward(double s, double sd, double acc) {
        if (curve_.size() < 2) {
            ok_ = false;
            return;
        }
        size_t i2 = curve_.size() - 1, i1 = i2 - 1;  // segment [i1, i2] of the forward curve
        std::vector<Step> back;                       // built back to front
        double slope = 0.0;
        while (i1 != 0 || s >= 0.0) {
            if (curve_[i1].s <= s) {
                back.push_back({s, sd, 0.0});
                sd -= kStep * acc;
                s -= kStep * 0.5 * (sd + back.back().sd);
                acc = accBound(s, sd, false);
                slope = (back.back().sd - sd) / (back.back().s - s);
                if (sd < 0.0) {
                    ok_ = false;
                    return;
                }
            } else {
                if (i1 == 0) break;  // (reference: steps before the curve's start)
                --i1;
                --i2;
            }
            if (back.empty()) continue;
            const Step& a = curve_[i1];
            const Step& b = curve_[i2];
            const double cslope = (b.sd - a.sd) / (b.s - a.s);
            const double xs = (a.sd - sd + slope * s - cslope * a.s) / (slope - cslope);
            if (std::max(a.s, s) - kEps <= xs && xs <= kEps + std::min(b.s, back.back().s)) {
                const double xsd = a.sd + cslope * (xs - a.s);
                curve_.resize(i2);
                curve_.push_back({xs, xsd, 0.0});
                curve_.insert(curve_.end(), back.rbegin(), back.rend());
                return;
            }
        }
        ok_ = false;
    }

    const BlendedPath& path_;
    const double vmax_, amax_;
    bool ok_ = true;
    std::vector<Step> curve_;
};

// velocity heading, with the reference's explicit axis cases (OptimalTimeParametrizer.cpp:60-88)
double headingOf(double vx, double vy) {
    if (vx == 0 && vy == 0) return 0;
    if (vx == 0) return vy > 0 ? M_PI / 2 : -M_PI / 2;
    if (vy == 0) return vx > 0 ? 0 : M_PI;
    return std::atan2(vy, vx);
}

}  // namespace

namespace OptimalTimeParametrizer {

// OptimalTimeParametrizer.cpp:11-108
Matrix calculateTrajectory(const std::vector<Vec3>& waypoints, const std::vector<Vec3>& preWaypoints, double v_max,
                           double a_max, double startTimeOffset, double samplingInterval, double maxDivergence) {
    if (waypoints.empty()) throw std::invalid_argument("optimal trajectory: need at least 2 waypoints");
    std::vector<P3> all;
    all.reserve(preWaypoints.size() + waypoints.size());
    for (const Vec3& p : preWaypoints) all.push_back({p.x, p.y, p.z});
    for (const Vec3& p : waypoints) all.push_back({p.x, p.y, p.z});
    const BlendedPath path(all, maxDivergence);
    const PhasePlane plane(path, v_max, a_max);
    if (!plane.valid()) throw std::runtime_error("Trajectory is not valid");

    const double duration = plane.duration();
    const int n = (int)(duration / samplingInterval);
    const P3 first = {waypoints[0].x, waypoints[0].y, waypoints[0].z};
    int offset = 0;
    double best = 1000;
    for (int i = 0; i < n; ++i) {
        double s, sd;
        plane.state(i * samplingInterval, s, sd);
        const double d = len3(diff(path.config(s), first));
        if (d < best) {
            offset = i;
            best = d;
        }
    }
    Matrix out((size_t)std::max(0, n - offset), 11);
    for (int i = 0; i < n - offset; ++i) {
        double s, sd;
        plane.state((i + offset) * samplingInterval, s, sd);
        const P3 pos = path.config(s), tan = path.tangent(s), cur = path.curvature(s);
        double* r = out.row((size_t)i);
        for (int d = 0; d < 3; ++d) {
            r[3 * d] = pos[d];
            r[3 * d + 1] = tan[d] * sd;
            r[3 * d + 2] = cur[d] * sd * sd;
        }
        r[9] = headingOf(r[1], r[4]);
        r[10] = (i * samplingInterval) + startTimeOffset;
    }
    return out;
}

}  // namespace OptimalTimeParametrizer
}  // namespace epp

// C ABI (include/epp.h): the "optimal" trajectory with host buffers.
#include <cstdlib>
#include <cstring>

#include "epp.h"
#include "epp_internal.h"

extern "C" epp_status epp_optimal_trajectory_host(const double* wp, int32_t n_wp, const double* pre, int32_t n_pre,
                                                  double v_max, double a_max, double dt, double t0,
                                                  double max_deviation, double** rows_out, int64_t* n_rows) {
    if (!rows_out || !n_rows || (n_wp > 0 && !wp) || (n_pre > 0 && !pre) || n_wp < 0 || n_pre < 0) {
        epp::set_error("optimal trajectory: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    *rows_out = nullptr;
    *n_rows = 0;
    std::vector<epp::Vec3> w, p;
    for (int32_t i = 0; i < n_wp; ++i) w.emplace_back(wp[3 * i], wp[3 * i + 1], wp[3 * i + 2]);
    for (int32_t i = 0; i < n_pre; ++i) p.emplace_back(pre[3 * i], pre[3 * i + 1], pre[3 * i + 2]);
    try {
        if (w.size() + p.size() < 2 || w.empty()) throw std::invalid_argument("optimal trajectory: need at least 2 waypoints");
        const epp::Matrix m = epp::OptimalTimeParametrizer::calculateTrajectory(w, p, v_max, a_max, t0, dt, max_deviation);
        const size_t bytes = std::max<size_t>(m.data.size(), 1) * sizeof(double);
        double* out = (double*)std::malloc(bytes);
        if (!out) {
            epp::set_error("optimal trajectory: out of host memory");
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

// c5_native.cpp — bench.py's native timing of the C5 latency legs on the product (the GPU
// path through its C++ API, no Python): the counterpart of oracle/cpu_bench.cpp, which
// times the same loops on the CPU oracle from the same input file.  Measurement tool, not
// part of the product library.
//
//   c5_native <config.json> <input.txt>
//
// Legs (one JSON object on stdout):
//   c5_refit_native   poly_traj::generateTrajectory of one 12-segment track (solve +
//                     sampling; src/OnlineTrajGenerator.cpp:374-379), 200 calls, first 20 dropped
//   c5_online_native  per step: gate pose perturbed -> World update
//                     (PathPlanner::updateGatePos, src/PathPlanner.cpp:170-173) -> A11
//                     (checkTrajectoryValidity of the lookahead rows, src/PathPlanner.cpp:267-280)
//                     and the 12-segment refit from the current state with the moved
//                     gate-centre waypoint, sampled at dt -- the product's online step:
//                     PathPlanner::checkTrajectoryValidityAndGenerate, ONE launch for both
//   c5_online_native_two_calls  the same step as two calls (checkTrajectoryValidity, then
//                     poly_traj::generateTrajectory), as the reference sequences them;
//                     the two loops must agree step for step (flags and rows)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "epp/ConfigParser.h"
#include "epp/PathPlanner.h"
#include "epp/trajectory_generator.h"

using namespace epp;

namespace {

struct Step {
    int gate, wp_index;
    double dx, dy, dyaw;
};

struct Input {
    Matrix gates, obstacles;
    double md = 0, vmax = 0, amax = 0, dt = 0;
    std::vector<Vec3> wp, refit_wp;
    Matrix look;  // R x 10 rows (positions in columns 0, 3, 6)
    Vec3 v0, a0;
    std::vector<Step> steps;
};

void skip_desc(std::ifstream& f) {
    size_t n = 0;
    f >> n;
    double x;
    int k;
    for (size_t i = 0; i < n; ++i) {
        for (int j = 0; j < 6; ++j) f >> x;
        f >> k;
    }
}

Matrix read_rows(std::ifstream& f, size_t cols) {
    size_t n = 0;
    f >> n;
    Matrix m(n, cols);
    for (size_t i = 0; i < n * cols; ++i) f >> m.data[i];
    return m;
}

std::vector<Vec3> read_points(std::ifstream& f) {
    size_t n = 0;
    f >> n;
    std::vector<Vec3> p(n);
    for (auto& v : p) f >> v.x >> v.y >> v.z;
    return p;
}

// The layout of oracle/cpu_bench.cpp's input (the OBB descriptions are skipped: the
// product reads the geometry from the config file).
Input read_input(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    Input in;
    skip_desc(f);
    size_t n = 0;
    f >> n;
    int off;
    for (size_t i = 0; i < n; ++i) f >> off;
    skip_desc(f);
    in.gates = read_rows(f, 7);
    in.obstacles = read_rows(f, 6);
    double rg, ro;
    f >> rg >> ro >> in.md >> in.vmax >> in.amax >> in.dt;
    in.wp = read_points(f);
    const std::vector<Vec3> look = read_points(f);
    in.look = Matrix(look.size(), 10);
    for (size_t i = 0; i < look.size(); ++i) {
        in.look(i, 0) = look[i].x;
        in.look(i, 3) = look[i].y;
        in.look(i, 6) = look[i].z;
    }
    in.refit_wp = read_points(f);
    f >> in.v0.x >> in.v0.y >> in.v0.z >> in.a0.x >> in.a0.y >> in.a0.z;
    f >> n;
    in.steps.resize(n);
    for (auto& s : in.steps) f >> s.gate >> s.wp_index >> s.dx >> s.dy >> s.dyaw;
    if (!f) throw std::runtime_error("malformed input " + path);
    return in;
}

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void print_pct(const char* key, std::vector<double> t, bool last) {
    double s = 0;
    for (double x : t) s += x;
    std::sort(t.begin(), t.end());
    auto at = [&](double q) {  // numpy.percentile's linear interpolation
        const double r = q * (t.size() - 1);
        const size_t i = (size_t)r;
        return i + 1 < t.size() ? t[i] + (t[i + 1] - t[i]) * (r - i) : t[i];
    };
    std::printf("\"%s\": {\"p50_us\": %.4f, \"p99_us\": %.4f, \"mean_us\": %.4f, \"steps\": %zu}%s", key, at(0.5),
                at(0.99), s / t.size(), t.size(), last ? "" : ", ");
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: c5_native <config.json> <input.txt>\n");
        return 2;
    }
    try {
        const Input in = read_input(argv[2]);
        auto cfg = std::make_shared<ConfigParser>(argv[1]);
        PathPlanner pp(in.gates, in.obstacles, cfg);
        Matrix traj;
        const Vec3 zero(0, 0, 0);
        std::vector<double> t_refit;
        for (int r = 0; r < 200; ++r) {
            const double t0 = now_us();
            poly_traj::generateTrajectory(in.refit_wp, in.vmax, in.amax, in.dt, 0.0, zero, zero, traj);
            const double t1 = now_us();
            if (r >= 20) t_refit.push_back(t1 - t0);
        }
        const size_t refit_rows = traj.rows;
        (void)pp;
        // the online loop, fused (the product's step) or as two calls; both record each
        // step's flag and final rows so they can be compared
        auto online = [&](bool fused, std::vector<double>& t_online, std::vector<char>& valid_of, Matrix& last) {
            PathPlanner p2(in.gates, in.obstacles, cfg);
            Matrix look = in.look, tr;
            (void)p2.checkTrajectoryValidity(look, in.md);  // (warm: first launch of the check)
            std::vector<Vec3> wp = in.wp;
            for (const Step& s : in.steps) {
                const double t0 = now_us();
                std::vector<double> pose(in.gates.row(s.gate), in.gates.row(s.gate) + 6);
                pose[0] += s.dx;
                pose[1] += s.dy;
                pose[5] += s.dyaw;
                p2.updateGatePos(s.gate, pose);
                wp = in.wp;
                wp[s.wp_index].x = pose[0];
                wp[s.wp_index].y = pose[1];
                bool ok;
                if (fused) {
                    ok = p2.checkTrajectoryValidityAndGenerate(look, in.md, wp, in.vmax, in.amax, in.dt, 0.0, in.v0, in.a0,
                                                               tr);
                } else {
                    ok = p2.checkTrajectoryValidity(look, in.md);
                    poly_traj::generateTrajectory(wp, in.vmax, in.amax, in.dt, 0.0, in.v0, in.a0, tr);
                }
                for (size_t i = 0; i < look.rows && i < tr.rows; ++i)  // the next step checks the new rows
                    for (int k = 0; k < 3; ++k) look(i, 3 * k) = tr(i, 3 * k);
                t_online.push_back(now_us() - t0);
                valid_of.push_back(ok ? 1 : 0);
            }
            last = tr;
        };
        std::vector<double> t_fused, t_two, t_update;
        std::vector<char> v_fused, v_two;
        Matrix last_fused, last_two;
        online(false, t_two, v_two, last_two);
        online(true, t_fused, v_fused, last_fused);
        {  // the step's world update alone (updateGatePos and the device world's refresh the
           // step's check then uses): the host share of the step
            PathPlanner p3(in.gates, in.obstacles, cfg);
            (void)p3.worldPtr->device();
            for (const Step& s : in.steps) {
                const double t0 = now_us();
                std::vector<double> pose(in.gates.row(s.gate), in.gates.row(s.gate) + 6);
                pose[0] += s.dx;
                pose[1] += s.dy;
                pose[5] += s.dyaw;
                p3.updateGatePos(s.gate, pose);
                (void)p3.worldPtr->device();
                t_update.push_back(now_us() - t0);
            }
        }
        int64_t invalid_steps = 0;
        for (char v : v_fused) invalid_steps += v ? 0 : 1;
        const bool agree = v_fused == v_two && last_fused.rows == last_two.rows && last_fused.data == last_two.data;
        std::printf("{");
        print_pct("c5_refit_native", t_refit, false);
        print_pct("c5_online_native", t_fused, false);
        print_pct("c5_online_native_two_calls", t_two, false);
        print_pct("c5_world_update_native", t_update, false);
        std::printf("\"refit_rows\": %zu, \"online_rows\": %zu, \"online_invalid_steps\": %lld, "
                    "\"fused_equals_two_calls\": %s, \"online_step\": \"fused: one launch (A11 check + refit)\"}\n",
                    refit_rows, last_fused.rows, (long long)invalid_steps, agree ? "true" : "false");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "c5_native: %s\n", e.what());
        return 1;
    }
    return 0;
}

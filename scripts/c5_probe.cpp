// c5_probe.cpp — per-call latency of the C5 step's pieces through the C++ API, without
// Python (diagnostics only; not part of the product).  Inputs are written by
// scripts/c5_probe.py (config path, gates, obstacles, 13 waypoints, 100 lookahead rows).
// Build (CPU side):
//   hipcc -O2 -std=c++17 -Iinclude -o scripts/c5_probe scripts/c5_probe.cpp \
//         -Lefficient-path-planner_amd -lepp -Wl,-rpath,'$ORIGIN/../efficient-path-planner_amd'
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "epp/ConfigParser.h"
#include "epp/PathPlanner.h"
#include "epp/trajectory_generator.h"

using namespace epp;

static Matrix read_matrix(const std::string& path) {
    std::ifstream f(path);
    size_t r = 0, c = 0;
    f >> r >> c;
    Matrix m(r, c);
    for (size_t i = 0; i < r * c; ++i) f >> m.data[i];
    return m;
}

template <typename F>
static void timeit(const char* name, int iters, F&& f) {
    std::vector<double> t(iters);
    for (int i = 0; i < iters; ++i) {
        auto a = std::chrono::steady_clock::now();
        f(i);
        auto b = std::chrono::steady_clock::now();
        t[i] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    std::vector<double> s(t.begin() + iters / 10, t.end());
    std::sort(s.begin(), s.end());
    std::printf("%-28s p50 %7.2f us  p99 %7.2f us  min %7.2f us\n", name, s[s.size() / 2],
                s[(size_t)(s.size() * 0.99)], s[0]);
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "gpurun_out";
    std::string cfg_path;
    {
        std::ifstream f(dir + "/c5_cfg.txt");
        f >> cfg_path;
    }
    const Matrix gates = read_matrix(dir + "/c5_gates.txt"), obst = read_matrix(dir + "/c5_obst.txt");
    const Matrix wpm = read_matrix(dir + "/c5_wp.txt"), rows = read_matrix(dir + "/c5_rows.txt");
    auto cfg = std::make_shared<ConfigParser>(cfg_path);
    PathPlanner pp(gates, obst, cfg);
    std::vector<Vec3> wp;
    for (size_t i = 0; i < wpm.rows; ++i) wp.emplace_back(wpm(i, 0), wpm(i, 1), wpm(i, 2));
    const double md = 0.2;
    std::vector<double> xyz(rows.rows * 3);
    for (size_t i = 0; i < rows.rows; ++i) {
        xyz[3 * i] = rows(i, 0);
        xyz[3 * i + 1] = rows(i, 3);
        xyz[3 * i + 2] = rows(i, 6);
    }
    std::vector<uint8_t> ok(rows.rows);
    const int it = 1000;
    pp.checkTrajectoryValidity(rows, md);
    std::vector<double> pose(gates.row(0), gates.row(0) + 6);
    timeit("checkPointsMinDistance clean", it,
           [&](int) { pp.worldPtr->checkPointsMinDistance(xyz.data(), (int64_t)rows.rows, md, ok.data()); });
    timeit("checkTrajectoryValidity", it, [&](int) { pp.checkTrajectoryValidity(rows, md); });
    timeit("updateGatePos", it, [&](int i) {
        pose[0] = gates(0, 0) + 0.001 * (i % 7);
        pp.updateGatePos(0, pose);
    });
    timeit("update + device()", it, [&](int i) {
        pose[0] = gates(0, 0) + 0.001 * (i % 7);
        pp.updateGatePos(0, pose);
        (void)pp.worldPtr->device();
    });
    timeit("update + checkPointsMinDist", it, [&](int i) {
        pose[0] = gates(0, 0) + 0.001 * (i % 7);
        pp.updateGatePos(0, pose);
        pp.worldPtr->checkPointsMinDistance(xyz.data(), (int64_t)rows.rows, md, ok.data());
    });
    Matrix traj;
    const Vec3 v0(0.4, -0.2, 0.1), a0(0.0, 0.3, 0.0);
    timeit("generateTrajectory", it, [&](int) { poly_traj::generateTrajectory(wp, 1.0, 2.0, 0.1, 0.0, v0, a0, traj); });
    timeit("C5 step", it, [&](int i) {
        pose[0] = gates(0, 0) + 0.001 * (i % 7);
        pp.updateGatePos(0, pose);
        pp.checkTrajectoryValidity(rows, md);
        poly_traj::generateTrajectory(wp, 1.0, 2.0, 0.1, 0.0, v0, a0, traj);
    });
    std::printf("rows %zu\n", traj.rows);
    return 0;
}

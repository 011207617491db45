// cpu_bench.cpp — TEST INFRASTRUCTURE ONLY: bench.py's native CPU baseline for the C5
// latency legs.  The reference's C5 step is a sequence of native C++ calls
// (src/OnlineTrajGenerator.cpp:141-212: World rebuild, checkTrajectoryValidity;
// :374-379: poly_traj::generateTrajectory), so the CPU side is timed here as native calls
// into the oracle (liboracle.so, the CPU restatement), without the Python/ctypes layer the
// ctypes figures include.  It mirrors scripts/c5_probe.cpp, the product's native probe.
//
// Input (text, written by bench.py's cpu_baseline): see read_input() below.
// Output: one JSON object on stdout.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "epp_oracle.h"

namespace {

struct Input {
    std::vector<or_obb_desc> gate_desc, obst_desc;
    std::vector<int32_t> gate_desc_off;
    std::vector<double> gates, obstacles;  // G x 7, O x 6
    double rg = 0, ro = 0, md = 0, vmax = 0, amax = 0, dt = 0;
    std::vector<double> wp;        // W x 3 (the refit window)
    std::vector<double> look;      // R x 3 (A11 lookahead positions)
    std::vector<double> refit_wp;  // W x 3 (the single-refit leg's track)
    double v0[3] = {0, 0, 0}, a0[3] = {0, 0, 0};
    struct Step {
        int gate, wp_index;
        double dx, dy, dyaw;
    };
    std::vector<Step> steps;
};

template <typename T>
void read_n(std::ifstream& f, std::vector<T>& v, size_t n) {
    v.resize(n);
    for (auto& x : v) f >> x;
}

std::vector<or_obb_desc> read_desc(std::ifstream& f) {
    size_t n = 0;
    f >> n;
    std::vector<or_obb_desc> d(n);
    for (auto& x : d) {
        for (double& p : x.pos) f >> p;
        for (double& s : x.size) f >> s;
        f >> x.filling;
        x.pad = 0;
    }
    return d;
}

// Layout: gate_desc (n, then pos3 size3 filling per line); gate_desc_off (n, ints);
// obst_desc; gates (G, G x 7); obstacles (O, O x 6); rg ro md vmax amax dt;
// wp (W, W x 3); look (R, R x 3); refit_wp (W, W x 3); v0 (3); a0 (3);
// steps (S, then gate wp_index dx dy dyaw per step).  Doubles as %.17g.
Input read_input(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    Input in;
    in.gate_desc = read_desc(f);
    size_t n = 0;
    f >> n;
    read_n(f, in.gate_desc_off, n);
    in.obst_desc = read_desc(f);
    f >> n;
    read_n(f, in.gates, 7 * n);
    f >> n;
    read_n(f, in.obstacles, 6 * n);
    f >> in.rg >> in.ro >> in.md >> in.vmax >> in.amax >> in.dt;
    f >> n;
    read_n(f, in.wp, 3 * n);
    f >> n;
    read_n(f, in.look, 3 * n);
    f >> n;
    read_n(f, in.refit_wp, 3 * n);
    for (double& v : in.v0) f >> v;
    for (double& v : in.a0) f >> v;
    f >> n;
    in.steps.resize(n);
    for (auto& s : in.steps) f >> s.gate >> s.wp_index >> s.dx >> s.dy >> s.dyaw;
    if (!f) throw std::runtime_error("malformed input " + path);
    return in;
}

struct Pct {
    double p50, p99, mean;
    size_t n;
};

Pct pct(std::vector<double> t) {
    Pct p{};
    p.n = t.size();
    if (t.empty()) return p;
    double s = 0;
    for (double x : t) s += x;
    p.mean = s / t.size();
    std::sort(t.begin(), t.end());
    // numpy.percentile's linear interpolation, as the Python legs report it
    auto at = [&](double q) {
        const double r = q * (t.size() - 1);
        const size_t i = (size_t)r;
        const double fr = r - i;
        return i + 1 < t.size() ? t[i] + (t[i + 1] - t[i]) * fr : t[i];
    };
    p.p50 = at(0.5);
    p.p99 = at(0.99);
    return p;
}

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void print_pct(const char* key, const Pct& p, bool last) {
    std::printf("\"%s\": {\"p50_us\": %.4f, \"p99_us\": %.4f, \"mean_us\": %.4f, \"steps\": %zu, \"threads\": 1}%s", key,
                p.p50, p.p99, p.mean, p.n, last ? "" : ", ");
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: cpu_bench <input.txt>\n");
        return 2;
    }
    const Input in = read_input(argv[1]);
    const int G = (int)(in.gates.size() / 7), O = (int)(in.obstacles.size() / 6);
    const int W = (int)(in.wp.size() / 3), R = (int)(in.look.size() / 3), WR = (int)(in.refit_wp.size() / 3);
    const int cap = G * (int)std::max<size_t>(1, in.gate_desc.size()) + O * (int)std::max<size_t>(1, in.obst_desc.size()) + 1;
    std::vector<or_obb> world(cap);
    std::vector<uint8_t> ok(R);
    std::vector<double> rows(1 << 16);
    const double zero[3] = {0, 0, 0};
    auto build = [&](const std::vector<double>& gates) {
        const int n = or_world_build(in.gate_desc.data(), in.gate_desc_off.data(), (int)in.gate_desc_off.size() - 1,
                                     in.obst_desc.data(), (int)in.obst_desc.size(), gates.data(), G,
                                     in.obstacles.data(), O, in.rg, in.ro, world.data(), cap);
        if (n < 0) throw std::runtime_error("or_world_build failed");
        return n;
    };
    auto generate = [&](const std::vector<double>& wp, int n_wp, const double* v0, const double* a0) {
        const int64_t n = or_generate_trajectory(wp.data(), n_wp, in.vmax, in.amax, in.dt, 0.0, v0, a0, rows.data(),
                                                 (int64_t)(rows.size() / 10));
        if (n < 0 || n > (int64_t)(rows.size() / 10)) throw std::runtime_error("or_generate_trajectory failed");
        return n;
    };

    // (1) C5 single refit: generateTrajectory of the 12-segment track (solve + sampling),
    // 200 calls, the first 20 dropped (as bench.py's ctypes leg)
    std::vector<double> t_refit;
    int64_t refit_rows = 0;
    for (int r = 0; r < 200; ++r) {
        const double t0 = now_us();
        refit_rows = generate(in.refit_wp, WR, zero, zero);
        const double t1 = now_us();
        if (r >= 20) t_refit.push_back(t1 - t0);
    }
    // (2) C5 online step: perturbed gate -> World rebuild (src/OnlineTrajGenerator.cpp:146)
    // -> A11 minDistance check of the lookahead rows (:192) -> 12-segment refit from the
    // current state with the moved gate-centre waypoint (:374-379), sampled at dt
    std::vector<double> t_online;
    std::vector<double> gates = in.gates, wp = in.wp, look = in.look;
    int64_t online_rows = 0, invalid = 0;
    for (const auto& s : in.steps) {
        const double t0 = now_us();
        gates = in.gates;
        gates[7 * s.gate + 0] += s.dx;
        gates[7 * s.gate + 1] += s.dy;
        gates[7 * s.gate + 5] += s.dyaw;
        const int n = build(gates);
        or_check_states_mindist(world.data(), n, look.data(), R, in.md, ok.data());
        for (int i = 0; i < R; ++i) invalid += ok[i] ? 0 : 1;
        wp = in.wp;
        wp[3 * s.wp_index + 0] = gates[7 * s.gate + 0];
        wp[3 * s.wp_index + 1] = gates[7 * s.gate + 1];
        online_rows = generate(wp, W, in.v0, in.a0);
        for (int i = 0; i < R && i < online_rows; ++i)  // the next step checks the new rows (as bench.py's loops)
            for (int k = 0; k < 3; ++k) look[3 * i + k] = rows[10 * i + 3 * k];
        t_online.push_back(now_us() - t0);
    }
    std::printf("{");
    print_pct("c5_refit_native", pct(t_refit), false);
    print_pct("c5_online_native", pct(t_online), false);
    std::printf("\"refit_rows\": %lld, \"online_rows\": %lld, \"online_invalid_rows\": %lld}\n", (long long)refit_rows,
                (long long)online_rows, (long long)invalid);
    return 0;
}

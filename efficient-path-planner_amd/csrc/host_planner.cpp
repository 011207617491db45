// host_planner.cpp — epp::PathPlanner (drop-in for src/PathPlanner.cpp) on the batch
// GPU planner.  See include/epp/PathPlanner.h for the algorithm.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <mutex>
#include <queue>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <stdexcept>
#include <thread>
#include <utility>

#include <hip/hip_runtime_api.h>

#include "epp/PathPlanner.h"
#include "epp/trajectory_generator.h"
#include "epp_internal.h"
#include "host_scratch.h"

namespace epp {

namespace {
std::mutex g_stats_mu;

// Worker threads for PathPlanner::planPaths.  Grown on demand and never torn down (the
// process exit ends them; their thread-local device scratch is then left to the runtime
// rather than freed after it).
class PlanPool {
public:
    void submit(std::function<void()> job) {
        std::lock_guard<std::mutex> lk(mu_);
        q_.push_back(std::move(job));
        // a waiting thread per queued job, else one more thread
        if (idle_ < (int)q_.size()) std::thread([this] { loop(); }).detach();
        else cv_.notify_one();
    }

private:
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            while (q_.empty()) {
                ++idle_;
                cv_.wait(lk);
                --idle_;
            }
            std::function<void()> job = std::move(q_.front());
            q_.pop_front();
            lk.unlock();
            job();
            lk.lock();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    int idle_ = 0;
};

PlanPool& plan_pool() {
    static PlanPool* pool = new PlanPool();  // intentionally leaked (see above)
    return *pool;
}

uint64_t mix(uint64_t a, uint64_t b) {
    uint64_t x = a ^ (b + 0x9E3779B97F4A7C15ull + (a << 6) + (a >> 2));
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
uint64_t bits_of(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
}  // namespace

PathPlanner::PathPlanner(const Matrix& gates, const Matrix& obstacles, std::shared_ptr<ConfigParser> cp)
    : configParser(std::move(cp)) {
    worldPtr = std::make_shared<World>(configParser);
    parseGatesAndObstacles(gates, obstacles);  // src/PathPlanner.cpp:27-35
    // the device world (index build, its HBM and pinned buffers, the upload) now, as the
    // reference builds its World here, not inside the first planPath
    (void)worldPtr->device();
}

// src/PathPlanner.cpp:60-78
void PathPlanner::parseGatesAndObstacles(const Matrix& gates, const Matrix& obstacles) {
    fillWorld(*worldPtr, gates, obstacles);
}

void PathPlanner::fillWorld(World& world, const Matrix& gates, const Matrix& obstacles) {
    world.resetWorld();
    for (size_t i = 0; i < gates.rows; ++i) {
        std::vector<double> g(gates.row(i), gates.row(i) + gates.cols);
        if (g.size() < 7) throw std::invalid_argument("gate rows need 7 columns");
        g[2] = 0.0;  // put all gates to ground  :68
        world.addGate((int)i, g);
    }
    for (size_t i = 0; i < obstacles.rows; ++i) {
        std::vector<double> o(obstacles.row(i), obstacles.row(i) + obstacles.cols);
        if (o.size() < 6) throw std::invalid_argument("obstacle rows need 6 columns");
        world.addObstacle((int)i, o);
    }
}

void PathPlanner::updateGatePos(int gateId, const std::vector<double>& newPose) {
    worldPtr->updateGatePosition(gateId, newPose);  // src/PathPlanner.cpp:170-173
}

bool PathPlanner::planOnce(const Vec3& start, const Vec3& goal, int64_t samples, uint64_t seed,
                           std::vector<Vec3>& out) const {
    const auto& pp = configParser->getPathPlannerProperties();
    const auto& wp = configParser->getWorldProperties();
    const bool canPass = pp.canPassGate;  // validators get can_pass_gate  src/PathPlanner.cpp:47-50
    const epp_world* w = worldPtr->device();
    const int k = k_;
    ThreadScratch& ts = ThreadScratch::get();
    void* st = ts.stream();
    const auto t_dev0 = std::chrono::steady_clock::now();
    // ---- 1. sample + validate states (StateValidator::isValid), all on the device ------
    // nodes = start, goal, then the valid samples in sample order (ordered compaction)
    const size_t n_s = (size_t)samples;
    const size_t max_nodes = n_s + 2;
    const size_t m_max = max_nodes * (size_t)k;
    const size_t ws_bytes = (size_t)epp_knn_workspace_size((int32_t)max_nodes);
    const size_t cws_bytes = (size_t)epp_compact_workspace_size((int64_t)n_s);
    ts.reset(ThreadScratch::rounded(n_s * 24) + ThreadScratch::rounded(n_s) + ThreadScratch::rounded(256 + max_nodes * 24) +
             ThreadScratch::rounded(8) + ThreadScratch::rounded(16) + ThreadScratch::rounded(m_max * 4) + 2 * ThreadScratch::rounded(m_max * 24) +
             ThreadScratch::rounded(m_max) + ThreadScratch::rounded(ws_bytes) + ThreadScratch::rounded(cws_bytes));
    double* d_s = static_cast<double*>(ts.carve(n_s * 24));
    uint8_t* d_v = static_cast<uint8_t*>(ts.carve(n_s));
    // [.. | edge counts (16 B) | 32 B | start, goal, the valid samples]: the counters and
    // the two end nodes are set by one upload (no separate clearing of the counters)
    char* d_head = static_cast<char*>(ts.carve(256 + max_nodes * 24));
    double* d_nodes = reinterpret_cast<double*>(d_head + 256);
    int64_t* d_ecnt = reinterpret_cast<int64_t*>(d_head + 256 - 48);
    int64_t* d_cnt = static_cast<int64_t*>(ts.carve(8));
    int32_t* d_nbr = static_cast<int32_t*>(ts.carve(m_max * 4));
    double* d_e1 = static_cast<double*>(ts.carve(m_max * 24));
    double* d_e2 = static_cast<double*>(ts.carve(m_max * 24));
    uint8_t* d_ev = static_cast<uint8_t*>(ts.carve(m_max));
    void* d_ws = ts.carve(ws_bytes);
    void* d_cws = ts.carve(cws_bytes);
    const double lo[3] = {wp.lowerBound.x, wp.lowerBound.y, wp.lowerBound.z};
    const double hi[3] = {wp.upperBound.x, wp.upperBound.y, wp.upperBound.z};
    const double ends[6] = {start.x, start.y, start.z, goal.x, goal.y, goal.z};
    // (the sampler also zeroes the compaction's look-back status words)
    check(sample_uniform_and_clear(seed, lo, hi, samples, d_s, d_cws, cws_bytes, st), "sample");
    check(epp_check_states(w, d_s, samples, canPass ? 1 : 0, d_v, nullptr, nullptr, st), "state check");
    check(compact_states_cleared(d_s, d_v, samples, d_nodes + 6, d_cnt, d_cws, cws_bytes, st), "compact");
    // start / goal up, the valid-state count down: both queued, one synchronisation
    // (pinned staging: [ends (6 doubles) | count | edge counts (2)])
    // pinned staging: [edge counts = 0 (2) | pad (4) | ends (6) | count | edge counts (2)]
    double* h_small = static_cast<double*>(ts.pinned(2, 16 * sizeof(double)));
    std::fill(h_small, h_small + 6, 0.0);
    std::copy(ends, ends + 6, h_small + 6);
    int64_t* h_cnt = reinterpret_cast<int64_t*>(h_small + 12);
    check(epp_memcpy_h2d_async(d_ecnt, h_small, 12 * sizeof(double), st), "upload");
    check(epp_memcpy_d2h_async(h_cnt, d_cnt, 8, st), "download");
    check(epp_stream_sync(st), "sync");
    const int64_t n_valid_states = h_cnt[0];
    const int32_t n = (int32_t)(n_valid_states + 2);
    // the node coordinates (final now) go down on the copy stream while the k-NN and the
    // motion checks run on this one (pinned staging sized for the attempt's largest node
    // count: a pinned buffer that grows is freed, and hipHostFree waits for the device)
    void* cst = ts.copy_stream();
    const double* nodes = static_cast<const double*>(ts.pinned(0, max_nodes * 24));
    check(epp_memcpy_d2h_async(const_cast<double*>(nodes), d_nodes, (uint64_t)n * 24, cst), "download");
    // ---- 2. k-NN graph + batched motion checks (MotionValidator::checkMotion) --------
    const size_t m = (size_t)n * k;
    // the grid over the sampling box widened by start and goal (every node lies inside)
    const double blo[3] = {std::min({lo[0], start.x, goal.x}), std::min({lo[1], start.y, goal.y}),
                           std::min({lo[2], start.z, goal.z})};
    const double bhi[3] = {std::max({hi[0], start.x, goal.x}), std::max({hi[1], start.y, goal.y}),
                           std::max({hi[2], start.z, goal.z})};
    // Row-restricted search first (narrow tables, n <= 65535): the k-NN rows, motion checks
    // and download only for the nodes in the ellipsoid |x - start| + |x - goal| <= bound.
    // A* pops nodes in increasing f = g + h >= |x - start| + |x - goal|, so a search that
    // reaches the goal with every popped f <= bound has expanded only rows held here, and
    // pops exactly what the search over the whole table pops (a node outside the ellipsoid
    // has f > bound >= the path's length): the same path.  Otherwise (bound passed, rows past
    // the packing capacity, no forward edge into the goal among the rows) the whole table
    // is built, checked and searched, as without the restriction.
    // bound = factor * |start - goal| + 0.25 m; EPP_PLAN_ELLIPSE sets the factor (default
    // 1.5; 0 = the whole table only).
    const bool narrow = n <= 65535;
    double factor = 1.5;
    if (const char* ev = std::getenv("EPP_PLAN_ELLIPSE")) factor = std::atof(ev);
    const double d_sg = (goal - start).norm();
    const double bound = factor * d_sg + 0.25;
    // packing capacity: 1.25 x the expected rows (the ellipsoid's volume, unclipped, over the
    // sampling box's) + 1024; not worth it past half the table
    int32_t cap = 0;
    if (narrow && factor >= 1.0 && n > 2048) {
        const double vbox = (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]);
        const double vell = M_PI * bound * (bound * bound - d_sg * d_sg) / 6.0;
        const double frac = vbox > 0 ? std::min(1.0, vell / vbox) : 1.0;
        const double want = 1.25 * frac * n + 1024.0;
        if (want < 0.5 * n) cap = (int32_t)want;
    }
    // packed buffers in d_e2 (free on this path): [ids16 | rows16] (the download), ids32, rows32
    const size_t ids_pad = ((size_t)cap + 7) & ~(size_t)7;  // (16-B aligned rows)
    uint16_t* d_ids16 = reinterpret_cast<uint16_t*>(d_e2);
    uint16_t* d_rows16 = d_ids16 + ids_pad;
    const size_t pack_bytes = (ids_pad + (size_t)cap * k) * 2;
    int32_t* d_ids32 = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(d_e2) + ((pack_bytes + 255) & ~(size_t)255));
    int32_t* d_rows32 = d_ids32 + ids_pad;
    void* h_tab = ts.pinned(1, m_max * 4);
    const int32_t* nbr32 = static_cast<const int32_t*>(h_tab);
    const uint16_t* nbr16 = static_cast<const uint16_t*>(h_tab);
    auto nbr = [&](size_t e) -> int {
        if (!narrow) return nbr32[e];
        const uint16_t x = nbr16[e];
        return x == 0xFFFF ? -1 : (int)x;
    };
    int64_t* ecnt = h_cnt + 1;  // [valid edges, of which into the goal, packed rows]
    int64_t edges_checked = 0, n_valid_edges = 0, rows_down = 0;
    bool goal_has_forward_edge = false;
    double ms_dev = 0.0;
    bool restricted = false;
    if (cap > 0) {
        const double sv[3] = {start.x, start.y, start.z}, gv[3] = {goal.x, goal.y, goal.z};
        check(knn_ws_box_ellipse(d_nodes, n, k, blo, bhi, sv, gv, bound, d_nbr, d_ws, ws_bytes, st), "knn");
        check(pack_ellipse_rows(d_nodes, d_nbr, n, k, sv, gv, bound, cap, d_ids32, d_ids16, d_rows32, d_ecnt + 2, st),
              "pack rows");
        const epp_status ks = check_knn_motions_rows(w, d_nodes, d_rows32, d_ids32, d_ecnt + 2, cap, k,
                                                     canPass ? 1 : 0, d_ev, d_rows16, 1, d_ecnt, st);
        if (ks != EPP_ERR_UNSUPPORTED) {
            check(ks, "motion check");
            restricted = true;
            check(epp_memcpy_d2h_async(ecnt, d_ecnt, 24, st), "download");
            check(epp_memcpy_d2h_async(h_tab, d_ids16, pack_bytes, st), "download");
            check(epp_stream_sync(st), "sync");
            check(epp_stream_sync(cst), "sync");
            const int64_t rows = std::min<int64_t>(ecnt[2], cap);
            edges_checked += rows * k;
            n_valid_edges += ecnt[0];
            rows_down += rows;
        }
    }
    // the whole table (as without the restriction): k-NN, motion checks straight off the
    // table with the mask folded in (failed motions -> -1; the valid edges and those into
    // the goal, node 1, counted), the table down (up to 65535 nodes as u16, 0xFFFF: no edge,
    // half the bytes, written into d_e1).  Small batches / worlds without tile tables:
    // materialised endpoints, then the mask kernel.
    uint16_t* d_nbr16 = narrow ? reinterpret_cast<uint16_t*>(d_e1) : nullptr;
    auto whole_table = [&] {
        if (restricted && hipMemsetAsync(d_ecnt, 0, 16, static_cast<hipStream_t>(st)) != hipSuccess)
            throw std::runtime_error("planPath: clearing the edge counts failed");
        check(epp_knn_ws_box(d_nodes, n, k, 0.0, blo, bhi, d_nbr, d_ws, ws_bytes, st), "knn");
        const epp_status ks =
            check_knn_motions_masked(w, d_nodes, d_nbr, n, k, canPass ? 1 : 0, d_ev, d_nbr16, 1, d_ecnt, st);
        if (ks == EPP_ERR_UNSUPPORTED) {
            check(epp_knn_edges(d_nodes, d_nbr, n, k, d_e1, d_e2, st), "edges");
            check(epp_check_motions(w, d_e1, d_e2, (int64_t)m, canPass ? 1 : 0, 0, d_ev, st), "motion check");
            check(mask_edges_count_acc(d_nbr, d_ev, (int64_t)m, 1, d_ecnt, st, d_nbr16), "mask edges");
        } else {
            check(ks, "motion check");
        }
        // the downloads queued back to back, one synchronisation (and the nodes' stream)
        check(epp_memcpy_d2h_async(ecnt, d_ecnt, 16, st), "download");
        if (narrow) check(epp_memcpy_d2h_async(h_tab, d_nbr16, m * 2, st), "download");
        else check(epp_memcpy_d2h_async(h_tab, d_nbr, m * 4, st), "download");
        check(epp_stream_sync(st), "sync");
        check(epp_stream_sync(cst), "sync");
        edges_checked += (int64_t)m;
        n_valid_edges += ecnt[0];
        goal_has_forward_edge = ecnt[1] > 0;
        rows_down += n;
    };
    if (!restricted) whole_table();
    ms_dev += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_dev0).count();
    // ---- 3. shortest path over the valid edges, start = 0, goal = 1 ----------------------
    // A* with the Euclidean distance to the goal (admissible and consistent for Euclidean
    // edge costs: an optimal path of the graph searched).  First over the forward k-NN
    // edges alone, read straight from the k-NN table (no graph build: A* touches only
    // the nodes it expands); only if the goal is not reached that way, again over the
    // symmetrised graph (reverse edges added as a CSR).
    auto node = [&](int v) { return Vec3(nodes[3 * v], nodes[3 * v + 1], nodes[3 * v + 2]); };
    const Vec3 gp = node(1);
    // Search state per host thread, reused across calls: a node's dist / prev hold this
    // search's values only when its stamp is the search's (no O(n) clearing per search:
    // A* touches a small part of the ~63k nodes); the heap keeps its storage.
    using QE = std::pair<double, int>;  // (g + h, node)
    struct SearchState {
        std::vector<double> dist;
        std::vector<int> prev;
        std::vector<uint32_t> seen, done;  // stamps: dist/prev valid, closed
        std::vector<QE> heap;
        uint32_t cur = 0;
    };
    thread_local SearchState ss;
    if (ss.dist.size() < (size_t)n) {
        ss.dist.resize(n);
        ss.prev.resize(n);
        ss.seen.resize(n, 0u);
        ss.done.resize(n, 0u);
    }
    std::vector<int32_t> roff, radj;  // reverse edges (second pass only)
    auto dist_of = [&](int v) { return ss.seen[v] == ss.cur ? ss.dist[v] : std::numeric_limits<double>::infinity(); };
    auto prev_of = [&](int v) { return ss.seen[v] == ss.cur ? ss.prev[v] : -1; };
    // (restricted: rows from the packed download via row_of; -1 = a pop above the bound or
    // of a row not held, so the caller takes the whole table)
    thread_local std::vector<int32_t> row_of;
    const uint16_t* pk_ids = nbr16;
    const uint16_t* pk_rows = nbr16 + ids_pad;
    auto astar = [&](bool with_reverse, bool restricted) -> int {
        if (++ss.cur == 0u) {  // (stamp wrap-around: clear once)
            std::fill(ss.seen.begin(), ss.seen.end(), 0u);
            std::fill(ss.done.begin(), ss.done.end(), 0u);
            ss.cur = 1u;
        }
        // (the heap as std::priority_queue keeps it: push_heap / pop_heap with std::greater,
        // over storage reused across searches)
        std::vector<QE>& q = ss.heap;
        q.clear();
        const std::greater<QE> cmp;
        auto push = [&](QE e) {
            q.push_back(e);
            std::push_heap(q.begin(), q.end(), cmp);
        };
        ss.seen[0] = ss.cur;
        ss.dist[0] = 0.0;
        ss.prev[0] = -1;
        push({(node(0) - gp).norm(), 0});
        auto relax = [&](int u, const Vec3& pu, int v) {
            if (ss.done[v] == ss.cur) return;
            const double nd = ss.dist[u] + (node(v) - pu).norm();
            if (nd < dist_of(v)) {
                ss.seen[v] = ss.cur;
                ss.dist[v] = nd;
                ss.prev[v] = u;
                push({nd + (node(v) - gp).norm(), v});
            }
        };
        while (!q.empty()) {
            const double f = q.front().first;
            const int u = q.front().second;
            std::pop_heap(q.begin(), q.end(), cmp);
            q.pop_back();
            if (ss.done[u] == ss.cur) continue;
            const uint16_t* row = nullptr;
            if (restricted) {
                if (!(f <= bound) || row_of[u] < 0) return -1;
                row = pk_rows + (size_t)row_of[u] * k;
            }
            ss.done[u] = ss.cur;
            if (u == 1) return 1;
            const Vec3 pu = node(u);
            if (restricted) {
                for (int c = 0; c < k; ++c)
                    if (row[c] != 0xFFFF) relax(u, pu, (int)row[c]);
            } else {
                const size_t e0 = (size_t)u * k;
                for (int c = 0; c < k; ++c) {
                    const int v = nbr(e0 + c);
                    if (v >= 0) relax(u, pu, v);
                }
            }
            if (with_reverse)
                for (int32_t r = roff[u]; r < roff[u + 1]; ++r) relax(u, pu, radj[r]);
        }
        return 0;
    };
    int found = -1;
    if (restricted && ecnt[1] > 0 && ecnt[2] <= cap) {
        if (row_of.size() < (size_t)n) row_of.resize(n, -1);
        for (int64_t r = 0; r < ecnt[2]; ++r) row_of[pk_ids[r]] = (int32_t)r;
        found = astar(false, true);
        for (int64_t r = 0; r < ecnt[2]; ++r) row_of[pk_ids[r]] = -1;
    }
    if (found != 1) {
        if (restricted) {  // the whole table after all
            const auto t0 = std::chrono::steady_clock::now();
            whole_table();
            ms_dev += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        // (no forward edge into the goal: the forward pass cannot reach it — it would only
        // explore start's whole component first; same result, so go straight to the second)
        if (!goal_has_forward_edge || astar(false, false) != 1) {
            roff.assign(n + 1, 0);
            for (size_t e = 0; e < m; ++e)
                if (nbr(e) >= 0) ++roff[nbr(e) + 1];
            for (int i = 0; i < n; ++i) roff[i + 1] += roff[i];
            radj.resize(roff[n]);
            std::vector<int32_t> fill(roff.begin(), roff.end() - 1);
            for (int i = 0; i < n; ++i)
                for (int c = 0; c < k; ++c) {
                    const size_t e = (size_t)i * k + c;
                    if (nbr(e) >= 0) radj[fill[nbr(e)]++] = i;
                }
            astar(true, false);
        }
    }
    {
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_.states_sampled += samples;
        stats_.states_valid += n - 2;
        stats_.edges_checked += edges_checked;
        stats_.edges_valid += n_valid_edges;
        stats_.rows_downloaded += rows_down;
    }
    auto account = [&] {
        const auto t_end = std::chrono::steady_clock::now();
        std::lock_guard<std::mutex> lk(g_stats_mu);
        const double total = std::chrono::duration<double, std::milli>(t_end - t_dev0).count();
        stats_.ms_device += ms_dev;
        stats_.ms_search += total - ms_dev;
    };
    if (prev_of(1) < 0) {
        account();
        return false;
    }
    std::vector<Vec3> path;
    for (int v = 1; v >= 0; v = prev_of(v)) path.push_back({nodes[3 * v], nodes[3 * v + 1], nodes[3 * v + 2]});
    std::reverse(path.begin(), path.end());
    out = shortcut(path);
    account();
    return true;
}

// Greedy shortcutting with one batched check of every vertex pair (the role of
// PathSimplifier::reduceVertices in src/PathPlanner.cpp:138-139).
std::vector<Vec3> PathPlanner::shortcut(const std::vector<Vec3>& p) const {
    const size_t L = p.size();
    if (L < 3) return p;
    std::vector<double> s1, s2;
    std::vector<std::pair<int, int>> idx;
    for (size_t i = 0; i < L; ++i)
        for (size_t j = i + 2; j < L; ++j) {
            s1.insert(s1.end(), {p[i].x, p[i].y, p[i].z});
            s2.insert(s2.end(), {p[j].x, p[j].y, p[j].z});
            idx.push_back({(int)i, (int)j});
        }
    std::vector<uint8_t> ok(idx.size());
    worldPtr->checkRays(s1.data(), s2.data(), (int64_t)idx.size(), configParser->getPathPlannerProperties().canPassGate,
                        ok.data());
    std::vector<std::vector<uint8_t>> vis(L, std::vector<uint8_t>(L, 0));
    for (size_t e = 0; e < idx.size(); ++e) vis[idx[e].first][idx[e].second] = ok[e];
    std::vector<Vec3> out = {p[0]};
    size_t cur = 0;
    while (cur + 1 < L) {
        size_t nxt = cur + 1;  // a path edge, valid by construction
        for (size_t j = L - 1; j > cur + 1; --j)
            if (vis[cur][j]) {
                nxt = j;
                break;
            }
        out.push_back(p[nxt]);
        cur = nxt;
    }
    return out;
}

// The planner choice of src/PathPlanner.cpp:106-123.  "rrt" cannot be honoured (OMPL's
// RRT* is third-party and not part of this build; its `range` has no counterpart): it
// runs the same batch planner as "fmt", and says so once per process.  The reference
// itself never reads optimality_threshold_percentage (getStraightLineObjective,
// src/PathPlanner.cpp:160-168, is never called), so neither does this build.
static void checkPlannerConfig(const PathPlannerProperties& pp) {
    if (pp.planner != "rrt" && pp.planner != "fmt") {
        std::cerr << "Unknown planner" << std::endl;
        throw std::runtime_error("Unknown planner");  // :121-123
    }
    if (pp.planner == "rrt") {
        static std::once_flag once;
        std::call_once(once, [] {
            std::cerr << "PathPlanner: planner \"rrt\" runs the batch sampling planner of this build (OMPL's RRT* "
                         "is not available); path_planner_properties.range is not used"
                      << std::endl;
        });
    }
}

// PathPlanner::planPath — src/PathPlanner.cpp:80-158
bool PathPlanner::planPath(const Vec3& start, const Vec3& goal, double timeLimit, std::vector<Vec3>& resultPath) const {
    if (!resultPath.empty()) {
        resultPath.clear();
        std::cerr << "Result path not empty, clearing it" << std::endl;
    }
    checkPlannerConfig(configParser->getPathPlannerProperties());
    const auto t0 = std::chrono::steady_clock::now();
    {
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_ = PlannerStats();
    }
    const uint64_t call = __atomic_fetch_add(&calls_, 1, __ATOMIC_RELAXED);
    int attempts = 0;
    const bool ok = planCall(start, goal, timeLimit, call, resultPath, attempts);
    {
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_.attempts = attempts;
        stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return ok;
}

// One planPath problem with its call number (the seed): up to 4 attempts with doubled
// samples while inside timeLimit (the role of solve(timeLimit), src/PathPlanner.cpp:126-136)
bool PathPlanner::planCall(const Vec3& start, const Vec3& goal, double timeLimit, uint64_t call,
                           std::vector<Vec3>& out, int& attempts) const {
    const auto t0 = std::chrono::steady_clock::now();
    const auto& pp = configParser->getPathPlannerProperties();
    int64_t samples = pp.samplesFMT > 0 ? pp.samplesFMT : 4096;
    uint64_t seed = mix(seed_, call);
    for (int d = 0; d < 3; ++d) seed = mix(mix(seed, bits_of(start[d])), bits_of(goal[d]));
    bool ok = false;
    attempts = 0;
    for (; attempts < 4 && !ok; ++attempts) {
        ok = planOnce(start, goal, samples, mix(seed, attempts), out);
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!ok && el > timeLimit) {  // out of time: give up like solve(timeLimit)
            ++attempts;
            break;
        }
        samples *= 2;
    }
    if (!ok) out.clear();
    return ok;
}

void PathPlanner::planPaths(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                            std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok) const {
    checkPlannerConfig(configParser->getPathPlannerProperties());
    const size_t n = problems.size();
    paths.assign(n, {});
    ok.assign(n, 0);
    if (n == 0) return;
    const auto t0 = std::chrono::steady_clock::now();
    {
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_ = PlannerStats();
    }
    const uint64_t base = __atomic_fetch_add(&calls_, (uint64_t)n, __ATOMIC_RELAXED);
    std::vector<int> attempts(n, 0);
    std::vector<std::exception_ptr> err(n);
    auto run = [&](size_t i) {
        try {
            ok[i] = planCall(problems[i].first, problems[i].second, timeLimit, base + i, paths[i], attempts[i]) ? 1 : 0;
        } catch (...) {
            err[i] = std::current_exception();
        }
    };
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    (void)worldPtr->device();  // build the device world once, before the threads share it
    // problems 1.. on persistent pool threads (their ThreadScratch -- stream, device and
    // pinned buffers -- survives between calls), problem 0 on the calling thread
    std::mutex done_mu;
    std::condition_variable done_cv;
    const char* conc = std::getenv("EPP_PLAN_CONCURRENT");  // 0: one after the other (A/B)
    if (conc && std::atoi(conc) == 0) {
        for (size_t i = 0; i < n; ++i) run(i);
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_.attempts = *std::max_element(attempts.begin(), attempts.end());
        stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        for (const auto& e : err)
            if (e) std::rethrow_exception(e);
        return;
    }
    // W concurrent planners (the caller + W-1 pool threads) pull problems in order: more
    // than the hardware queues a process gets (4) only adds host contention
    const char* thr = std::getenv("EPP_PLAN_THREADS");
    const size_t W = std::min(n, (size_t)std::max(1, thr ? std::atoi(thr) : 4));
    std::atomic<size_t> next{0};
    auto drain = [&] {
        for (size_t i = next++; i < n; i = next++) run(i);
    };
    size_t pending = W - 1;
    for (size_t w = 1; w < W; ++w)
        plan_pool().submit([&, dev] {
            (void)hipSetDevice(dev);
            drain();
            std::lock_guard<std::mutex> lk(done_mu);
            if (--pending == 0) done_cv.notify_all();
        });
    drain();
    {
        std::unique_lock<std::mutex> lk(done_mu);
        done_cv.wait(lk, [&] { return pending == 0; });
    }
    for (const auto& e : err)
        if (e) std::rethrow_exception(e);
    std::lock_guard<std::mutex> lk(g_stats_mu);
    stats_.attempts = *std::max_element(attempts.begin(), attempts.end());
    stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// PathPlanner::includeGates2 — src/PathPlanner.cpp:175-230
std::vector<Vec3> PathPlanner::includeGates2(std::vector<std::vector<Vec3>> waypoints) const {
    std::vector<Vec3> gateCenters;
    for (size_t s = 0; s + 1 < waypoints.size(); ++s) {
        const Vec3& a = waypoints[s].back();
        const Vec3& b = waypoints[s + 1].front();
        gateCenters.push_back((a + b) / 2);
    }
    for (size_t i = 0; i < gateCenters.size(); ++i) {
        waypoints[i].push_back(gateCenters[i]);
        waypoints[i + 1].insert(waypoints[i + 1].begin(), gateCenters[i]);
    }
    const std::string method = configParser->getPathPlannerProperties().pathSimplification;
    std::vector<Vec3> flat;
    for (const auto& seg : waypoints) {
        std::vector<Vec3> pruned;
        if (method == "none") {
            pruned = seg;
        } else if (method == "custom") {
            pruned = pruneWaypoints(seg);
        } else if (method == "ompl") {
            // smoothBSpline (OMPL) is not part of this build; the shortcut keeps the path valid
            pruned = shortcut(seg);
        } else {
            std::cerr << "Unknown pruning method" << std::endl;
            throw std::runtime_error("Unknown pruning method");
        }
        for (const auto& w : pruned) {
            if (!flat.empty() && (flat.back() - w).norm() < 0.05) continue;  // :222
            flat.push_back(w);
        }
    }
    return flat;
}

// PathPlanner::pruneWaypoints — src/PathPlanner.cpp:232-265.  The reference checks
// ray(reference, current) one at a time; every pair it could ask for is checked in one
// batch and the same greedy walk is replayed on the answers.
std::vector<Vec3> PathPlanner::pruneWaypoints(const std::vector<Vec3>& w) const {
    if (w.size() < 3) return w;
    const size_t L = w.size();
    std::vector<double> s1, s2;
    std::vector<std::pair<int, int>> idx;
    for (size_t i = 0; i < L; ++i)
        for (size_t j = i + 2; j < L; ++j) {
            s1.insert(s1.end(), {w[i].x, w[i].y, w[i].z});
            s2.insert(s2.end(), {w[j].x, w[j].y, w[j].z});
            idx.push_back({(int)i, (int)j});
        }
    std::vector<uint8_t> ok(idx.size());
    worldPtr->checkRays(s1.data(), s2.data(), (int64_t)idx.size(), true, ok.data());  // canPassGate = true
    std::vector<std::vector<uint8_t>> vis(L, std::vector<uint8_t>(L, 1));
    for (size_t e = 0; e < idx.size(); ++e) vis[idx[e].first][idx[e].second] = ok[e];
    std::vector<Vec3> pruned = {w[0]};
    size_t ref = 0;
    for (size_t cur = 2; cur < L; ++cur) {
        if (!vis[ref][cur]) {
            pruned.push_back(w[cur - 1]);
            ref = cur - 1;
        }
    }
    pruned.push_back(w[L - 1]);
    return pruned;
}

// PathPlanner::checkTrajectoryValidity — src/PathPlanner.cpp:267-280 (one batched launch)
bool PathPlanner::checkTrajectoryValidity(const Matrix& traj, double minDistance) const {
    return checkTrajectoryValidityOn(*worldPtr, traj, minDistance);
}

bool PathPlanner::checkTrajectoryValidityAndGenerate(const Matrix& traj, double minDistance,
                                                     const std::vector<Vec3>& waypoints, double vMax, double aMax,
                                                     double samplingInterval, double startTimeOffset, const Vec3& v0,
                                                     const Vec3& a0, Matrix& result) const {
    if (waypoints.size() < 2) throw std::invalid_argument("At least two waypoints are required");
    thread_local std::vector<double> xyz, wp;
    thread_local std::vector<uint8_t> ok;
    xyz.resize(traj.rows * 3);
    for (size_t i = 0; i < traj.rows; ++i) {
        xyz[3 * i] = traj(i, 0);
        xyz[3 * i + 1] = traj(i, 3);
        xyz[3 * i + 2] = traj(i, 6);
    }
    wp.resize(waypoints.size() * 3);
    for (size_t i = 0; i < waypoints.size(); ++i) {
        wp[3 * i] = waypoints[i].x;
        wp[3 * i + 1] = waypoints[i].y;
        wp[3 * i + 2] = waypoints[i].z;
    }
    ok.assign(traj.rows, 0);
    const double v[3] = {v0.x, v0.y, v0.z}, a[3] = {a0.x, a0.y, a0.z};
    const FusedCheck chk{worldPtr->device(), xyz.data(), (int64_t)traj.rows, minDistance, ok.data()};
    Matrix tmp;
    std::swap(tmp, result);  // (result keeps its old value if the call throws)
    auto into = [](void* ctx, int64_t R) -> double* {
        Matrix& m = *static_cast<Matrix*>(ctx);
        m.rows = (size_t)R;
        m.cols = 10;
        m.data.resize((size_t)std::max<int64_t>(R, 1) * 10);
        return m.data.data();
    };
    int64_t n = 0;
    const epp_status rc = check_and_generate_into(traj.rows ? &chk : nullptr, wp.data(), (int32_t)waypoints.size(),
                                                  nullptr, vMax, aMax, samplingInterval, startTimeOffset, v, a, into,
                                                  &tmp, &n);
    if (rc == EPP_ERR_UNSUPPORTED) {  // (a large check: the two calls)
        std::swap(tmp, result);
        const bool valid = checkTrajectoryValidity(traj, minDistance);
        poly_traj::generateTrajectory(waypoints, vMax, aMax, samplingInterval, startTimeOffset, v0, a0, result);
        return valid;
    }
    if (rc != EPP_OK) {
        std::swap(tmp, result);
        if (rc == EPP_ERR_INVALID_ARGUMENT) throw std::invalid_argument(epp_last_error());
        throw std::runtime_error(std::string("generateTrajectory: ") + epp_last_error());
    }
    tmp.data.resize((size_t)n * 10);
    std::swap(tmp, result);
    for (uint8_t v8 : ok)
        if (!v8) return false;
    return true;
}

bool PathPlanner::checkTrajectoryValidityOn(const World& world, const Matrix& traj, double minDistance) {
    if (traj.rows == 0) return true;
    std::vector<double> xyz(traj.rows * 3);
    for (size_t i = 0; i < traj.rows; ++i) {
        xyz[3 * i] = traj(i, 0);
        xyz[3 * i + 1] = traj(i, 3);
        xyz[3 * i + 2] = traj(i, 6);
    }
    std::vector<uint8_t> ok(traj.rows);
    world.checkPointsMinDistance(xyz.data(), (int64_t)traj.rows, minDistance, ok.data());
    for (uint8_t v : ok)
        if (!v) return false;
    return true;
}

}  // namespace epp

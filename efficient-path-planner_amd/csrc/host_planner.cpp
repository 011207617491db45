// host_planner.cpp — epp::PathPlanner (drop-in for src/PathPlanner.cpp) on the batch
// GPU planner.  See include/epp/PathPlanner.h for the algorithm.
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
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
#include <immintrin.h>

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

PathPlanner::PathPlanner(const Matrix& gates, const Matrix& obstacles, std::shared_ptr<ConfigParser> cp,
                         AbiTag abi)
    : configParser(std::move(cp)) {
    if (abi.planner_size != sizeof(PathPlanner) || abi.stats_size != sizeof(PlannerStats) ||
        abi.version != kPlannerAbiVersion)
        throw std::runtime_error("PathPlanner: caller built against another epp/PathPlanner.h (PathPlanner " +
                                 std::to_string(abi.planner_size) + " B, PlannerStats " +
                                 std::to_string(abi.stats_size) + " B, version " + std::to_string(abi.version) +
                                 "; this library: " + std::to_string(sizeof(PathPlanner)) + " B, " +
                                 std::to_string(sizeof(PlannerStats)) + " B, version " +
                                 std::to_string(kPlannerAbiVersion) + "): rebuild the caller");
    worldPtr = std::make_shared<World>(configParser);
    parseGatesAndObstacles(gates, obstacles);  // src/PathPlanner.cpp:27-35
    // knobs of this build, read once: EPP_PLAN_ELLIPSE the row-restricted search's bound
    // factor (0: the whole table only; else >= 1), EPP_PLAN_THREADS the planner threads
    if (const char* ev = std::getenv("EPP_PLAN_ELLIPSE")) {
        char* end = nullptr;
        const double f = std::strtod(ev, &end);
        if (end != ev && *end == '\0' && (f == 0.0 || f >= 1.0)) ellipse_ = f;
        else std::cerr << "PathPlanner: EPP_PLAN_ELLIPSE=" << ev << " ignored (0, or a factor >= 1)" << std::endl;
    }
    if (const char* tv = std::getenv("EPP_PLAN_THREADS")) {
        const int t = std::atoi(tv);
        if (t >= 1 && t <= 64) threads_ = t;
    }
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

namespace {
// Per calling thread: the batched planner's device workspace, pinned host block and stream
// (grown geometrically; freeing pinned memory synchronises the device).
class BatchScratch {
public:
    static BatchScratch& get() {
        thread_local BatchScratch b;
        return b;
    }
    void ensure(size_t dev_bytes, size_t host_bytes) {
        if (dev_bytes > dcap_) {
            dev_bytes = std::max(dev_bytes, dcap_ + dcap_ / 2);
            if (dev_) epp_free(dev_);
            dev_ = nullptr;
            dcap_ = 0;
            check(epp_malloc(&dev_, dev_bytes), "planner batch workspace");
            dcap_ = dev_bytes;
        }
        if (host_bytes > hcap_) {
            host_bytes = std::max(host_bytes, hcap_ + hcap_ / 2);
            if (host_) (void)hipHostFree(host_);
            host_ = nullptr;
            hcap_ = 0;
            if (hipHostMalloc(&host_, host_bytes, hipHostMallocDefault) != hipSuccess) {
                host_ = nullptr;
                throw std::runtime_error("planner batch: hipHostMalloc failed");
            }
            std::memset(host_, 0, host_bytes);  // (completion slots: no stale sequence numbers)
            hcap_ = host_bytes;
        }
    }
    void* dev() const { return dev_; }
    char* host() const { return static_cast<char*>(host_); }
    uint32_t next_seq() { return ++seq_ ? seq_ : ++seq_; }  // (never 0: fresh slots read 0)
    // Buffers of the whole-table search of one problem per planner thread (w), sized here
    // for n nodes: allocated with the batch, not on the planner threads when a search falls
    // back (a first allocation of pinned memory there took milliseconds).
    struct Area {
        void* dev = nullptr;
        void* pin = nullptr;
        void* stream = nullptr;
        size_t dcap = 0, pcap = 0;
        bool cold = true;  // no whole-table search has run on it yet
    };
    static size_t r256(size_t b) { return (b + 255) & ~size_t(255); }
    // device: [edge counts | table (i32) | table (u16) | motion flags | k-NN workspace | the
    // reverse CSR: counts, fill, roff (n + 1), radj (i32), radj (u16)]; pinned: [edge counts
    // | nodes | table | roff | radj]
    static size_t area_dev_bytes(int64_t n, int k) {
        const size_t m = (size_t)n * k;
        return r256(16) + r256(m * 4) + r256(m * 2) + r256(m) + r256((size_t)epp_knn_workspace_size((int32_t)n)) +
               3 * r256((size_t)(n + 1) * 4) + r256(m * 4) + r256(m * 2);
    }
    static size_t area_pin_bytes(int64_t n, int k) {
        return r256(64) + r256((size_t)n * 24) + r256((size_t)n * k * 4) + r256((size_t)(n + 1) * 4) +
               r256((size_t)n * k * 4);
    }
    void ensure_areas(size_t W, int64_t n, int k) {
        if (areas_.size() < W) areas_.resize(W);
        const size_t db = area_dev_bytes(n, k), pb = area_pin_bytes(n, k);
        for (size_t w = 0; w < W; ++w) {
            Area& a = areas_[w];
            if (!a.stream) check(epp_stream_create(&a.stream), "stream");
            if (db > a.dcap) {
                if (a.dev) epp_free(a.dev);
                a.dev = nullptr;
                a.dcap = 0;
                check(epp_malloc(&a.dev, db), "planner fallback workspace");
                a.dcap = db;
            }
            if (pb > a.pcap) {
                if (a.pin) (void)hipHostFree(a.pin);
                a.pin = nullptr;
                a.pcap = 0;
                if (hipHostMalloc(&a.pin, pb, hipHostMallocDefault) != hipSuccess) {
                    a.pin = nullptr;
                    throw std::runtime_error("planner fallback: hipHostMalloc failed");
                }
                a.pcap = pb;
                // one DMA over the whole buffer now: the first transfers into fresh pinned
                // memory are slow (a first fallback took ~10 ms), and they belong here, with
                // the allocation (the cold first plan), not in a search
                check(epp_memcpy_d2h_async(a.pin, a.dev, std::min(pb, a.dcap), a.stream), "planner fallback warm-up");
                check(epp_stream_sync(a.stream), "planner fallback warm-up");
                // (cold stays as it was: a grown area -- a retry with doubled samples -- has
                // had its warm-up search; a new one starts cold)
            }
        }
    }
    Area& area(size_t w) { return areas_[w]; }
    void* stream() {
        if (!stream_) check(epp_stream_create(&stream_), "stream");
        return stream_;
    }
    ~BatchScratch() {
        if (dev_) epp_free(dev_);
        if (host_) (void)hipHostFree(host_);
        if (stream_) epp_stream_destroy(stream_);
        for (Area& a : areas_) {
            if (a.dev) epp_free(a.dev);
            if (a.pin) (void)hipHostFree(a.pin);
            if (a.stream) epp_stream_destroy(a.stream);
        }
    }

private:
    std::vector<Area> areas_;
    void* dev_ = nullptr;
    void* host_ = nullptr;
    void* stream_ = nullptr;
    size_t dcap_ = 0, hcap_ = 0;
    uint32_t seq_ = 0;
};

// A*'s state per host thread, reused across searches: an entry counts only when its stamp
// is the search's (no O(n) clearing per search); the heap keeps its storage.
struct QE {  // (16 bytes: the heap moves less than with a separate tie-break key)
    double f;
    int v;  // the node (its index is in node order): ties in f pop the lower index first, as
            // std::priority_queue<pair<double, int>, ..., std::greater<>> does
};
struct QECmp {
    bool operator()(const QE& a, const QE& b) const { return b.f < a.f || (!(a.f < b.f) && b.v < a.v); }
};
struct SearchState {
    std::vector<double> dist;
    std::vector<int> prev;
    std::vector<uint32_t> seen, done;  // stamps: dist/prev valid, closed
    std::vector<QE> heap;
    uint32_t cur = 0;
    int64_t pops = 0;  // (diagnostics: nodes closed by the last search)
    void begin(size_t n) {
        if (dist.size() < n) {  // (grown with room to spare, the heap's storage reserved: a
                                // thread's first searches pay the page faults, not later ones)
            const size_t c = std::max<size_t>(n, std::max<size_t>(2 * dist.size(), 16384));
            dist.resize(c);
            prev.resize(c);
            seen.resize(c, 0u);
            done.resize(c, 0u);
            heap.reserve(16 * c);
        }
        if (++cur == 0u) {  // (stamp wrap-around: clear once)
            std::fill(seen.begin(), seen.end(), 0u);
            std::fill(done.begin(), done.end(), 0u);
            cur = 1u;
        }
        heap.clear();
    }
    int prev_of(int v) const { return seen[v] == cur ? prev[v] : -1; }
};

// A planner thread's buffers of the restricted search (grown with room to spare; warmed
// once per thread, before its first problem: a thread whose first problem came in a timed
// call paid the page faults there -- the second plan of a generator took ~2x).
struct SolveScratch {
    std::vector<double> ndc;      // the problem's referenced nodes (a private copy)
    std::vector<uint16_t> rowc;   // its rows (a private copy)
    std::vector<int32_t> row_of;  // compact node -> row
    std::vector<int32_t> roff, radj, rfill;  // the rows' reverse edges (symmetrised search)
    SearchState ss;
    bool warm = false;
    static SolveScratch& get() {
        thread_local SolveScratch s;
        return s;
    }
    void warmup(int k) {
        if (warm) return;
        warm = true;
        ndc.assign(3 * 16384, 0.0);
        rowc.assign((size_t)16384 * k, 0);
        row_of.assign(16384, -1);
        roff.assign(16385, 0);  // (the symmetrised search's: rare, but its first use is in a timed plan)
        rfill.assign(16384, 0);
        radj.assign((size_t)16384 * k, 0);
        ss.begin(16384);
        ss.heap.resize(ss.heap.capacity() / 4);  // (touch part of the heap's storage)
        ss.heap.clear();
    }
};

// EPP_PLAN_TRACE=1 (diagnostics): the fallback's phases on stderr
// EPP_PAIRS_TRACE=1 (diagnostics): the shortcut's and the pruning's batched ray checks --
// pairs and wall time of each batch -- to stderr
static bool pairs_trace() {
    static const bool t = [] {
        const char* e = std::getenv("EPP_PAIRS_TRACE");
        return e && std::atoi(e) == 1;
    }();
    return t;
}

bool plan_trace() {
    static const bool t = [] {
        const char* e = std::getenv("EPP_PLAN_TRACE");
        return e && std::atoi(e) == 1;
    }();
    return t;
}

// A* from node 0 to node 1 with the Euclidean distance to the goal (admissible and
// consistent for Euclidean edge costs).  pos(v): coordinates (node indices in node order:
// the lower breaks ties); expand(u, f, relax) calls relax(v) for u's edges and returns false to abort
// (the caller then takes another graph).  Returns 1 (goal closed), 0 (exhausted), -1
// (aborted).
template <class Pos, class Expand>
int astar(SearchState& ss, size_t nv, Pos&& pos, Expand&& expand) {
    ss.begin(nv);
    ss.pops = 0;
    const QECmp cmp;
    std::vector<QE>& q = ss.heap;
    const Vec3 gp = pos(1);
    auto push = [&](QE e) {
        q.push_back(e);
        std::push_heap(q.begin(), q.end(), cmp);
    };
    ss.seen[0] = ss.cur;
    ss.dist[0] = 0.0;
    ss.prev[0] = -1;
    push({(pos(0) - gp).norm(), 0});
    while (!q.empty()) {
        const QE top = q.front();
        std::pop_heap(q.begin(), q.end(), cmp);
        q.pop_back();
        const int u = top.v;
        if (ss.done[u] == ss.cur) continue;
        ++ss.pops;
        const Vec3 pu = pos(u);
        auto relax = [&](int v) {
            if (ss.done[v] == ss.cur) return;
            const Vec3 pv = pos(v);
            const double nd = ss.dist[u] + (pv - pu).norm();
            if (!(ss.seen[v] == ss.cur) || nd < ss.dist[v]) {
                ss.seen[v] = ss.cur;
                ss.dist[v] = nd;
                ss.prev[v] = u;
                push({nd + (pv - gp).norm(), v});
            }
        };
        if (!expand(u, top.f, relax, /*closing=*/false)) return -1;
        ss.done[u] = ss.cur;
        if (u == 1) return 1;
        expand(u, top.f, relax, /*closing=*/true);
    }
    return 0;
}
}  // namespace

// One attempt for a batch of problems (the same sample count; their own seeds):
// the device stages in one launch each (plan_batch_launch), then per problem, on the
// planner threads, A* over its emitted rows (the row-restricted search) or, when that
// cannot decide, over the whole k-NN table of its nodes; then one batched shortcut.
void PathPlanner::planAttempt(const std::vector<std::pair<Vec3, Vec3>>& problems, const std::vector<uint64_t>& seeds,
                              int64_t samples, std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                              GateEnds* ends) const {
    const size_t np = problems.size();
    paths.assign(np, {});
    ok.assign(np, 0);
    for (size_t b0 = 0; b0 < np; b0 += 64) {  // (at most 64 problems per launch set)
        const size_t b1 = std::min(np, b0 + 64);
        std::vector<std::pair<Vec3, Vec3>> sub(problems.begin() + b0, problems.begin() + b1);
        std::vector<uint64_t> sseeds(seeds.begin() + b0, seeds.begin() + b1);
        std::vector<std::vector<Vec3>> sp;
        std::vector<char> so;
        planChunk(sub, sseeds, samples, sp, so, ends ? ends + b0 : nullptr);
        for (size_t i = b0; i < b1; ++i) {
            paths[i] = std::move(sp[i - b0]);
            ok[i] = so[i - b0];
        }
    }
}

void PathPlanner::planChunk(const std::vector<std::pair<Vec3, Vec3>>& problems, const std::vector<uint64_t>& seeds,
                            int64_t samples, std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                            GateEnds* ends) const {
    const auto& pp = configParser->getPathPlannerProperties();
    const auto& wp = configParser->getWorldProperties();
    const bool canPass = pp.canPassGate;  // validators get can_pass_gate  src/PathPlanner.cpp:47-50
    const epp_world* w = worldPtr->device();
    const int k = k_;
    const int S = (int)problems.size();
    const auto t_dev0 = std::chrono::steady_clock::now();
    const double lo[3] = {wp.lowerBound.x, wp.lowerBound.y, wp.lowerBound.z};
    const double hi[3] = {wp.upperBound.x, wp.upperBound.y, wp.upperBound.z};
    // ---- the problems: seeds, ends, the k-NN box, the restricted rows' ellipsoid -------
    // Row-restricted search: A* pops nodes in increasing f = g + h >= |x - start| + |x - goal|,
    // so a search that reaches the goal with every popped f <= bound has expanded only
    // nodes inside the ellipsoid |x - start| + |x - goal| <= bound, and pops exactly what the
    // search over the whole table pops (a node outside has f > bound >= the path's length):
    // the same path.  bound = ellipse_ * |start - goal| + 0.25 m; capacity 1.25 x the
    // ellipsoid's expected rows (its volume, unclipped, over the sampling box's) + 1024, not
    // past half the nodes.  Otherwise (a pop above the bound, rows past the capacity, no kept
    // edge into the goal among the rows, more than 65,535 nodes) the whole table is built.
    const int64_t nmax = samples + 2;
    // (the rows' motion check needs the world's tile tables: a world without OBBs or past the
    // LDS budget builds every problem's whole table, whose check has the other kernels)
    const bool restrict_ok = ellipse_ >= 1.0 && (k == 4 || k == 8 || k == 16) && nmax <= 4 * 65536 &&
                             knn_motions_rows_supported(w);
    // the rows' k-NN grid: cells of ~1.5 nodes (the sampling density), over the nodes of the
    // ellipsoid bound + 7.5 cells (a query's search radius r stays below half the margin:
    // |x - s| + |x - g| is 2-Lipschitz, so every node within r of a row's node is in it)
    const double vbox = (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]);
    const double cell = std::cbrt(1.5 * std::max(vbox, 1e-12) / (double)nmax);
    std::vector<PlanSeg> segs(S);
    std::vector<std::array<double, 6>> kbox(S);  // the whole table's k-NN box (fallback)
    for (int p = 0; p < S; ++p) {
        const Vec3& s = problems[p].first;
        const Vec3& g = problems[p].second;
        PlanSeg& q = segs[p];
        q = PlanSeg{};
        q.seed = seeds[p];
        for (int d = 0; d < 3; ++d) {
            q.s[d] = s[d];
            q.g[d] = g[d];
            // the grid over the sampling box widened by start and goal (every node lies inside)
            kbox[p][d] = std::min({lo[d], s[d], g[d]});
            kbox[p][3 + d] = std::max({hi[d], s[d], g[d]});
        }
        const double d_sg = (g - s).norm();
        q.bound = ellipse_ * d_sg + 0.25;
        q.gbound = q.bound + 7.5 * cell;
        q.h = cell;
        {  // the gbound ellipsoid's box (foci s, g), padded, clipped to the k-NN box
            const double a = 0.5 * q.gbound, b2 = std::max(0.0, a * a - 0.25 * d_sg * d_sg);
            for (int d = 0; d < 3; ++d) {
                const double u = d_sg > 0 ? (g[d] - s[d]) / d_sg : 0.0;
                const double e = std::sqrt(a * a * u * u + b2 * (1.0 - u * u)) * (1.0 + 1e-6) + 1e-6;
                const double c = 0.5 * (s[d] + g[d]);
                q.glo[d] = std::max(kbox[p][d], c - e);
                q.ghi[d] = std::min(kbox[p][3 + d], c + e);
            }
        }
        q.cap = 0;
        if (restrict_ok) {
            const double vbox = (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]);
            const double vell = M_PI * q.bound * (q.bound * q.bound - d_sg * d_sg) / 6.0;
            const double frac = vbox > 0 ? std::min(1.0, vell / vbox) : 1.0;
            const double want = 1.25 * frac * (double)nmax + 1024.0;
            if (want < 0.5 * (double)nmax) q.cap = (int32_t)want;
        }
    }
    const PlanBatchLayout L = plan_batch_layout(S, samples, k, segs.data());
    BatchScratch& bs = BatchScratch::get();
    bs.ensure(L.dev_bytes, L.host_bytes);
    // W concurrent solvers (the caller + W - 1 pool threads), each with its fallback buffers
    const size_t W = std::min((size_t)S, (size_t)std::max(1, threads_));  // (threads_: 16 by default)
    bs.ensure_areas(W, nmax, k);
    char* H = bs.host();
    std::memcpy(H + L.h_seg, segs.data(), sizeof(PlanSeg) * S);
    void* st = bs.stream();
    const uint64_t* hdr = reinterpret_cast<const uint64_t*>(H + L.h_hdr);
    const uint32_t* slots = reinterpret_cast<const uint32_t*>(H + L.h_slot);
    const uint16_t* rows = reinterpret_cast<const uint16_t*>(H + L.h_rows);
    const double* need = reinterpret_cast<const double*>(H + L.h_need);
    auto hv = [&](int field, int p) { return (int64_t)hdr[kPbPerSeg + field * S + p]; };
    std::vector<int64_t> first(S + 1, 0);  // rows are dense in problem order (set once the results are in)
    const char* dev = static_cast<const char*>(bs.dev());

    // ---- per problem: the restricted search, else the whole table ----------------------
    struct Out {
        int64_t n = 0, edges_checked = 0, edges_valid = 0, rows_down = 0, restricted_rows = 0;
        int fallback = 0;  // 1: the whole table after the restricted rows could not decide
        int why = -1;      // (PlannerStats::fallback_why)
        double ms_dev = 0, ms_search = 0;
        double ms_restricted = 0;  // the restricted search alone (row_of + A*)
        double ms_copy = 0;        // (of which: the copy out of pinned memory)
        int64_t pops = 0, nodes = 0;
        int symmetrised = 0;       // the restricted rows decided the symmetrised search
        int census = 0;            // ... after the whole table's k-NN counted the goal's edges
    };
    std::vector<Out> res(S);
    std::vector<std::vector<Vec3>> raw(S);
    std::vector<char> found(S, 0);
    std::vector<std::exception_ptr> err(S);
    auto solve = [&](int p, size_t w) {
        Out& o = res[p];
        const int64_t n = hv(3, p);
        o.n = n;
        const int64_t packed = hv(0, p);
        const int64_t m = std::min<int64_t>(hv(4, p), segs[p].need_cap);
        const auto t0 = std::chrono::steady_clock::now();
        int r = 0;
        // (restricted: rows within capacity, exact (hv 5), node ids in u16; start and goal are
        // compact indices 0 and 1: rows of their own)
        if (segs[p].cap > 0) o.why = (n > 65535 || packed > segs[p].cap || m < 2) ? 0 : hv(5, p) != 0 ? 1 : -1;
        if (segs[p].cap > 0 && n <= 65535 && packed <= segs[p].cap && hv(5, p) == 0 && m >= 2) {
            // this problem's rows and referenced nodes (compact indices: node order), copied
            // out of the pinned buffer first: the device wrote them, so they are in no CPU
            // cache, and A*'s scattered reads would each wait out a DRAM access (~70 ns; the
            // slowest search of a call took 0.15 ms for ~130 pops), where one sequential copy
            // streams them in
            const int64_t nrow = first[p + 1] - first[p];
            SolveScratch& sc = SolveScratch::get();
            std::vector<double>& ndc = sc.ndc;
            std::vector<uint16_t>& rowc = sc.rowc;
            auto grow = [](auto& v, size_t need, size_t init) {  // (room to spare: see SearchState::begin)
                if (v.size() < need) v.resize(std::max<size_t>(need, std::max<size_t>(2 * v.size(), init)));
            };
            grow(ndc, (size_t)m * 3, 3 * 16384);
            grow(rowc, (size_t)nrow * k, (size_t)16384 * k);
            std::memcpy(ndc.data(), need + 3 * segs[p].need_off, (size_t)m * 24);
            std::memcpy(rowc.data(), rows + (size_t)first[p] * k, (size_t)nrow * k * 2);
            o.ms_copy = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            const double* nd = ndc.data();
            std::vector<int32_t>& row_of = sc.row_of;
            grow(row_of, (size_t)m, 16384);
            std::fill(row_of.begin(), row_of.begin() + m, -1);
            for (int64_t sl = first[p]; sl < first[p + 1]; ++sl) row_of[slots[sl] & 0xFFFFu] = (int32_t)(sl - first[p]);
            SearchState& ss = sc.ss;
            const double bound = segs[p].bound;
            auto pos = [&](int v) { return Vec3(nd[3 * v], nd[3 * v + 1], nd[3 * v + 2]); };
            // (no kept edge into the goal among the rows: the forward search on them cannot
            // reach it -- the goal-edge count below decides instead, r = -1)
            const bool goal_edges = hv(2, p) > 0;
            r = -1;
            if (goal_edges)
                r = astar(ss, (size_t)m, pos, [&](int u, double f, auto&& relax, bool closing) {
                    if (!closing) return (f <= bound) && row_of[u] >= 0;
                    const uint16_t* row = rowc.data() + (size_t)row_of[u] * k;
                    for (int c = 0; c < k; ++c)
                        if (row[c] != 0xFFFF) relax((int)row[c]);
                    return true;
                });
            o.restricted_rows = packed;
            o.pops = goal_edges ? ss.pops : 0;
            o.nodes = m;
            o.why = r == -1 ? 3 : r == 0 ? 4 : -1;
            // The symmetrised search on the rows.  The reference's next step after a failed
            // forward search is the symmetrised graph (wholeTableSearch): a node's edges are
            // its row and the reverse of every row holding it.  While the pops stay within the
            // bound the reverse edges needed are those of rows here: a node without a row lies
            // outside the ellipse (|s w| + |w g| > bound), so it is pushed with f > bound and
            // never popped first.  Reverse edges ascending (compact = node order), as the
            // device's reverse CSR gives them.  Valid only once the whole table's forward
            // search is known to fail (below).
            auto symmetrised = [&]() -> int {
                std::vector<int32_t>& roff = sc.roff;
                std::vector<int32_t>& radj = sc.radj;
                grow(roff, (size_t)m + 1, 16384);
                std::fill(roff.begin(), roff.begin() + m + 1, 0);
                for (int u = 0; u < m; ++u) {
                    if (row_of[u] < 0) continue;
                    const uint16_t* row = rowc.data() + (size_t)row_of[u] * k;
                    for (int c = 0; c < k; ++c)
                        if (row[c] != 0xFFFF) ++roff[(size_t)row[c] + 1];
                }
                for (int64_t v = 0; v < m; ++v) roff[(size_t)v + 1] += roff[(size_t)v];
                grow(radj, (size_t)roff[(size_t)m], (size_t)16384 * k);
                std::vector<int32_t>& fill = sc.rfill;
                grow(fill, (size_t)m, 16384);
                std::copy(roff.begin(), roff.begin() + m, fill.begin());
                for (int u = 0; u < m; ++u) {  // (u ascending: every run comes out sorted)
                    if (row_of[u] < 0) continue;
                    const uint16_t* row = rowc.data() + (size_t)row_of[u] * k;
                    for (int c = 0; c < k; ++c)
                        if (row[c] != 0xFFFF) radj[(size_t)fill[row[c]]++] = u;
                }
                const int r2 = astar(ss, (size_t)m, pos, [&](int u, double f, auto&& relax, bool closing) {
                    if (!closing) return (f <= bound) && row_of[u] >= 0;
                    const uint16_t* row = rowc.data() + (size_t)row_of[u] * k;
                    for (int c = 0; c < k; ++c)
                        if (row[c] != 0xFFFF) relax((int)row[c]);
                    for (int32_t q = roff[(size_t)u]; q < roff[(size_t)u + 1]; ++q) relax(radj[(size_t)q]);
                    return true;
                });
                o.pops += ss.pops;
                o.why = r2 == -1 ? 5 : r2 == 0 ? 6 : -1;
                o.symmetrised = r2 == 1 ? 1 : 0;
                return r2;
            };
            auto take_path = [&]() {
                std::vector<Vec3> path;
                for (int v = 1; v >= 0; v = ss.prev_of(v)) path.push_back(pos(v));
                std::reverse(path.begin(), path.end());
                raw[p] = std::move(path);
                found[p] = 1;
            };
            if (r == 0) {
                // The forward search exhausted its component with every pop inside the bound:
                // every node it reached has its row here, so the whole table's forward search
                // reaches the same nodes and fails too.
                r = symmetrised();
            } else if (!goal_edges) {
                // No kept edge into the goal among the rows: the whole table's forward search
                // fails if no node outside the rows keeps one either.  Its masked k-NN (on the
                // device) counts them while the symmetrised search runs on the rows here; with
                // none, that search decides and the table is not downloaded.
                o.ms_restricted = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                o.ms_search += o.ms_restricted;
                o.fallback = 1;
                o.why = 2;
                const std::function<bool()> rows_sym = [&]() {
                    const auto ts0 = std::chrono::steady_clock::now();
                    const int r2 = symmetrised();  // (o.why: 5 / 6 when it fails)
                    if (plan_trace())
                        std::cerr << "[plan trace] problem " << p << ": symmetrised search on " << nrow << " rows / "
                                  << m << " nodes: " << o.pops << " closed, "
                                  << std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count()
                                  << " ms, result " << r2 << " (copies before: " << o.ms_restricted << " ms)" << std::endl;
                    return r2 == 1;
                };
                bool on_rows = false;
                int64_t census = 0;
                const double* d_nodes = reinterpret_cast<const double*>(dev + L.o_nodes) + (size_t)p * L.NS * 3;
                found[p] = wholeTableSearch(d_nodes, (int32_t)n, kbox[p].data(), kbox[p].data() + 3, &bs.area(w),
                                            raw[p], o.edges_checked, o.edges_valid, o.ms_dev, o.ms_search, &rows_sym,
                                            &on_rows, &census)
                               ? 1
                               : 0;
                // why the whole table was searched: a kept goal edge outside the rows (2), else
                // the rows' symmetrised search failed (5 / 6, set by it)
                if (census > 0) o.why = 2;
                if (on_rows) {
                    take_path();
                    o.fallback = 0;
                    o.census = 1;
                    o.rows_down = packed;
                } else {
                    o.rows_down = n;
                    o.symmetrised = 0;
                }
                return;
            }
            if (r == 1) {
                take_path();
                o.edges_checked = packed * k;
                o.edges_valid = hv(1, p);
                o.rows_down = packed;
            }
        }
        o.ms_restricted = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        o.ms_search += o.ms_restricted;
        if (r != 1) {
            o.fallback = segs[p].cap > 0 ? 1 : 0;
            const double* d_nodes = reinterpret_cast<const double*>(dev + L.o_nodes) + (size_t)p * L.NS * 3;
            found[p] = wholeTableSearch(d_nodes, (int32_t)n, kbox[p].data(), kbox[p].data() + 3, &bs.area(w), raw[p],
                                        o.edges_checked, o.edges_valid, o.ms_dev, o.ms_search)
                           ? 1
                           : 0;
            o.rows_down += n;
        }
    };
    auto run = [&](int p, size_t w) {
        try {
            solve(p, w);
        } catch (...) {
            err[p] = std::current_exception();
        }
    };
    // The W - 1 planner threads are started before the launch and wait for the results, so
    // their wake-up overlaps the device stages; then the W solvers pull problems in order.
    // go: 1 results in, -1 no results (the launch failed).  A thread spins for at most
    // kSpinUs (a warm batch is ~0.17 ms: the spin keeps the wake-up off the critical path)
    // and then blocks on go_cv, so a slow batch (the cold first plan's warm-up, a hung
    // device) does not keep W - 1 cores busy.
    std::atomic<int> go{0};
    std::atomic<int> next{0};
    std::mutex go_mu;
    std::condition_variable go_cv;
    auto set_go = [&](int v) {
        {
            std::lock_guard<std::mutex> lk(go_mu);
            go.store(v, std::memory_order_release);
        }
        go_cv.notify_all();
    };
    auto drain = [&](size_t w) {
        SolveScratch::get().warmup(k);
        for (int p = next++; p < S; p = next++) run(p, w);
    };
    std::mutex done_mu;
    std::condition_variable done_cv;
    size_t pending = W - 1;
    int devno = 0;
    if (hipGetDevice(&devno) != hipSuccess) devno = 0;
    for (size_t t = 1; t < W; ++t)
        plan_pool().submit([&, devno, t] {
            (void)hipSetDevice(devno);
            constexpr int64_t kSpinUs = 400;
            const auto ts = std::chrono::steady_clock::now();
            int g;
            for (uint32_t i = 0; (g = go.load(std::memory_order_acquire)) == 0; ++i) {
                _mm_pause();
                if ((i & 255) == 255 &&
                    std::chrono::steady_clock::now() - ts > std::chrono::microseconds(kSpinUs)) {
                    std::unique_lock<std::mutex> lk(go_mu);
                    go_cv.wait(lk, [&] { return go.load(std::memory_order_acquire) != 0; });
                }
            }
            if (g > 0) drain(t);
            std::lock_guard<std::mutex> lk(done_mu);
            if (--pending == 0) done_cv.notify_all();
        });
    auto join = [&] {
        std::unique_lock<std::mutex> lk(done_mu);
        done_cv.wait(lk, [&] { return pending == 0; });
    };
    double ms_enqueue = 0;
    try {
        const uint32_t seq = bs.next_seq();
        check(plan_batch_launch(w, canPass ? 1 : 0, lo, hi, L, bs.dev(), H, seq, st), "planner batch");
        ms_enqueue = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_dev0).count();
        // the emit's completion slots (polled: no stream synchronisation), the stream's
        // state every ~1k polls (a failed launch ends the wait)
        static const bool sync_wait = [] {  // (A/B knob: EPP_PB_SYNC=1 synchronises the stream instead)
            const char* e = std::getenv("EPP_PB_SYNC");
            return e && std::atoi(e) == 1;
        }();
        if (sync_wait) check(epp_stream_sync(st), "sync");
        // (a deadline: a batch that has not completed in kBatchDeadlineS raises instead of
        // polling forever; the scratch it writes into stays allocated)
        constexpr double kBatchDeadlineS = 30.0;
        const uint32_t* done = reinterpret_cast<const uint32_t*>(H + L.h_done);
        const auto tw0 = std::chrono::steady_clock::now();
        for (uint64_t spin = 0;; ++spin) {
            int b = 0;
            while (b < L.done_n && __atomic_load_n(done + b, __ATOMIC_ACQUIRE) == seq) ++b;
            if (b == L.done_n) break;
            if ((spin & 1023) == 1023) {
                const hipError_t q = hipStreamQuery(static_cast<hipStream_t>(st));
                if (q == hipErrorNotReady) {
                    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - tw0).count() > kBatchDeadlineS)
                        throw std::runtime_error("planner batch: not complete after 30 s (device hung?)");
                    continue;
                }
                if (q != hipSuccess) throw std::runtime_error(std::string("planner batch: ") + hipGetErrorString(q));
                b = 0;
                while (b < L.done_n && __atomic_load_n(done + b, __ATOMIC_ACQUIRE) == seq) ++b;
                if (b != L.done_n) throw std::runtime_error("planner batch: completed without its completion slots");
                break;
            }
            _mm_pause();
        }
        plan_batch_trace_print();
        for (int p = 0; p < S; ++p) first[p + 1] = first[p] + std::min<int64_t>(hv(0, p), segs[p].cap);
        // Cold areas (this thread's first plans): one whole-table search on problem 0's
        // nodes, so that the fallback's first launches and transfers are paid here, in the
        // cold first plan, rather than by the first search that falls back.
        for (size_t a = 0; a < W; ++a) {
            BatchScratch::Area& ar = bs.area(a);
            if (!ar.cold) continue;
            ar.cold = false;
            std::vector<Vec3> dummy;
            int64_t e0 = 0, e1 = 0;
            double m0 = 0, m1 = 0;
            (void)wholeTableSearch(reinterpret_cast<const double*>(dev + L.o_nodes), (int32_t)hdr[kPbPerSeg + 3 * S],
                                   kbox[0].data(), kbox[0].data() + 3, &ar, dummy, e0, e1, m0, m1);
        }
    } catch (...) {
        set_go(-1);
        join();
        throw;
    }
    const double ms_batch = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_dev0).count();
    set_go(1);
    drain(0);
    join();
    for (const auto& e : err)
        if (e) std::rethrow_exception(e);
    // ---- one batched shortcut for every path found (reduceVertices' role) ---------------
    const auto t_sc = std::chrono::steady_clock::now();
    const double ms_solve = std::chrono::duration<double, std::milli>(t_sc - t_dev0).count() - ms_batch;
    std::vector<std::vector<Vec3>> shortcut_in;
    std::vector<int> which;
    std::vector<GateEnds*> sc_ends;  // (planPathsIncludeGates2: the pruning's pairs too)
    for (int p = 0; p < S; ++p)
        if (found[p]) {
            shortcut_in.push_back(std::move(raw[p]));
            which.push_back(p);
            if (ends) sc_ends.push_back(ends + p);
        }
    std::vector<std::vector<Vec3>> shortcut_out = shortcutAll(shortcut_in, ends ? &sc_ends : nullptr);
    paths.assign(S, {});
    ok.assign(S, 0);
    for (size_t i = 0; i < which.size(); ++i) {
        paths[which[i]] = std::move(shortcut_out[i]);
        ok[which[i]] = 1;
    }
    const double ms_sc = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_sc).count();
    std::lock_guard<std::mutex> lk(g_stats_mu);
    stats_.ms_device += ms_batch;
    stats_.ms_search += ms_sc;
    stats_.ms_batch += ms_batch;
    stats_.ms_enqueue += ms_enqueue;
    stats_.ms_solve += ms_solve;
    stats_.ms_shortcut += ms_sc;
    for (int p = 0; p < S; ++p) {
        const Out& o = res[p];
        stats_.states_sampled += samples;
        stats_.states_valid += o.n - 2;
        stats_.edges_checked += o.edges_checked;
        stats_.edges_valid += o.edges_valid;
        stats_.rows_downloaded += o.rows_down;
        stats_.restricted_rows += o.restricted_rows;
        stats_.fallbacks += o.fallback;
        if (o.fallback && o.why >= 0) ++stats_.fallback_why[o.why];
        stats_.astar_pops += o.pops;
        stats_.restricted_symmetrised += o.symmetrised;
        stats_.symmetrised_after_census += o.census;
        stats_.restricted_nodes += o.nodes;
        if (o.ms_restricted > stats_.ms_restricted_max) {
            stats_.ms_restricted_max = o.ms_restricted;
            stats_.ms_copy_of_max = o.ms_copy;
        }
        stats_.ms_device += o.ms_dev;
        stats_.ms_search += o.ms_search;
    }
}

// The whole k-NN table of one problem's nodes (device, start and goal first): k-NN, motion
// checks straight off the table with the mask folded in (failed motions -> -1; the kept
// edges and those into the goal, node 1, counted), the table down (up to 65535 nodes as
// u16, 0xFFFF: no edge) with the nodes, then A* over the forward edges and, if that does not
// reach the goal, over the symmetrised graph.  Runs on the calling thread's own stream.
bool PathPlanner::wholeTableSearch(const double* d_nodes, int32_t n, const double box_lo[3], const double box_hi[3],
                                   void* area_, std::vector<Vec3>& path, int64_t& edges_checked, int64_t& edges_valid,
                                   double& ms_dev, double& ms_search, const std::function<bool()>* rows_sym,
                                   bool* decided_on_rows, int64_t* census_goal_edges) const {
    const auto t0 = std::chrono::steady_clock::now();
    if (decided_on_rows) *decided_on_rows = false;
    const bool canPass = configParser->getPathPlannerProperties().canPassGate;
    const epp_world* w = worldPtr->device();
    const int k = k_;
    BatchScratch::Area& area = *static_cast<BatchScratch::Area*>(area_);
    void* st = area.stream;
    const size_t m = (size_t)n * k;
    const size_t ws_bytes = (size_t)epp_knn_workspace_size(n);
    if (BatchScratch::area_dev_bytes(n, k) > area.dcap || BatchScratch::area_pin_bytes(n, k) > area.pcap)
        throw std::runtime_error("planPath: fallback workspace too small");
    char* dp = static_cast<char*>(area.dev);
    int64_t* d_ecnt = reinterpret_cast<int64_t*>(dp);
    int32_t* d_nbr = reinterpret_cast<int32_t*>(dp + BatchScratch::r256(16));
    const bool narrow = n <= 65535;
    uint16_t* d_nbr16 = narrow ? reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(d_nbr) + BatchScratch::r256(m * 4))
                               : nullptr;
    uint8_t* d_ev = reinterpret_cast<uint8_t*>(d_nbr) + BatchScratch::r256(m * 4) + BatchScratch::r256(m * 2);
    void* d_ws = d_ev + BatchScratch::r256(m);
    if (hipMemsetAsync(d_ecnt, 0, 16, static_cast<hipStream_t>(st)) != hipSuccess)
        throw std::runtime_error("planPath: clearing the edge counts failed");
    check(epp_knn_ws_box(d_nodes, n, k, 0.0, box_lo, box_hi, d_nbr, d_ws, ws_bytes, st), "knn");
    const epp_status ks = check_knn_motions_masked(w, d_nodes, d_nbr, n, k, canPass ? 1 : 0, d_ev, d_nbr16, 1, d_ecnt, st);
    if (ks == EPP_ERR_UNSUPPORTED) {  // (worlds without tile tables: materialised endpoints)
        ThreadScratch& ts = ThreadScratch::get();
        ts.reset(2 * ThreadScratch::rounded(m * 24));
        double* d_e1 = static_cast<double*>(ts.carve(m * 24));
        double* d_e2 = static_cast<double*>(ts.carve(m * 24));
        check(epp_knn_edges(d_nodes, d_nbr, n, k, d_e1, d_e2, st), "edges");
        check(epp_check_motions(w, d_e1, d_e2, (int64_t)m, canPass ? 1 : 0, 0, d_ev, st), "motion check");
        check(mask_edges_count_acc(d_nbr, d_ev, (int64_t)m, 1, d_ecnt, st, d_nbr16), "mask edges");
    } else {
        check(ks, "motion check");
    }
    // the downloads queued back to back, one synchronisation
    char* hp = static_cast<char*>(area.pin);
    int64_t* ecnt = reinterpret_cast<int64_t*>(hp);
    double overlap_ms = 0;  // (the rows' search, while the device worked: not device time)
    if (rows_sym) {  // the edge counts first, the caller's search on the rows meanwhile: no
                     // kept edge into the goal lets that search decide (its path: the caller's)
        check(epp_memcpy_d2h_async(ecnt, d_ecnt, 16, st), "download");
        const auto tc = std::chrono::steady_clock::now();
        const bool ok = (*rows_sym)();
        const auto tr = std::chrono::steady_clock::now();
        check(epp_stream_sync(st), "sync");
        const auto tw = std::chrono::steady_clock::now();
        overlap_ms = std::chrono::duration<double, std::milli>(tr - tc).count();
        ms_search += overlap_ms;
        if (plan_trace())
            std::cerr << "[plan trace] whole table n " << n << " for its goal-edge count: "
                      << std::chrono::duration<double, std::milli>(tw - t0).count() << " ms (waited "
                      << std::chrono::duration<double, std::milli>(tw - tr).count() << " ms after the rows' search)"
                      << ", kept edges into the goal " << ecnt[1] << std::endl;
        if (census_goal_edges) *census_goal_edges = ecnt[1];
        if (ecnt[1] == 0 && ok) {
            ms_dev += std::chrono::duration<double, std::milli>(tw - t0).count() - overlap_ms;
            edges_checked = (int64_t)m;
            edges_valid = ecnt[0];
            if (decided_on_rows) *decided_on_rows = true;
            return true;
        }
    }
    const double* nodes = reinterpret_cast<const double*>(hp + BatchScratch::r256(64));
    void* h_tab = hp + BatchScratch::r256(64) + BatchScratch::r256((size_t)n * 24);
    check(epp_memcpy_d2h_async(ecnt, d_ecnt, 16, st), "download");
    check(epp_memcpy_d2h_async(const_cast<double*>(nodes), d_nodes, (uint64_t)n * 24, st), "download");
    if (narrow) check(epp_memcpy_d2h_async(h_tab, d_nbr16, m * 2, st), "download");
    else check(epp_memcpy_d2h_async(h_tab, d_nbr, m * 4, st), "download");
    check(epp_stream_sync(st), "sync");
    edges_checked = (int64_t)m;
    edges_valid = ecnt[0];
    const bool goal_has_forward_edge = ecnt[1] > 0;
    const auto t1 = std::chrono::steady_clock::now();
    ms_dev += std::chrono::duration<double, std::milli>(t1 - t0).count() - overlap_ms;
    const int32_t* nbr32 = static_cast<const int32_t*>(h_tab);
    const uint16_t* nbr16 = static_cast<const uint16_t*>(h_tab);
    auto nbr = [&](size_t e) -> int {
        if (!narrow) return nbr32[e];
        const uint16_t x = nbr16[e];
        return x == 0xFFFF ? -1 : (int)x;
    };
    auto pos = [&](int v) { return Vec3(nodes[3 * v], nodes[3 * v + 1], nodes[3 * v + 2]); };
    thread_local SearchState ss;
    // (no forward edge into the goal: the forward pass cannot reach it -- it would only
    // explore start's whole component first; same result, so go straight to the second)
    int r = 0;
    if (goal_has_forward_edge)
        r = astar(ss, (size_t)n, pos, [&](int u, double, auto&& relax, bool closing) {
            if (closing)
                for (int c = 0; c < k; ++c) {
                    const int v = nbr((size_t)u * k + c);
                    if (v >= 0) relax(v);
                }
            return true;
        });
    const bool trace = plan_trace();
    const auto t_fwd = std::chrono::steady_clock::now();
    if (r != 1) {  // the symmetrised graph: the reverse edges as a CSR, built on the device
        // (counting sort of the masked table; every node's sources ascending, the order of a
        // host build scanning the rows in node order) and downloaded with one synchronisation
        char* rp = reinterpret_cast<char*>(d_ws) + BatchScratch::r256((size_t)epp_knn_workspace_size(n));
        int32_t* d_cnt = reinterpret_cast<int32_t*>(rp);
        int32_t* d_fill = reinterpret_cast<int32_t*>(rp + BatchScratch::r256((size_t)(n + 1) * 4));
        int32_t* d_roff = reinterpret_cast<int32_t*>(rp + 2 * BatchScratch::r256((size_t)(n + 1) * 4));
        int32_t* d_radj = reinterpret_cast<int32_t*>(rp + 3 * BatchScratch::r256((size_t)(n + 1) * 4));
        uint16_t* d_radj16 = narrow ? reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(d_radj) + BatchScratch::r256(m * 4))
                                    : nullptr;
        check(reverse_csr(d_nbr, n, k, d_cnt, d_fill, d_roff, d_radj, d_radj16, st), "reverse edges");
        int32_t* roff = reinterpret_cast<int32_t*>(static_cast<char*>(h_tab) + BatchScratch::r256(m * 4));
        void* h_radj = reinterpret_cast<char*>(roff) + BatchScratch::r256((size_t)(n + 1) * 4);
        check(epp_memcpy_d2h_async(roff, d_roff, (uint64_t)(n + 1) * 4, st), "download");
        check(epp_stream_sync(st), "sync");
        const int64_t ne = roff[n];
        if (narrow) check(epp_memcpy_d2h_async(h_radj, d_radj16, (uint64_t)ne * 2, st), "download");
        else check(epp_memcpy_d2h_async(h_radj, d_radj, (uint64_t)ne * 4, st), "download");
        check(epp_stream_sync(st), "sync");
        const uint16_t* radj16 = static_cast<const uint16_t*>(h_radj);
        const int32_t* radj32 = static_cast<const int32_t*>(h_radj);
        auto radj = [&](int64_t q) -> int { return narrow ? (int)radj16[q] : radj32[q]; };
        const auto t_csr = std::chrono::steady_clock::now();
        int64_t pops = 0;
        r = astar(ss, (size_t)n, pos, [&](int u, double, auto&& relax, bool closing) {
            pops += closing ? 1 : 0;
            if (closing) {
                for (int c = 0; c < k; ++c) {
                    const int v = nbr((size_t)u * k + c);
                    if (v >= 0) relax(v);
                }
                for (int32_t q = roff[u]; q < roff[u + 1]; ++q) relax(radj(q));
            }
            return true;
        });
        if (trace) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::cerr << "[plan trace] whole table n " << n << " forward edge into goal " << goal_has_forward_edge
                      << ": device " << ms(t0, t1) << " ms, forward A* " << ms(t1, t_fwd) << " ms, reverse CSR "
                      << ms(t_fwd, t_csr) << " ms, symmetrised A* " << ms(t_csr, std::chrono::steady_clock::now())
                      << " ms (" << pops << " closed), found " << (r == 1) << std::endl;
        }
    }
    path.clear();
    if (r == 1) {
        for (int v = 1; v >= 0; v = ss.prev_of(v)) path.push_back(pos(v));
        std::reverse(path.begin(), path.end());
    }
    ms_search += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    return r == 1;
}

bool PathPlanner::planOnce(const Vec3& start, const Vec3& goal, int64_t samples, uint64_t seed,
                           std::vector<Vec3>& out) const {
    std::vector<std::vector<Vec3>> paths;
    std::vector<char> ok;
    planAttempt({{start, goal}}, {seed}, samples, paths, ok);
    if (ok[0]) out = std::move(paths[0]);
    return ok[0] != 0;
}

// Greedy shortcutting with one batched check of every vertex pair of every path (the role
// of PathSimplifier::reduceVertices in src/PathPlanner.cpp:138-139).
// (pairs (i, j), j >= i + 2, of an L-point list are queued row by row: the index of one)
static size_t pair_index(size_t L, size_t i, size_t j) {
    const size_t before = i * (L - 2) - (i * (i - 1)) / 2;  // pairs of rows < i: sum (L - 2 - r)
    return before + (j - i - 2);
}

std::vector<std::vector<Vec3>> PathPlanner::shortcutAll(const std::vector<std::vector<Vec3>>& ps,
                                                        const std::vector<GateEnds*>* ends) const {
    // ends: each path's list is [prev] + path + [next] (the pruning's points): all its pairs
    // are queued and each ray answers both canPassGate values (World::checkRaysBoth); the
    // shortcut reads the path's pairs, the pruning keeps the true answers of all of them
    const bool canPass = configParser->getPathPlannerProperties().canPassGate;
    std::vector<double> s1, s2;
    std::vector<size_t> base(ps.size() + 1, 0), off(ps.size(), 0);
    for (size_t q = 0; q < ps.size(); ++q) {
        const auto& p = ps[q];
        base[q + 1] = base[q];
        std::vector<Vec3> ext;
        if (ends) {
            GateEnds& g = *(*ends)[q];
            if (g.has_prev) ext.push_back(g.prev);
            off[q] = g.has_prev ? 1 : 0;
            ext.insert(ext.end(), p.begin(), p.end());
            if (g.has_next) ext.push_back(g.next);
        }
        const std::vector<Vec3>& w = ends ? ext : p;
        const size_t L = w.size();
        if (L >= 3)
            for (size_t i = 0; i < L; ++i)
                for (size_t j = i + 2; j < L; ++j) {
                    s1.insert(s1.end(), {w[i].x, w[i].y, w[i].z});
                    s2.insert(s2.end(), {w[j].x, w[j].y, w[j].z});
                    ++base[q + 1];
                }
        if (ends) (*ends)[q]->pts = std::move(ext);
    }
    std::vector<uint8_t> ok(base.back());
    const auto t_rays = std::chrono::steady_clock::now();
    if (!ok.empty()) {
        if (ends) worldPtr->checkRaysBoth(s1.data(), s2.data(), (int64_t)ok.size(), ok.data());
        else worldPtr->checkRays(s1.data(), s2.data(), (int64_t)ok.size(), canPass, ok.data());
    }
    if (pairs_trace())
        std::fprintf(stderr, "pairs_trace: shortcut paths %zu pairs %zu rays%s %.1f us\n", ps.size(), ok.size(),
                     ends ? " (both answers: the pruning's too)" : "",
                     std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_rays).count());
    const uint8_t bit = ends ? (canPass ? 2 : 1) : 0xFF;  // the shortcut's answer in a flag byte
    if (ends)
        for (size_t q = 0; q < ps.size(); ++q) {
            GateEnds& g = *(*ends)[q];
            g.vis.resize(base[q + 1] - base[q]);
            for (size_t t = 0; t < g.vis.size(); ++t) g.vis[t] = (ok[base[q] + t] >> 1) & 1;
            g.filled = true;
        }
    std::vector<std::vector<Vec3>> out(ps.size());
    for (size_t q = 0; q < ps.size(); ++q) {
        const auto& p = ps[q];
        const size_t L = p.size();
        if (L < 3) {
            out[q] = p;
            continue;
        }
        // vis(i, j) of pair (i, j), j >= i + 2, in the order they were queued
        const size_t LE = ends ? (*ends)[q]->pts.size() : L;
        auto vis = [&](size_t i, size_t j) {
            return (ok[base[q] + pair_index(LE, i + off[q], j + off[q])] & bit) != 0;
        };
        std::vector<Vec3> o = {p[0]};
        size_t cur = 0;
        while (cur + 1 < L) {
            size_t nxt = cur + 1;  // a path edge, valid by construction
            for (size_t j = L - 1; j > cur + 1; --j)
                if (vis(cur, j)) {
                    nxt = j;
                    break;
                }
            o.push_back(p[nxt]);
            cur = nxt;
        }
        out[q] = std::move(o);
    }
    return out;
}

std::vector<Vec3> PathPlanner::shortcut(const std::vector<Vec3>& p) const { return shortcutAll({p})[0]; }

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
    std::vector<std::vector<Vec3>> paths;
    std::vector<char> ok;
    const int attempts = planCalls({{start, goal}}, call, timeLimit, paths, ok);
    if (ok[0]) resultPath = std::move(paths[0]);
    {
        std::lock_guard<std::mutex> lk(g_stats_mu);
        stats_.attempts = attempts;
        stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return ok[0] != 0;
}

// Problems with the call numbers base, base + 1, ...: attempt a with samples_fmt x 2^a
// samples and the seed mix(seed(call), a), the problems still without a path batched
// together; up to 4 attempts while inside timeLimit (the role of solve(timeLimit),
// src/PathPlanner.cpp:126-136).  Returns the attempts made.
int PathPlanner::planCalls(const std::vector<std::pair<Vec3, Vec3>>& problems, uint64_t base, double timeLimit,
                           std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                           std::vector<GateEnds>* ends) const {
    const auto t0 = std::chrono::steady_clock::now();
    const auto& pp = configParser->getPathPlannerProperties();
    const size_t n = problems.size();
    paths.assign(n, {});
    ok.assign(n, 0);
    std::vector<uint64_t> seeds(n);
    for (size_t i = 0; i < n; ++i) {
        uint64_t seed = mix(seed_, base + i);
        for (int d = 0; d < 3; ++d) seed = mix(mix(seed, bits_of(problems[i].first[d])), bits_of(problems[i].second[d]));
        seeds[i] = seed;
    }
    std::vector<size_t> pending(n);
    for (size_t i = 0; i < n; ++i) pending[i] = i;
    int64_t samples = pp.samplesFMT > 0 ? pp.samplesFMT : 4096;
    int attempts = 0;
    for (int a = 0; a < 4 && !pending.empty(); ++a) {
        std::vector<std::pair<Vec3, Vec3>> sub;
        std::vector<uint64_t> sseeds;
        for (size_t i : pending) {
            sub.push_back(problems[i]);
            sseeds.push_back(mix(seeds[i], (uint64_t)a));
        }
        std::vector<std::vector<Vec3>> sp;
        std::vector<char> so;
        std::vector<GateEnds> se;
        if (ends)
            for (size_t i : pending) se.push_back((*ends)[i]);
        planAttempt(sub, sseeds, samples, sp, so, ends ? se.data() : nullptr);
        attempts = a + 1;
        std::vector<size_t> still;
        for (size_t j = 0; j < pending.size(); ++j) {
            if (so[j]) {
                paths[pending[j]] = std::move(sp[j]);
                ok[pending[j]] = 1;
                if (ends) (*ends)[pending[j]] = std::move(se[j]);
            } else {
                still.push_back(pending[j]);
            }
        }
        pending.swap(still);
        // (every pending problem ran in each attempt, concurrently with the others, so the
        // batch's elapsed time is each problem's own, as for concurrent planPath calls
        // (src/OnlineTrajGenerator.cpp:324-340); consecutive planPath calls -- the
        // reference's preComputeTraj -- would each restart the clock: a problem that keeps
        // failing here gets at most the attempts timeLimit allows from the batch's start)
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!pending.empty() && el > timeLimit) break;  // out of time: give up like solve(timeLimit)
        samples *= 2;
    }
    return attempts;
}

void PathPlanner::planPaths(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                            std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok) const {
    planPathsWith(problems, timeLimit, paths, ok, nullptr);
}

bool PathPlanner::planPathsIncludeGates2(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                                         std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                                         std::vector<Vec3>& pruned) const {
    // (EPP_FUSED_PRUNE=0: the two calls as they are, for A/B)
    static const bool fused = [] {
        const char* e = std::getenv("EPP_FUSED_PRUNE");
        return !(e && std::string(e) == "0");
    }();
    std::vector<GateEnds> ends;
    if (fused && configParser->getPathPlannerProperties().pathSimplification == "custom") {
        ends.resize(problems.size());
        for (size_t s = 0; s + 1 < problems.size(); ++s) {  // includeGates2's (a + b) / 2 of the ends
            const Vec3 c = (problems[s].second + problems[s + 1].first) / 2;
            ends[s].has_next = ends[s + 1].has_prev = true;
            ends[s].next = ends[s + 1].prev = c;
        }
    }
    planPathsWith(problems, timeLimit, paths, ok, ends.empty() ? nullptr : &ends);
    for (char o : ok)
        if (!o) return false;
    pruned = includeGates2With(paths, ends.empty() ? nullptr : &ends);
    return true;
}

void PathPlanner::planPathsWith(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                                std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                                std::vector<GateEnds>* ends) const {
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
    (void)worldPtr->device();  // the device world, before the planner threads share it
    const uint64_t base = __atomic_fetch_add(&calls_, (uint64_t)n, __ATOMIC_RELAXED);
    const int attempts = planCalls(problems, base, timeLimit, paths, ok, ends);
    std::lock_guard<std::mutex> lk(g_stats_mu);
    stats_.attempts = attempts;
    stats_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// PathPlanner::includeGates2 — src/PathPlanner.cpp:175-230.  The segments' pruning checks
// are one batch (pruneAll).
std::vector<Vec3> PathPlanner::includeGates2(std::vector<std::vector<Vec3>> waypoints) const {
    return includeGates2With(std::move(waypoints), nullptr);
}

std::vector<Vec3> PathPlanner::includeGates2With(std::vector<std::vector<Vec3>> waypoints,
                                                 const std::vector<GateEnds>* ends) const {
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
    std::vector<std::vector<Vec3>> pruned;
    if (method == "none") {
        pruned = waypoints;
    } else if (method == "custom") {
        pruned = pruneAll(waypoints, ends);
    } else if (method == "ompl") {
        pruned = smoothAll(waypoints);
    } else {
        std::cerr << "Unknown pruning method" << std::endl;
        throw std::runtime_error("Unknown pruning method");
    }
    std::vector<Vec3> flat;
    for (const auto& seg : pruned)
        for (const auto& w : seg) {
            if (!flat.empty() && (flat.back() - w).norm() < 0.05) continue;  // :222
            flat.push_back(w);
        }
    return flat;
}

// PathPlanner::omplPrunePathAndInterpolate — src/PathPlanner.cpp:282-313: OMPL's
// PathSimplifier::smoothBSpline(path) with its defaults (maxSteps = 5, minChange = double
// epsilon), as OMPL 1.6 publishes it (PathSimplifier.cpp, PathGeometric::subdivide,
// RealVectorStateSpace::interpolate / distance).  Per step every live path is subdivided
// (a midpoint between every two states); then each even state i (2 <= i < n - 1) moves to
// the midpoint of the midpoints (i-1, i) and (i, i+1) when state i-1 is valid, both
// motions (i-1 -> new, new -> i+1) are valid and the move exceeds minChange.  The moves of
// one step touch only even states and read only odd ones, so they are independent: the
// step's state checks (all paths) are one batch, its motion checks another, on the
// planner's validators (src/PathPlanner.cpp:47-50: can_pass_gate from the config).  A path
// whose step moves nothing stops (OMPL's break); paths of < 3 states are returned as they
// are.
std::vector<std::vector<Vec3>> PathPlanner::smoothAll(const std::vector<std::vector<Vec3>>& segs) const {
    const bool canPass = configParser->getPathPlannerProperties().canPassGate;
    constexpr int kMaxSteps = 5;
    const double minChange = std::numeric_limits<double>::epsilon();
    auto half = [](const Vec3& a, const Vec3& b) {  // interpolate(a, b, 0.5): a + (b - a) * t
        return Vec3(a.x + (b.x - a.x) * 0.5, a.y + (b.y - a.y) * 0.5, a.z + (b.z - a.z) * 0.5);
    };
    auto distance = [](const Vec3& a, const Vec3& b) {  // left-to-right sum of squares
        double t = 0.0;
        for (int d = 0; d < 3; ++d) {
            const double diff = a[d] - b[d];
            t += diff * diff;
        }
        return std::sqrt(t);
    };
    std::vector<std::vector<Vec3>> st = segs;
    std::vector<char> live(st.size());
    for (size_t q = 0; q < st.size(); ++q) live[q] = st[q].size() >= 3;
    std::vector<double> pts, r1, r2;
    std::vector<Vec3> cand;
    std::vector<std::pair<uint32_t, uint32_t>> at;  // (path, state i) of each candidate move
    std::vector<uint8_t> okp, okr;
    for (int step = 0; step < kMaxSteps; ++step) {
        pts.clear();
        r1.clear();
        r2.clear();
        cand.clear();
        at.clear();
        for (size_t q = 0; q < st.size(); ++q) {
            if (!live[q]) continue;
            std::vector<Vec3>& s = st[q];
            std::vector<Vec3> sub;  // PathGeometric::subdivide
            sub.reserve(2 * s.size() - 1);
            sub.push_back(s[0]);
            for (size_t i = 1; i < s.size(); ++i) {
                const Vec3 m = half(sub.back(), s[i]);
                sub.push_back(m);
                sub.push_back(s[i]);
            }
            s.swap(sub);
            for (size_t i = 2; i + 1 < s.size(); i += 2) {
                Vec3 t1 = half(s[i - 1], s[i]);
                const Vec3 t2 = half(s[i], s[i + 1]);
                t1 = half(t1, t2);
                pts.insert(pts.end(), {s[i - 1].x, s[i - 1].y, s[i - 1].z});
                r1.insert(r1.end(), {s[i - 1].x, s[i - 1].y, s[i - 1].z, t1.x, t1.y, t1.z});
                r2.insert(r2.end(), {t1.x, t1.y, t1.z, s[i + 1].x, s[i + 1].y, s[i + 1].z});
                cand.push_back(t1);
                at.emplace_back((uint32_t)q, (uint32_t)i);
            }
        }
        if (cand.empty()) break;
        const int64_t n = (int64_t)cand.size();
        okp.assign((size_t)n, 0);
        okr.assign((size_t)(2 * n), 0);
        worldPtr->checkPoints(pts.data(), n, canPass, okp.data());
        worldPtr->checkRays(r1.data(), r2.data(), 2 * n, canPass, okr.data());
        std::vector<int> moved(st.size(), 0);
        for (int64_t j = 0; j < n; ++j) {
            if (!okp[j] || !okr[2 * j] || !okr[2 * j + 1]) continue;
            Vec3& si = st[at[j].first][at[j].second];
            if (distance(si, cand[j]) > minChange) {
                si = cand[j];
                ++moved[at[j].first];
            }
        }
        bool any = false;
        for (size_t q = 0; q < st.size(); ++q) {
            if (live[q] && moved[q] == 0) live[q] = 0;  // OMPL: a step that moved nothing ends the loop
            any = any || live[q];
        }
        if (!any) break;
    }
    return st;
}

// PathPlanner::pruneWaypoints — src/PathPlanner.cpp:232-265.  The reference checks
// ray(reference, current) one at a time; every pair it could ask for is checked in one
// batch (for all segments at once) and the same greedy walk is replayed on the answers.
std::vector<std::vector<Vec3>> PathPlanner::pruneAll(const std::vector<std::vector<Vec3>>& segs,
                                                     const std::vector<GateEnds>* ends) const {
    // ends (planPathsIncludeGates2): a segment whose points are, in order, among its
    // GateEnds' pts (bit for bit) reads the answers the shortcut's batch already holds
    auto same = [](const Vec3& a, const Vec3& b) { return std::memcmp(&a, &b, sizeof(Vec3)) == 0; };
    std::vector<std::vector<size_t>> at(segs.size());  // segment point -> its index in pts
    for (size_t q = 0; ends && q < segs.size() && q < ends->size(); ++q) {
        const GateEnds& g = (*ends)[q];
        if (!g.filled || segs[q].size() < 3) continue;
        std::vector<size_t> m;
        size_t k = 0;
        for (const Vec3& v : segs[q]) {
            while (k < g.pts.size() && !same(g.pts[k], v)) ++k;
            if (k == g.pts.size()) break;
            m.push_back(k++);
        }
        if (m.size() == segs[q].size()) at[q] = std::move(m);
    }
    std::vector<double> s1, s2;
    std::vector<size_t> base(segs.size() + 1, 0);
    size_t answered = 0;
    for (size_t q = 0; q < segs.size(); ++q) {
        const auto& w = segs[q];
        const size_t L = w.size();
        base[q + 1] = base[q];
        if (L < 3) continue;
        if (!at[q].empty()) {
            ++answered;
            continue;
        }
        for (size_t i = 0; i < L; ++i)
            for (size_t j = i + 2; j < L; ++j) {
                s1.insert(s1.end(), {w[i].x, w[i].y, w[i].z});
                s2.insert(s2.end(), {w[j].x, w[j].y, w[j].z});
                ++base[q + 1];
            }
    }
    std::vector<uint8_t> ok(base.back());
    const auto t_rays = std::chrono::steady_clock::now();
    if (!ok.empty()) worldPtr->checkRays(s1.data(), s2.data(), (int64_t)ok.size(), true, ok.data());  // canPassGate = true
    if (pairs_trace())
        std::fprintf(stderr, "pairs_trace: prune segments %zu (%zu answered by the shortcut's batch) pairs %zu rays %.1f us\n",
                     segs.size(), answered, ok.size(),
                     std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_rays).count());
    std::vector<std::vector<Vec3>> out(segs.size());
    for (size_t q = 0; q < segs.size(); ++q) {
        const auto& w = segs[q];
        const size_t L = w.size();
        if (L < 3) {
            out[q] = w;
            continue;
        }
        auto vis = [&](size_t i, size_t j) {  // pair (i, j), j >= i + 2, in the order queued
            if (!at[q].empty()) {
                const GateEnds& g = (*ends)[q];
                return g.vis[pair_index(g.pts.size(), at[q][i], at[q][j])] != 0;
            }
            return ok[base[q] + pair_index(L, i, j)] != 0;
        };
        std::vector<Vec3> pruned = {w[0]};
        size_t ref = 0;
        for (size_t cur = 2; cur < L; ++cur) {
            if (!vis(ref, cur)) {
                pruned.push_back(w[cur - 1]);
                ref = cur - 1;
            }
        }
        pruned.push_back(w[L - 1]);
        out[q] = std::move(pruned);
    }
    return out;
}

std::vector<Vec3> PathPlanner::pruneWaypoints(const std::vector<Vec3>& w) const { return pruneAll({w})[0]; }

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

// host_world.cpp — epp::World, the drop-in for the reference's World
// (src/World.cpp:13-162) over the device index of include/epp.h.
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "epp/World.h"
#include "host_scratch.h"
#include "small_sync.h"

namespace epp {

namespace {
std::vector<epp_obb_desc> descs_of(const std::vector<OBBDescription>& in) {
    std::vector<epp_obb_desc> out(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        std::memset(&out[i], 0, sizeof(epp_obb_desc));
        for (int k = 0; k < 3; ++k) {
            out[i].pos[k] = in[i].center[k];
            out[i].size[k] = in[i].halfSize[k] * 2;  // exact; epp_build_obbs halves it again
        }
        out[i].filling = in[i].type == "filling" ? 1 : 0;
    }
    return out;
}
}  // namespace

World::World(std::shared_ptr<ConfigParser> configParser) : config_(std::move(configParser)) {
    const auto& wp = config_->getWorldProperties();
    rGate_ = wp.inflateRadius.at("gate");      // include/World.h:22-23
    rObst_ = wp.inflateRadius.at("obstacle");
}

World::~World() {
    if (dev_) epp_world_destroy(dev_);
}

void World::resetWorld() {
    std::lock_guard<std::mutex> lk(mu_);
    entries_.clear();
    dirty_ = true;
}

void World::addObject(int id, bool gate, const std::vector<double>& c, bool update) {
    std::vector<epp_obb_desc> gd, od;
    std::vector<int32_t> off = {0, 0};
    std::vector<double> row;
    int type = -1;
    if (gate) {
        if (c.size() >= 7) {
            type = (int)c[6];  // World.cpp:18
        } else if (update && c.size() == 6) {  // a pose only: the gate keeps its type
            std::lock_guard<std::mutex> lk(mu_);
            for (const auto& e : entries_)
                if (e.gate && e.id == id) type = e.type;
        }
        if (type < 0) throw std::invalid_argument("gate coordinates need 7 values");
        gd = descs_of(config_->getGateGeometryByTypeId(type));
        off[1] = (int32_t)gd.size();
        row.assign(c.begin(), c.begin() + 6);
        row.push_back(0);  // descriptors passed as type 0
    } else {
        if (c.size() < 6) throw std::invalid_argument("obstacle coordinates need 6 values");
        od = descs_of(config_->getObstacleGeometry());
        row.assign(c.begin(), c.begin() + 6);
    }
    const size_t cap = gate ? gd.size() : od.size();
    std::vector<epp_obb> out(std::max<size_t>(cap, 1));
    int32_t n = 0;
    check(epp_build_obbs(gd.data(), off.data(), gate ? 1 : 0, od.data(), (int32_t)od.size(),
                         gate ? row.data() : nullptr, gate ? 1 : 0, gate ? nullptr : row.data(),
                         gate ? 0 : 1, out.data(), (int32_t)out.size(), &n),
          "World::addObject");
    out.resize(n);
    std::lock_guard<std::mutex> lk(mu_);
    if (update) {  // removeObject + addObject (World.cpp:20-27)
        for (auto& e : entries_)
            if (e.gate == gate && e.id == id) {
                e.obbs = out;
                e.type = type;
                dirty_ = true;
                return;
            }
    }
    entries_.push_back({id, gate, type, out});
    dirty_ = true;
}

void World::addGate(int gateId, const std::vector<double>& coordinates) {
    addObject(gateId, true, coordinates, false);
}
void World::updateGatePosition(int gateId, const std::vector<double>& coordinates) {
    addObject(gateId, true, coordinates, true);
}
void World::addObstacle(int obstacleId, const std::vector<double>& coordinates) {
    addObject(obstacleId, false, coordinates, false);
}

void World::sync() const {
    // caller holds mu_
    if (!dirty_) return;
    obbs_.clear();
    for (const auto& e : entries_) obbs_.insert(obbs_.end(), e.obbs.begin(), e.obbs.end());
    if (!dev_) {
        check(epp_world_create(obbs_.data(), (int32_t)obbs_.size(), rGate_, rObst_, &dev_), "World upload");
    } else {
        check(epp_world_update(dev_, obbs_.data(), (int32_t)obbs_.size()), "World upload");
    }
    dirty_ = false;
}

const epp_world* World::device() const {
    std::lock_guard<std::mutex> lk(mu_);
    sync();
    return dev_;
}

// Host-array queries.  Small batches (the reference's one-at-a-time validator calls,
// checkTrajectoryValidity's few hundred rows) run zero-copy: the kernel reads the query
// from and writes the flags to pinned host memory, so a call is one launch and one
// stream synchronisation.  Large batches are staged through HBM by DMA.
namespace {
constexpr int64_t kZeroCopyMax = 16384;  // queries per call read straight from host memory
}

// (the small-query lambdas run the synchronous brute-force path of small.hip when the
// query qualifies and report whether they did)
void World::checkPoints(const double* xyz, int64_t n, bool canPassGate, uint8_t* out) const {
    query(n, 1, [&](const double* const* in, uint8_t* flags, void* st) {
        check(epp_check_states(device(), in[0], n, canPassGate ? 1 : 0, flags, nullptr, nullptr, st), "checkPoints");
    }, [&](const double* const* in, uint8_t* flags, void* st) {
        bool handled = false;
        check(states_small_sync(device(), false, in[0], n, canPassGate ? 1 : 0, 0.0, flags, (hipStream_t)st, &handled),
              "checkPoints");
        return handled;
    }, &xyz, out);
}

void World::checkPointsMinDistance(const double* xyz, int64_t n, double minDistance, uint8_t* out) const {
    query(n, 1, [&](const double* const* in, uint8_t* flags, void* st) {
        check(epp_check_states_mindist(device(), in[0], n, minDistance, flags, st), "checkPointsMinDistance");
    }, [&](const double* const* in, uint8_t* flags, void* st) {
        bool handled = false;
        check(states_small_sync(device(), true, in[0], n, 0, minDistance, flags, (hipStream_t)st, &handled),
              "checkPointsMinDistance");
        return handled;
    }, &xyz, out);
}

void World::checkRays(const double* s1, const double* s2, int64_t n, bool canPassGate, uint8_t* out,
                      int mode) const {
    const double* in[2] = {s1, s2};
    query(n, 2, [&](const double* const* d, uint8_t* flags, void* st) {
        check(epp_check_motions(device(), d[0], d[1], n, canPassGate ? 1 : 0, mode, flags, st), "checkRays");
    }, [&](const double* const* d, uint8_t* flags, void* st) {
        bool handled = false;
        check(motions_small_sync(device(), mode, d[0], d[1], n, canPassGate ? 1 : 0, flags, (hipStream_t)st, &handled),
              "checkRays");
        return handled;
    }, in, out);
}

void World::checkRaysBoth(const double* s1, const double* s2, int64_t n, uint8_t* out) const {
    const double* in[2] = {s1, s2};
    bool two = false;  // (past the small path: two launches, below)
    query(n, 2, [&](const double* const*, uint8_t*, void*) { two = true; },
          [&](const double* const* d, uint8_t* flags, void* st) {
              bool handled = false;
              check(motions_small_sync(device(), 0, d[0], d[1], n, kCanPassBoth, flags, (hipStream_t)st, &handled),
                    "checkRays");
              return handled;
          },
          in, out);
    if (!two) return;
    std::vector<uint8_t> t((size_t)n);
    checkRays(s1, s2, n, false, out);
    checkRays(s1, s2, n, true, t.data());
    for (int64_t i = 0; i < n; ++i) out[i] = (uint8_t)((out[i] ? 1 : 0) | (t[i] ? 2 : 0));
}

template <typename Launch, typename Small>
void World::query(int64_t n, int n_in, Launch&& launch, Small&& small, const double* const* in, uint8_t* out) const {
    if (n <= 0) return;
    (void)device();  // upload a changed world before the launch (not inside it)
    ThreadScratch& ts = ThreadScratch::get();
    void* st = ts.stream();
    const size_t in_b = (size_t)n * 24;
    const double* d_in[2] = {nullptr, nullptr};
    if (n <= kZeroCopyMax) {
        char* h = static_cast<char*>(ts.pinned(0, n_in * ThreadScratch::rounded(in_b) + ThreadScratch::rounded((size_t)n)));
        for (int k = 0; k < n_in; ++k) {
            std::memcpy(h + k * ThreadScratch::rounded(in_b), in[k], in_b);
            d_in[k] = reinterpret_cast<const double*>(h + k * ThreadScratch::rounded(in_b));
        }
        uint8_t* flags = reinterpret_cast<uint8_t*>(h + n_in * ThreadScratch::rounded(in_b));
        if (!small(d_in, flags, st)) {
            launch(d_in, flags, st);
            check(epp_stream_sync(st), "query");
        }
        std::memcpy(out, flags, (size_t)n);
        return;
    }
    ts.reset(n_in * ThreadScratch::rounded(in_b) + ThreadScratch::rounded((size_t)n));
    for (int k = 0; k < n_in; ++k) {
        double* d = static_cast<double*>(ts.carve(in_b));
        check(epp_memcpy_h2d(d, in[k], (uint64_t)in_b, st), "upload");
        d_in[k] = d;
    }
    uint8_t* d_out = static_cast<uint8_t*>(ts.carve((size_t)n));
    launch(d_in, d_out, st);
    check(epp_memcpy_d2h(out, d_out, (uint64_t)n, st), "download");
}

bool World::checkPointValidity(const Vec3& p, bool canPassGate) const {
    const double xyz[3] = {p.x, p.y, p.z};
    uint8_t v = 0;
    checkPoints(xyz, 1, canPassGate, &v);
    return v != 0;
}

bool World::checkPointValidityMinDistance(const Vec3& p, double minDistance) const {
    const double xyz[3] = {p.x, p.y, p.z};
    uint8_t v = 0;
    checkPointsMinDistance(xyz, 1, minDistance, &v);
    return v != 0;
}

bool World::checkRayValid(const Vec3& s, const Vec3& e, bool canPassGate) const {
    const double a[3] = {s.x, s.y, s.z}, b[3] = {e.x, e.y, e.z};
    uint8_t v = 0;
    checkRays(a, b, 1, canPassGate, &v);
    return v != 0;
}

}  // namespace epp

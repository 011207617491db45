// host_world.cpp — epp::World, the drop-in for the reference's World
// (src/World.cpp:13-162) over the device index of include/epp.h.
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "epp/World.h"
#include "host_scratch.h"

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
    if (gate) {
        if (c.size() < 7) throw std::invalid_argument("gate coordinates need 7 values");
        const int type = (int)c[6];  // World.cpp:18
        gd = descs_of(config_->getGateGeometryByTypeId(type));
        off[1] = (int32_t)gd.size();
        row.assign(c.begin(), c.begin() + 7);
        row[6] = 0;  // descriptors passed as type 0
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
                dirty_ = true;
                return;
            }
    }
    entries_.push_back({id, gate, out});
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

void World::checkPoints(const double* xyz, int64_t n, bool canPassGate, uint8_t* out) const {
    if (n <= 0) return;
    const epp_world* w = device();
    ThreadScratch& ts = ThreadScratch::get();
    void* st = ts.stream();
    ts.reset(ThreadScratch::rounded((size_t)n * 24) + ThreadScratch::rounded((size_t)n));
    double* d_xyz = static_cast<double*>(ts.carve((size_t)n * 24));
    uint8_t* d_out = static_cast<uint8_t*>(ts.carve((size_t)n));
    check(epp_memcpy_h2d(d_xyz, xyz, (uint64_t)n * 24, st), "upload");
    check(epp_check_states(w, d_xyz, n, canPassGate ? 1 : 0, d_out, nullptr, nullptr, st), "checkPoints");
    check(epp_memcpy_d2h(out, d_out, (uint64_t)n, st), "download");
}

void World::checkPointsMinDistance(const double* xyz, int64_t n, double minDistance, uint8_t* out) const {
    if (n <= 0) return;
    const epp_world* w = device();
    ThreadScratch& ts = ThreadScratch::get();
    void* st = ts.stream();
    ts.reset(ThreadScratch::rounded((size_t)n * 24) + ThreadScratch::rounded((size_t)n));
    double* d_xyz = static_cast<double*>(ts.carve((size_t)n * 24));
    uint8_t* d_out = static_cast<uint8_t*>(ts.carve((size_t)n));
    check(epp_memcpy_h2d(d_xyz, xyz, (uint64_t)n * 24, st), "upload");
    check(epp_check_states_mindist(w, d_xyz, n, minDistance, d_out, st), "checkPointsMinDistance");
    check(epp_memcpy_d2h(out, d_out, (uint64_t)n, st), "download");
}

void World::checkRays(const double* s1, const double* s2, int64_t n, bool canPassGate, uint8_t* out,
                      int mode) const {
    if (n <= 0) return;
    const epp_world* w = device();
    ThreadScratch& ts = ThreadScratch::get();
    void* st = ts.stream();
    ts.reset(2 * ThreadScratch::rounded((size_t)n * 24) + ThreadScratch::rounded((size_t)n));
    double* d1 = static_cast<double*>(ts.carve((size_t)n * 24));
    double* d2 = static_cast<double*>(ts.carve((size_t)n * 24));
    uint8_t* d_out = static_cast<uint8_t*>(ts.carve((size_t)n));
    check(epp_memcpy_h2d(d1, s1, (uint64_t)n * 24, st), "upload");
    check(epp_memcpy_h2d(d2, s2, (uint64_t)n * 24, st), "upload");
    check(epp_check_motions(w, d1, d2, n, canPassGate ? 1 : 0, mode, d_out, st), "checkRays");
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

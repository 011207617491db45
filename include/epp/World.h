// epp/World.h — drop-in for the reference's World (include/World.h:20-92,
// src/World.cpp:13-162).  The OBB table and its AABB index live in HBM (epp_world,
// include/epp.h); every query runs on the GPU.  Single-point queries keep the
// reference's signatures for API compatibility; planners should use the batched forms.
//
// Thread safety: queries are const and may run concurrently from several host
// threads (each call uses its own stream); mutations (addGate, updateGatePosition,
// addObstacle, resetWorld) must not overlap queries (the reference has the same
// requirement).
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

#include "epp.h"
#include "epp/ConfigParser.h"
#include "epp/types.h"

namespace epp {

class World {
public:
    explicit World(std::shared_ptr<ConfigParser> configParser);
    ~World();
    World(const World&) = delete;
    World& operator=(const World&) = delete;

    void resetWorld();
    // coordinates: (x, y, z, roll, pitch, yaw, type); z is forced to 0 (World.cpp:16)
    void addGate(int gateId, const std::vector<double>& coordinates);
    // coordinates: (x, y, z, roll, pitch, yaw, type), or the 6-value pose alone (the gate
    // keeps its type; the reference reads coordinates(6), src/World.cpp:18)
    void updateGatePosition(int gateId, const std::vector<double>& coordinates);
    // coordinates: (x, y, z, roll, pitch, yaw)
    void addObstacle(int obstacleId, const std::vector<double>& coordinates);

    // World::checkPointValidity(p, canPassGate) — src/World.cpp:80-104
    bool checkPointValidity(const Vec3& point, bool canPassGate) const;
    // World::checkPointValidity(p, minDistance) — src/World.cpp:106-128
    bool checkPointValidityMinDistance(const Vec3& point, double minDistance) const;
    // World::checkRayValid — src/World.cpp:130-162
    bool checkRayValid(const Vec3& start, const Vec3& end, bool canPassGate = false) const;

    // Batched host-array forms (one GPU launch each); out[i] = 1 if valid.
    void checkPoints(const double* xyz, int64_t n, bool canPassGate, uint8_t* out) const;
    void checkPointsMinDistance(const double* xyz, int64_t n, double minDistance, uint8_t* out) const;
    void checkRays(const double* s1, const double* s2, int64_t n, bool canPassGate, uint8_t* out,
                   int mode = 0) const;
    // Both answers of checkRayValid per ray (an addition of this build): out[i] bit 0 = valid
    // with canPassGate = false, bit 1 = valid with true.  One launch when the batch takes the
    // small path (k_motions_small tests each ray once for both), else two.
    void checkRaysBoth(const double* s1, const double* s2, int64_t n, uint8_t* out) const;

    // Device handle (rebuilt lazily after mutations); nullptr for an empty world.
    const epp_world* device() const;
    const std::vector<epp_obb>& obbs() const { return obbs_; }
    double inflateGate() const { return rGate_; }
    double inflateObstacle() const { return rObst_; }

private:
    struct Entry {
        int id;
        bool gate;
        int type;  // gate type (-1 for obstacles)
        std::vector<epp_obb> obbs;
    };
    void addObject(int id, bool gate, const std::vector<double>& coordinates, bool update);
    void sync() const;
    template <typename Launch, typename Small>
    void query(int64_t n, int n_in, Launch&& launch, Small&& small, const double* const* in, uint8_t* out) const;

    std::shared_ptr<ConfigParser> config_;
    double rGate_, rObst_;
    std::vector<Entry> entries_;        // insertion order
    mutable std::vector<epp_obb> obbs_;  // flattened, rebuilt on sync
    mutable epp_world* dev_ = nullptr;
    mutable bool dirty_ = true;
    mutable std::mutex mu_;
};

}  // namespace epp

// epp/OnlineTrajGenerator.h — drop-in for the reference's OnlineTrajGenerator
// (include/OnlineTrajGenerator.h:26-77, src/OnlineTrajGenerator.cpp).
//
// Concurrency: the reference recomputes on a detached std::thread and writes the
// trajectory while Python may read it, and rebuilds the World under the planning threads
// (SURVEY.md §5).  Here every access to the planned trajectory goes through one mutex;
// with recalculate_online the recomputation runs on a worker thread.  An update arriving
// while it runs keeps the reference's return values: the gate is recorded, the current
// trajectory is checked against a snapshot world holding the new pose (the worker's
// world is not touched; the rebuild is applied once the worker finished), false is
// returned when it is still valid and the reference's "Call to update trajectory, while
// previous update is still going on" is thrown only when a new recomputation is needed
// (src/OnlineTrajGenerator.cpp:203-212).  The destructor and wait_for_update() wait for
// the worker.
#pragma once
#include <atomic>
#include <cstdint>
#include <future>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "epp/ConfigParser.h"
#include "epp/PathPlanner.h"
#include "epp/PathWriter.h"
#include "epp/types.h"

namespace epp {

class OnlineTrajGenerator {
public:
    OnlineTrajGenerator(const Vec3& start, const Vec3& goal, const Matrix& nominalGatePositionAndType,
                        const Matrix& nominalObstaclePosition, const std::string& configPath);
    OnlineTrajGenerator(const Vec3& start, const Vec3& goal, const Matrix& nominalGatePositionAndType,
                        const Matrix& nominalObstaclePosition, std::shared_ptr<ConfigParser> config);
    ~OnlineTrajGenerator();

    void preComputeTraj(double takeoffTime);
    bool updateGatePos(int gateId, const std::vector<double>& newPose, const Vec3& dronePos,
                       bool nextGateWithinRange, double flightTime);
    std::vector<double> sampleTraj(double currentTime) const;
    double getTrajEndTime() const;
    Matrix getPlannedTraj() const;

    const std::vector<Vec3>& getCheckpoints() const { return checkpoints; }
    // waypoints of the last (re)planned trajectory, after includeGates2
    std::vector<Vec3> getWaypoints() const;
    PathPlanner& planner() { return pathPlanner; }
    // waits for an in-flight online recomputation (recalculate_online); rethrows its
    // failure as std::runtime_error("previous trajectory update failed: ...")
    void waitForUpdate();
    // Which exit the recomputations took so far (an addition of this build, for callers
    // that time or log them): `planned` ran the two segment plans, includeGates2 and the
    // refit; `skippedInvalidStart` took the reference's "Advanced trajectory does not end
    // at valid position" exit (updateGatePos still returned true,
    // src/OnlineTrajGenerator.cpp:304-310); `failed` threw.  updateGatePos calls that
    // returned false never recompute.
    struct RecomputeCounts {
        uint64_t planned = 0, skippedInvalidStart = 0, failed = 0;
    };
    RecomputeCounts recomputeCounts() const {
        return {nPlanned.load(), nSkipped.load(), nFailed.load()};
    }

private:
    void init(const Vec3& start, const Vec3& goal);
    bool getGateCenterAndNormal(const std::vector<double>& gate, Vec3& center, Vec3& normal) const;
    bool checkGatePassed(const Vec3& p1, const Vec3& p2, int gateId) const;
    void recomputeTraj(int gateId, const Vec3& dronePos, double flightTime);
    void collectUpdate();
    void applyDeferredGates();
    Matrix generate(const std::vector<Vec3>& path, double t0, const Vec3& v0, const Vec3& a0,
                    const std::vector<Vec3>& pre = {}) const;
    static size_t nearestRow(const Matrix& traj, double t);
    std::vector<double> gateRow(int gateId) const;

    std::shared_ptr<ConfigParser> configParser;
    PathPlanner pathPlanner;
    Matrix nominalGatePositionAndType;
    Matrix nominalObstaclePosition;
    std::vector<Vec3> checkpoints;
    std::set<int> gatesObservedWithinRange;
    std::vector<std::vector<Vec3>> pathSegments;
    std::vector<int> deferredGates;  // gate updates received while the worker ran (world rebuild pending)
    mutable std::mutex cpMu;         // checkpoints: written by the worker, read by updateGatePos
    Matrix plannedTraj;
    std::vector<Vec3> waypoints;  // guarded by trajMu
    mutable std::mutex trajMu;
    std::atomic<bool> trajectoryCurrentlyUpdating{false};
    std::atomic<uint64_t> nPlanned{0}, nSkipped{0}, nFailed{0};
    std::future<void> pending;
    PathWriter pathWriter{"path_segments"};  // include/OnlineTrajGenerator.h:132
};

}  // namespace epp

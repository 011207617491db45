#include <algorithm>
#include <cstdlib>
#include <thread>
// host_online.cpp — epp::OnlineTrajGenerator, the drop-in for the reference's
// OnlineTrajGenerator (src/OnlineTrajGenerator.cpp).  Each function cites the lines it
// follows; planning and the min-snap refit run on the GPU (PathPlanner,
// poly_traj::generateTrajectory).
#include <chrono>
#include <cstdio>
#include <cmath>
#include <iostream>
#include <limits>
#include <stdexcept>

#include "epp/OnlineTrajGenerator.h"
#include "epp/OptimalTimeParametrizer.h"
#include "epp/TrajInterpolation.h"
#include "epp/trajectory_generator.h"

namespace epp {

OnlineTrajGenerator::OnlineTrajGenerator(const Vec3& start, const Vec3& goal, const Matrix& gates,
                                         const Matrix& obstacles, const std::string& configPath)
    : OnlineTrajGenerator(start, goal, gates, obstacles, std::make_shared<ConfigParser>(configPath)) {}

OnlineTrajGenerator::OnlineTrajGenerator(const Vec3& start, const Vec3& goal, const Matrix& gates,
                                         const Matrix& obstacles, std::shared_ptr<ConfigParser> config)
    : configParser(std::move(config)),
      pathPlanner(gates, obstacles, configParser),
      nominalGatePositionAndType(gates),
      nominalObstaclePosition(obstacles) {
    init(start, goal);
}

OnlineTrajGenerator::~OnlineTrajGenerator() {
    try {
        waitForUpdate();
    } catch (...) {
    }
}

void OnlineTrajGenerator::waitForUpdate() {
    if (pending.valid()) pending.wait();
    collectUpdate();
}

// Takes the finished online recomputation's result; its failure (e.g. "Pre path not
// found. Exiting") is reported here, named as the previous update's.  Gate updates that
// arrived meanwhile are applied to the world now.
void OnlineTrajGenerator::collectUpdate() {
    if (!pending.valid()) return;
    std::exception_ptr failure;
    try {
        pending.get();
    } catch (const std::exception& e) {
        failure = std::make_exception_ptr(std::runtime_error(std::string("previous trajectory update failed: ") + e.what()));
    }
    applyDeferredGates();
    if (failure) std::rethrow_exception(failure);
}

// src/OnlineTrajGenerator.cpp:146-147 for the updates received while the worker planned
void OnlineTrajGenerator::applyDeferredGates() {
    if (deferredGates.empty()) return;
    pathPlanner.parseGatesAndObstacles(nominalGatePositionAndType, nominalObstaclePosition);
    for (int g : deferredGates) pathWriter.updateGatePos(g, gateRow(g));
    deferredGates.clear();
}

std::vector<double> OnlineTrajGenerator::gateRow(int gateId) const {
    if (gateId < 0 || (size_t)gateId >= nominalGatePositionAndType.rows)
        throw std::out_of_range("gate id " + std::to_string(gateId));
    return std::vector<double>(nominalGatePositionAndType.row(gateId),
                               nominalGatePositionAndType.row(gateId) + nominalGatePositionAndType.cols);
}

// debug dumps + checkpoints — src/OnlineTrajGenerator.cpp:20-47
void OnlineTrajGenerator::init(const Vec3& start, const Vec3& goal) {
    for (size_t i = 0; i < nominalGatePositionAndType.rows; ++i) pathWriter.updateGatePos((int)i, gateRow((int)i));
    for (size_t i = 0; i < nominalObstaclePosition.rows; ++i)
        pathWriter.updateObstaclePos((int)i, std::vector<double>(nominalObstaclePosition.row(i),
                                                                 nominalObstaclePosition.row(i) + nominalObstaclePosition.cols));
    checkpoints.push_back(start);
    const double offset = configParser->getPathPlannerProperties().checkpointGateOffset;
    for (size_t i = 0; i < nominalGatePositionAndType.rows; ++i) {
        Vec3 center, normal;
        getGateCenterAndNormal(gateRow((int)i), center, normal);
        checkpoints.push_back(center - normal * offset);
        checkpoints.push_back(center + normal * offset);
    }
    checkpoints.push_back(goal);
    pathWriter.writeCheckpoints(checkpoints);
}

// src/OnlineTrajGenerator.cpp:50-70
bool OnlineTrajGenerator::getGateCenterAndNormal(const std::vector<double>& g, Vec3& center, Vec3& normal) const {
    if (g[3] != 0 || g[4] != 0) {
        std::cerr << "Only simple rotation around z axis is supported" << std::endl;
        return false;
    }
    const double h = configParser->getObjectPropertiesByTypeId((int)g[6]).height;
    center = Vec3(g[0], g[1], g[2]) + Vec3(0, 0, h);
    normal = Vec3(-std::sin(g[5]), std::cos(g[5]), 0);
    const double nn = normal.norm();
    if (nn > 0) normal = normal / nn;  // normalize()
    return true;
}

// trajectory of the given type through `path` (src/OnlineTrajGenerator.cpp:95-119 and
// :375-410); `pre` = the "optimal" type's re-simulated lead-in points
Matrix OnlineTrajGenerator::generate(const std::vector<Vec3>& path, double t0, const Vec3& v0, const Vec3& a0,
                                     const std::vector<Vec3>& pre) const {
    const auto& tg = configParser->getTrajectoryGeneratorProperties();
    if (tg.type == "snap") {
        Matrix traj;
        poly_traj::generateTrajectory(path, tg.maxVelocity, tg.maxAcceleration, tg.samplingInterval, t0, v0, a0, traj);
        return traj;
    }
    if (tg.type == "optimal")
        return OptimalTimeParametrizer::calculateTrajectory(path, pre, tg.maxVelocity, tg.maxAcceleration, t0,
                                                            tg.samplingInterval, tg.maxTrajDivergence);
    if (tg.type == "spline") return TrajInterpolation().interpolateTraj(path, tg.maxTime, t0, tg.samplingInterval);
    std::cerr << "Trajectory type not supported" << std::endl;
    throw std::runtime_error("Trajectory type not supported");
}

// OnlineTrajGenerator::preComputeTraj — src/OnlineTrajGenerator.cpp:72-121
void OnlineTrajGenerator::preComputeTraj(double takeoffTime) {
    waitForUpdate();
    const double timeLimit = configParser->getPathPlannerProperties().timeLimitOffline;
    pathSegments.clear();
    // the gate-to-gate segments are independent: planned concurrently (the reference
    // loops over them); the first failure in segment order throws, as in the loop
    std::vector<std::pair<Vec3, Vec3>> problems;
    for (size_t i = 0; i + 1 < checkpoints.size(); i += 2) problems.emplace_back(checkpoints[i], checkpoints[i + 1]);
    std::vector<std::vector<Vec3>> paths;
    std::vector<char> ok;
    // (EPP_PRECOMPUTE_TRACE=1, diagnostics: the phases' times to stderr, one line per call)
    static const bool trace = [] {
        const char* e = std::getenv("EPP_PRECOMPUTE_TRACE");
        return e && std::atoi(e) == 1;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    // the plans and includeGates2 in one call: the pruning's ray checks ride in the
    // shortcut's batch (PathPlanner::planPathsIncludeGates2; same answers as the two calls)
    std::vector<Vec3> pruned;
    const bool all = pathPlanner.planPathsIncludeGates2(problems, timeLimit, paths, ok, pruned);
    for (size_t s = 0; s < problems.size(); ++s) {
        if (!ok[s]) throw std::runtime_error("Path not found");
        pathSegments.push_back(paths[s]);
    }
    if (!all) throw std::runtime_error("Path not found");
    const auto t1 = std::chrono::steady_clock::now();
    const auto t2 = t1;  // (includeGates2: inside the call above)
    // the path file is written on the writer's thread while the trajectory is fitted; both
    // are done before the call returns (src/OnlineTrajGenerator.cpp:90-93 in sequence)
    pathWriter.writePathAsync(pruned);
    const auto t3 = std::chrono::steady_clock::now();
    Matrix traj;
    try {
        traj = generate(pruned, takeoffTime, Vec3(0, 0, 0), Vec3(0, 0, 0));
    } catch (...) {
        pathWriter.wait();
        throw;
    }
    pathWriter.wait();
    if (trace) {
        const auto t4 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        std::fprintf(stderr, "precompute_trace: plan=%.0f gates=%.0f write=%.0f generate=%.0f\n", us(t0, t1), us(t1, t2),
                     us(t2, t3), us(t3, t4));
    }
    std::lock_guard<std::mutex> lk(trajMu);
    plannedTraj = std::move(traj);
    waypoints = pruned;
}

// OnlineTrajGenerator::checkGatePassed — src/OnlineTrajGenerator.cpp:228-256
bool OnlineTrajGenerator::checkGatePassed(const Vec3& pos1, const Vec3& pos2, int gateId) const {
    const std::vector<double> gate = gateRow(gateId);
    Vec3 center, normal;
    getGateCenterAndNormal(gate, center, normal);
    const double c = std::cos(gate[5]), s = std::sin(gate[5]);
    const Vec3 t1 = pos1 - center, t2 = pos2 - center;
    const Vec3 g1(c * t1.x - s * t1.y, s * t1.x + c * t1.y, t1.z);
    const Vec3 g2(c * t2.x - s * t2.y, s * t2.x + c * t2.y, t2.z);
    if (g1.y < 0 && g2.y > 0) {
        const Vec3 m = (g1 + g2) / 2;
        const double edgeLength = 0.425;
        if (std::abs(m.x) <= edgeLength && std::abs(m.z) <= edgeLength) return true;
    }
    return false;
}

// OnlineTrajGenerator::updateGatePos — src/OnlineTrajGenerator.cpp:123-226
bool OnlineTrajGenerator::updateGatePos(int gateId, const std::vector<double>& newPose, const Vec3& dronePos,
                                        bool nextGateWithinRange, double flightTime) {
    if (!nextGateWithinRange) return false;
    if (gatesObservedWithinRange.count(gateId)) return false;
    if (!pathPlanner.worldPtr->checkPointValidity(dronePos, false)) return false;
    if (newPose.size() < 6) throw std::invalid_argument("newPose needs 6 values");
    (void)gateRow(gateId);  // range check before anything is recorded
    // a finished online recomputation is collected first (its failure surfaces here)
    if (pending.valid() && pending.wait_for(std::chrono::seconds(0)) == std::future_status::ready) collectUpdate();
    // still running (recalculate_online): it plans on the current world, which is left
    // alone; the new pose is checked on a snapshot and the rebuild deferred (see header)
    const bool busy = pending.valid();
    gatesObservedWithinRange.insert(gateId);
    for (int k = 0; k < 6; ++k) nominalGatePositionAndType(gateId, k) = newPose[k];
    if (busy) {
        deferredGates.push_back(gateId);
    } else {
        pathPlanner.parseGatesAndObstacles(nominalGatePositionAndType, nominalObstaclePosition);
        pathWriter.updateGatePos(gateId, gateRow(gateId));
    }

    Matrix traj;
    {
        std::lock_guard<std::mutex> lk(trajMu);
        traj = plannedTraj;
    }
    if (traj.rows == 0) throw std::runtime_error("No trajectory data available.");
    const size_t tc = traj.cols - 1;
    size_t startIdx = 0;
    double best = std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < traj.rows; ++i) {  // timeDifferences.minCoeff(&startIdx): first minimum
        const double d = std::abs(traj(i, tc) - flightTime);
        if (d < best) {
            best = d;
            startIdx = i;
        }
    }
    Vec3 nc;
    {
        std::lock_guard<std::mutex> lk(cpMu);
        const size_t next = 2 * (size_t)gateId + 3 < checkpoints.size() ? 2 * (size_t)gateId + 3 : checkpoints.size() - 1;
        nc = checkpoints[next];
    }
    size_t endIdx = 0;
    best = std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < traj.rows; ++i) {
        const double d = (Vec3(traj(i, 0), traj(i, 3), traj(i, 6)) - nc).norm();
        if (d < best) {
            best = d;
            endIdx = i;
        }
    }
    Matrix look(endIdx > startIdx ? endIdx - startIdx : 0, traj.cols);
    for (size_t i = 0; i < look.rows; ++i)
        for (size_t c = 0; c < traj.cols; ++c) look(i, c) = traj(startIdx + i, c);
    bool passing = false, valid = false;
    for (size_t i = 0; i + 1 < look.rows; ++i) {
        if (checkGatePassed(Vec3(look(i, 0), look(i, 3), look(i, 6)), Vec3(look(i + 1, 0), look(i + 1, 3), look(i + 1, 6)),
                            gateId)) {
            passing = true;
            break;
        }
    }
    if (passing) {
        const double md = configParser->getPathPlannerProperties().minDistCheckTrajCollision;
        if (busy) {
            World snapshot(configParser);
            PathPlanner::fillWorld(snapshot, nominalGatePositionAndType, nominalObstaclePosition);
            valid = PathPlanner::checkTrajectoryValidityOn(snapshot, look, md);
        } else {
            valid = pathPlanner.checkTrajectoryValidity(look, md);
        }
    }
    if (valid && passing) return false;
    if (busy || trajectoryCurrentlyUpdating.load()) {
        std::cerr << "Call to update trajectory, while previous update is still going on";
        throw std::runtime_error("Call to update trajectory, while previous update is still going on");
    }
    trajectoryCurrentlyUpdating = true;
    if (configParser->getPathPlannerProperties().recalculateOnline) {
#ifdef EPP_TEST_HOOKS
        // EPP_TEST_REPLAN_HOLD_MS (test builds only, -DEPP_TEST_HOOKS: testhooks/): the
        // worker starts that much later, so a test can rely on the recomputation still
        // running while it makes further calls
        const char* hold = std::getenv("EPP_TEST_REPLAN_HOLD_MS");
        const int hold_ms = hold && *hold ? std::max(0, std::atoi(hold)) : 0;
#else
        const int hold_ms = 0;
#endif
        pending = std::async(std::launch::async, [this, gateId, dronePos, flightTime, hold_ms] {
            if (hold_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(hold_ms));
            recomputeTraj(gateId, dronePos, flightTime);
        });
    } else {
        recomputeTraj(gateId, dronePos, flightTime);
    }
    return true;
}

// OnlineTrajGenerator::recomputeTraj — src/OnlineTrajGenerator.cpp:258-421
void OnlineTrajGenerator::recomputeTraj(int gateId, const Vec3& /*dronePos*/, double flightTime) {
    struct Reset {
        std::atomic<bool>& f;
        std::atomic<uint64_t>& failed;
        bool done = false;
        ~Reset() {
            if (!done) ++failed;  // (an exception left the recomputation)
            f = false;
        }
    } reset{trajectoryCurrentlyUpdating, nFailed};
    const auto& pp = configParser->getPathPlannerProperties();
    const int segPre = gateId, segPost = gateId + 1;
    const size_t cpPre = 2 * (size_t)gateId + 1, cpPost = 2 * (size_t)gateId + 2, cpNext = 2 * (size_t)gateId + 3;
    Vec3 center, normal;
    getGateCenterAndNormal(gateRow(segPre), center, normal);
    {
        std::lock_guard<std::mutex> lk(cpMu);
        checkpoints[cpPre] = center - normal * pp.checkpointGateOffset;
        checkpoints[cpPost] = center + normal * pp.checkpointGateOffset;
    }
    pathWriter.writeCheckpoints(checkpoints);

    double advancedTime = flightTime;
    if (pp.advanceForCalculation) advancedTime += pp.timeLimitOnline + 0.01;
    Matrix traj;
    {
        std::lock_guard<std::mutex> lk(trajMu);
        traj = plannedTraj;
    }
    const size_t tc = traj.cols - 1;
    size_t startAdv = 0;
    for (; startAdv < traj.rows; ++startAdv)
        if (traj(startAdv, tc) > advancedTime) break;
    const size_t sRow = std::min(startAdv + 1, traj.rows - 1);  // plannedTraj.row(startIdxAdvanced + 1)
    const Vec3 posA(traj(sRow, 0), traj(sRow, 3), traj(sRow, 6));
    const Vec3 velA(traj(sRow, 1), traj(sRow, 4), traj(sRow, 7));
    const Vec3 accA(traj(sRow, 2), traj(sRow, 5), traj(sRow, 8));
    if (!pathPlanner.worldPtr->checkPointValidity(posA, pp.canPassGate)) {
        std::cerr << "Advanced trajectory does not end at valid position. No recomputation and hope for best"
                  << std::endl;
        ++nSkipped;
        reset.done = true;
        return;
    }
    if (cpNext >= checkpoints.size()) throw std::runtime_error("Post segment path not found. Exiting");
    // the two segments are planned concurrently, like the reference's two threads
    // (src/OnlineTrajGenerator.cpp:324-340)
    std::vector<std::vector<Vec3>> two;
    std::vector<char> okTwo;
    pathPlanner.planPaths({{posA, checkpoints[cpPre]}, {checkpoints[cpPost], checkpoints[cpNext]}}, pp.timeLimitOnline,
                          two, okTwo);
    const std::vector<Vec3>& pre = two[0];
    const std::vector<Vec3>& post = two[1];
    const bool okPre = okTwo[0] != 0, okPost = okTwo[1] != 0;
    if (!okPre) {
        std::cerr << "Pre path not found. Exiting" << std::endl;
        throw std::runtime_error("Pre path not found. Exiting");
    }
    pathSegments[segPre] = pre;
    if (!okPost) {
        std::cerr << "Post segment path not found. Exiting" << std::endl;
        throw std::runtime_error("Post segment path not found. Exiting");
    }
    pathSegments[segPost] = post;
    std::vector<std::vector<Vec3>> slice(pathSegments.begin() + segPre, pathSegments.end());
    const std::vector<Vec3> filled = pathPlanner.includeGates2(slice);
    pathWriter.writePath(filled);
    std::vector<Vec3> lead;  // "optimal": the last prepend_traj_time seconds, re-simulated
    if (configParser->getTrajectoryGeneratorProperties().type == "optimal") {
        const double from = std::max(0.0, advancedTime - configParser->getTrajectoryGeneratorProperties().prependTrajTime);
        for (double t = from; t < advancedTime; t += 0.1) {
            const double* r = traj.row(nearestRow(traj, t));
            lead.emplace_back(r[0], r[3], r[6]);
        }
    }
    const Matrix postTraj = generate(filled, advancedTime, velA, accA, lead);
    Matrix merged(startAdv + postTraj.rows, traj.cols);
    for (size_t i = 0; i < startAdv; ++i)
        for (size_t c = 0; c < traj.cols; ++c) merged(i, c) = traj(i, c);
    for (size_t i = 0; i < postTraj.rows; ++i)
        for (size_t c = 0; c < traj.cols; ++c) merged(startAdv + i, c) = postTraj(i, c);
    std::lock_guard<std::mutex> lk(trajMu);
    plannedTraj = std::move(merged);
    waypoints = filled;
    ++nPlanned;
    reset.done = true;
}

// the row whose time (last column) is nearest to t, first on ties (src/OnlineTrajGenerator.cpp:423-439)
size_t OnlineTrajGenerator::nearestRow(const Matrix& traj, double t) {
    const size_t tc = traj.cols - 1;
    size_t best_i = 0;
    double best = std::numeric_limits<double>::infinity();
    for (size_t i = 0; i < traj.rows; ++i) {
        const double d = std::abs(traj(i, tc) - t);
        if (d < best) {
            best = d;
            best_i = i;
        }
    }
    return best_i;
}

std::vector<double> OnlineTrajGenerator::sampleTraj(double currentTime) const {
    std::lock_guard<std::mutex> lk(trajMu);
    if (plannedTraj.rows == 0) throw std::runtime_error("No trajectory data available.");
    const size_t i = nearestRow(plannedTraj, currentTime);
    return std::vector<double>(plannedTraj.row(i), plannedTraj.row(i) + plannedTraj.cols);
}

std::vector<Vec3> OnlineTrajGenerator::getWaypoints() const {
    std::lock_guard<std::mutex> lk(trajMu);
    return waypoints;
}

double OnlineTrajGenerator::getTrajEndTime() const {
    std::lock_guard<std::mutex> lk(trajMu);
    if (plannedTraj.rows == 0) throw std::runtime_error("No trajectory data available.");
    return plannedTraj(plannedTraj.rows - 1, plannedTraj.cols - 1);
}

Matrix OnlineTrajGenerator::getPlannedTraj() const {
    std::lock_guard<std::mutex> lk(trajMu);
    if (plannedTraj.rows == 0) throw std::runtime_error("No trajectory data available.");
    return plannedTraj;
}

}  // namespace epp

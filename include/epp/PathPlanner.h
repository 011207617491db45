// epp/PathPlanner.h — drop-in for the reference's PathPlanner (include/PathPlanner.h:30-80,
// src/PathPlanner.cpp).  OMPL is replaced by a batch planner on the GPU:
//
//   planPath:  sample `samples_fmt` states in the world bounds (counter RNG), check them
//              (StateValidator semantics), connect every node to its k = 16 nearest
//              neighbours, check all edges at once (MotionValidator semantics), search the
//              shortest valid path on the host, then shortcut it greedily with one batched
//              motion check of all vertex pairs (the role of reduceVertices).
//   includeGates2 / pruneWaypoints / checkTrajectoryValidity: the reference's host logic,
//              with every validity query batched into one GPU launch.
//
// Unlike RRT* with no cost threshold (which always runs to timeLimit), planPath returns
// as soon as the batch search is done; timeLimit only bounds the retries with more
// samples when no path is found.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <functional>
#include <vector>

#include "epp/ConfigParser.h"
#include "epp/World.h"
#include "epp/types.h"

namespace epp {

// Layout version of PlannerStats / PathPlanner below: raise it whenever either changes.
constexpr uint32_t kPlannerAbiVersion = 6;

struct PlannerStats {
    // ABI guard (first, so a caller built against any version reads it): the size of the
    // struct the library filled in; a caller checks lastStats().size == sizeof(PlannerStats)
    uint32_t size = sizeof(PlannerStats);
    uint32_t version = kPlannerAbiVersion;
    int64_t states_sampled = 0;
    int64_t states_valid = 0;
    int64_t edges_checked = 0;    // edges of the graphs searched (the final table's on a fallback)
    int64_t edges_valid = 0;
    int attempts = 0;
    int64_t rows_downloaded = 0;  // k-NN table rows copied to the host (see planPath)
    int64_t restricted_rows = 0;  // of which packed rows of the row-restricted searches
    int64_t fallbacks = 0;        // searches that took the whole table after the restricted rows
    // why (diagnostics): [0] rows past the capacity or > 65,535 nodes, [1] an inexact row,
    // [2] no kept edge into the goal among the rows but one elsewhere in the whole table,
    // [3] a pop above the bound,
    // [4] (forward exhausted: the symmetrised search follows), [5] symmetrised: a pop above
    // the bound, [6] symmetrised: exhausted in the rows
    int64_t fallback_why[7] = {0, 0, 0, 0, 0, 0, 0};
    int64_t restricted_symmetrised = 0;  // searches the rows' symmetrised graph decided
    // of which: after the whole table's k-NN (run for its goal-edge count only: the forward
    // search popped above the bound with no kept edge into the goal among the rows)
    int64_t symmetrised_after_census = 0;
    int64_t astar_pops = 0, restricted_nodes = 0;  // (diagnostics) the restricted searches' closed nodes / node lists
    double ms_restricted_max = 0;                  // (diagnostics) the slowest problem's restricted search
    double ms_copy_of_max = 0;                     // (diagnostics) of which its copy out of pinned memory
    double ms = 0;         // wall time of the last planPath
    double ms_device = 0;  // of which: sampling, checks, k-NN, transfers (GPU phases)
    double ms_search = 0;  // of which: graph build + A* + shortcut on the host
    // wall time of the batched planner's phases (summed over its attempts): the device
    // stages up to the emitted results, the searches on the planner threads, the shortcut
    double ms_batch = 0, ms_solve = 0, ms_shortcut = 0;
    double ms_enqueue = 0;  // of ms_batch: the host until every stage of the batch was queued
};

class PathPlanner {
public:
    // The caller's view of the layout (sizes and version compiled into the CALLER from this
    // header) is handed to the library, which throws std::runtime_error when it differs from
    // its own: a caller built against a stale header (PlannerStats grew, cd38a05) fails at
    // construction instead of reading or writing past the object.
    struct AbiTag {
        uint32_t planner_size, stats_size, version;
    };
    PathPlanner(const Matrix& nominalGatePositionAndType, const Matrix& nominalObstaclePosition,
                std::shared_ptr<ConfigParser> configParser)
        : PathPlanner(nominalGatePositionAndType, nominalObstaclePosition, std::move(configParser),
                      AbiTag{sizeof(PathPlanner), sizeof(PlannerStats), kPlannerAbiVersion}) {}
    PathPlanner(const Matrix& nominalGatePositionAndType, const Matrix& nominalObstaclePosition,
                std::shared_ptr<ConfigParser> configParser, AbiTag callerAbi);

    void parseGatesAndObstacles(const Matrix& nominalGatePositionAndType, const Matrix& nominalObstaclePosition);
    // The world build of parseGatesAndObstacles into any World (src/PathPlanner.cpp:60-78):
    // reset, gates with z := 0, obstacles.
    static void fillWorld(World& world, const Matrix& nominalGatePositionAndType, const Matrix& nominalObstaclePosition);
    // checkTrajectoryValidity against any World (one batched launch)
    static bool checkTrajectoryValidityOn(const World& world, const Matrix& trajectory, double minDistance);
    bool planPath(const Vec3& start, const Vec3& goal, double timeLimit, std::vector<Vec3>& resultPath) const;
    // Independent (start, goal) problems planned together: every device stage runs once
    // for all of them (one launch each, blockIdx.y = the problem), the searches run on
    // planner threads, the shortcut checks are one batch.  Problem i gets the seed of the
    // i-th of consecutive planPath calls, so results do not depend on the batching or on
    // thread timing.  ok[i] / paths[i] as planPath's return value / resultPath; stats =
    // the sum, ms = the batch's wall time.
    void planPaths(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                   std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok) const;
    void updateGatePos(int gateId, const std::vector<double>& newPose);
    bool checkTrajectoryValidity(const Matrix& trajectory, double minDistance) const;
    // The C5 online step in one GPU launch (an addition of this build): returns
    // checkTrajectoryValidity(trajectory, minDistance) and sets `result` to
    // poly_traj::generateTrajectory(waypoints, vMax, aMax, samplingInterval,
    // startTimeOffset, v0, a0) -- the two are independent, so the check runs on extra
    // workgroups of the refit's kernel (epp_check_and_generate_trajectory_host).  Same
    // answers as the two calls; a check too large for the small path makes the two calls.
    bool checkTrajectoryValidityAndGenerate(const Matrix& trajectory, double minDistance,
                                            const std::vector<Vec3>& waypoints, double vMax, double aMax,
                                            double samplingInterval, double startTimeOffset, const Vec3& v0,
                                            const Vec3& a0, Matrix& result) const;
    std::vector<Vec3> includeGates2(std::vector<std::vector<Vec3>> waypoints) const;
    // planPaths of consecutive gate-to-gate segments, then includeGates2 of their paths (an
    // addition of this build, for OnlineTrajGenerator::preComputeTraj): the same answers as
    // the two calls.  The gate centres includeGates2 inserts are the midpoints of the
    // segments' ends, known before the plans, so with the "custom" pruning every ray the
    // pruning can ask rides in the shortcut's batch (each ray tested once for both
    // canPassGate answers): one synchronised launch fewer.  Returns false, `pruned`
    // untouched, when some ok[i] is 0.
    bool planPathsIncludeGates2(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                                std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                                std::vector<Vec3>& pruned) const;

    // batch-planner knobs (defaults follow the config: samples_fmt samples, k = 16)
    void setSeed(uint64_t seed) { seed_ = seed; }
    void setNeighbours(int k) { k_ = k; }
    const PlannerStats& lastStats() const { return stats_; }
    // One batch-planner attempt with an explicit sample count and RNG seed (planPath makes
    // up to 4 of them); public for the CPU restatement's path-equality tests and baselines.
    bool planOnce(const Vec3& start, const Vec3& goal, int64_t samples, uint64_t seed,
                  std::vector<Vec3>& out) const;

    std::shared_ptr<World> worldPtr;

private:
    // A problem of a chain of gate-to-gate segments (planPathsIncludeGates2): the gate
    // centres includeGates2 will put before / after its path and, once the shortcut's batch
    // has run, the canPassGate = true answers of every pair the pruning can ask.
    struct GateEnds {
        bool has_prev = false, has_next = false;
        Vec3 prev, next;
        bool filled = false;       // pts / vis hold the answers
        std::vector<Vec3> pts;     // [prev] + the shortcut's input path + [next]
        std::vector<uint8_t> vis;  // pair (i, j) of pts, j >= i + 2, in the shortcut's queue order
    };
    std::vector<Vec3> pruneWaypoints(const std::vector<Vec3>& waypoints) const;
    std::vector<Vec3> shortcut(const std::vector<Vec3>& path) const;
    std::vector<std::vector<Vec3>> shortcutAll(const std::vector<std::vector<Vec3>>& paths,
                                               const std::vector<GateEnds*>* ends = nullptr) const;
    std::vector<std::vector<Vec3>> pruneAll(const std::vector<std::vector<Vec3>>& segments,
                                            const std::vector<GateEnds>* ends = nullptr) const;
    std::vector<Vec3> includeGates2With(std::vector<std::vector<Vec3>> waypoints,
                                        const std::vector<GateEnds>* ends) const;
    void planPathsWith(const std::vector<std::pair<Vec3, Vec3>>& problems, double timeLimit,
                       std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                       std::vector<GateEnds>* ends) const;
    // omplPrunePathAndInterpolate (src/PathPlanner.cpp:282-313) for every segment at once:
    // OMPL's PathSimplifier::smoothBSpline with its defaults, each step's state and motion
    // checks for all segments in one batch each
    std::vector<std::vector<Vec3>> smoothAll(const std::vector<std::vector<Vec3>>& segments) const;
    // ends (optional): one per problem, filled for the problems whose path is found
    int planCalls(const std::vector<std::pair<Vec3, Vec3>>& problems, uint64_t base, double timeLimit,
                  std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                  std::vector<GateEnds>* ends = nullptr) const;
    void planAttempt(const std::vector<std::pair<Vec3, Vec3>>& problems, const std::vector<uint64_t>& seeds,
                     int64_t samples, std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                     GateEnds* ends = nullptr) const;
    void planChunk(const std::vector<std::pair<Vec3, Vec3>>& problems, const std::vector<uint64_t>& seeds,
                   int64_t samples, std::vector<std::vector<Vec3>>& paths, std::vector<char>& ok,
                   GateEnds* ends = nullptr) const;
    // rows_sym (optional): the caller's symmetrised search on its restricted rows, run while
    // the device builds the whole table's masked k-NN; when that shows no kept edge into the
    // goal and rows_sym found the path, *decided_on_rows = true and the table is neither
    // downloaded nor searched (the caller takes its own path); *census_goal_edges (with
    // rows_sym): the whole table's kept edges into the goal
    bool wholeTableSearch(const double* d_nodes, int32_t n, const double box_lo[3], const double box_hi[3], void* area,
                          std::vector<Vec3>& path, int64_t& edges_checked, int64_t& edges_valid, double& ms_dev,
                          double& ms_search, const std::function<bool()>* rows_sym = nullptr,
                          bool* decided_on_rows = nullptr, int64_t* census_goal_edges = nullptr) const;

    std::shared_ptr<ConfigParser> configParser;
    uint64_t seed_ = 0x5eedull;
    int k_ = 16;
    double ellipse_ = 1.25;  // row-restricted search: bound = ellipse_ |start - goal| + 0.25 m (0: off)
    int threads_ = 16;      // planner threads of a batch's searches (at most one per problem)
    mutable uint64_t calls_ = 0;
    mutable PlannerStats stats_;
};

}  // namespace epp

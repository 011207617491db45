// epp/MultiTrackPlanner.h — independent tracks planned across the GPUs of one node
// (BASELINE config 4).  No reference counterpart: the reference plans one
// track on the CPU.  One host thread per device plans its tracks end to end through
// OnlineTrajGenerator::preComputeTraj (track i on devices[i % n]); the final waypoint
// sets are then all-gathered over RCCL (xGMI), the path's only exchange step, so every
// device ends up holding every track's waypoints.
#pragma once
#include <string>
#include <vector>

#include "epp/types.h"

namespace epp {

struct TrackProblem {
    Vec3 start, goal;
    Matrix gates;      // G x 7 (x, y, z, roll, pitch, yaw, type)
    Matrix obstacles;  // O x 6
};

struct TrackResult {
    std::vector<Vec3> waypoints;  // as all-gathered over RCCL
    Matrix trajectory;            // rows x 10, on the host of the planning thread
    int device = -1;
};

// Throws the exception of the lowest failed rank on a planning failure (e.g.
// std::runtime_error "Path not found"): the failed rank still joins that round's
// all-gather with a count of -1, so every rank leaves at the same round (no rank waits in
// RCCL for one that stopped).  Also throws on an RCCL error or a track with more than 4096
// waypoints (reported on every rank).  A fault of the communicator itself is not
// recoverable.
std::vector<TrackResult> planTracks(const std::vector<TrackProblem>& tracks, const std::string& configPath,
                                    const std::vector<int>& devices, double takeoffTime = 0.0);

}  // namespace epp

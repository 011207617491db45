// epp/OptimalTimeParametrizer.h — the "optimal" trajectory type: time-optimal path
// parametrisation under per-axis velocity / acceleration bounds (Kunz & Stilman, RSS
// 2012) of the waypoint polyline with circular blends.  Replaces
// external/time_parametrization/include/OptimalTimeParametrizer.h:5-16 (same arguments,
// same 11-column result [x, vx, ax, y, vy, ay, z, vz, az, yaw, t + t0]).
#pragma once
#include <vector>

#include "epp/types.h"

namespace epp {
namespace OptimalTimeParametrizer {

// preWaypoints are prepended to waypoints (the reference's way of approximating a
// non-zero initial state); rows start where the trajectory passes closest to
// waypoints[0].  Throws std::runtime_error("Trajectory is not valid") when the
// phase-plane integration fails, std::invalid_argument for fewer than 2 points.
Matrix calculateTrajectory(const std::vector<Vec3>& waypoints, const std::vector<Vec3>& preWaypoints, double v_max,
                           double a_max, double startTimeOffset, double samplingInterval, double maxDivergence);

}  // namespace OptimalTimeParametrizer
}  // namespace epp

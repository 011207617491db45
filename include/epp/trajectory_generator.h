// epp/trajectory_generator.h — drop-in for poly_traj::generateTrajectory
// (external/poly_traj/include/poly_traj/trajectory_generator.h:20,
// external/poly_traj/src/trajectory_generator.cpp:12-100), computed by the batched
// min-snap kernels (include/epp.h epp_minsnap_batch / epp_sample_batch).
#pragma once
#include <vector>

#include "epp/types.h"

namespace poly_traj {

// result: rows x 10 [x, vx, ax, y, vy, ay, z, vz, az, t + startTimeOffset].
// Throws std::invalid_argument("At least two waypoints are required") for < 2 waypoints
// and std::runtime_error for a non-positive segment time (the reference CHECK-aborts).
bool generateTrajectory(const std::vector<epp::Vec3>& waypoints, double v_max, double a_max,
                        double sampling_intervall, double startTimeOffset, const epp::Vec3& initialVel,
                        const epp::Vec3& initialAcc, epp::Matrix& result);

}  // namespace poly_traj

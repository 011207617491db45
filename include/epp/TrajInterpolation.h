// epp/TrajInterpolation.h — the "spline" trajectory type (include/TrajInterpolation.h,
// src/TrajInterpolation.cpp:1-133): a cubic B-spline interpolating the waypoints at
// chord-length parameters (Eigen::SplineFitting<Spline3d>::Interpolate: averaged knots,
// collocation solve), sampled uniformly in the parameter.  A debug type in the
// reference ("for good performance Minimum Snap or Time Optimal Parametrization should
// be utilized"); positions only, velocity/acceleration columns are zero.
#pragma once
#include <vector>

#include "epp/types.h"

namespace epp {

class TrajInterpolation {
public:
    // rows [x 0 0 y 0 0 z 0 0 t]: floor((maxT - advancedTime) / dt) + 1 samples, t = i dt + advancedTime
    Matrix interpolateTraj(const std::vector<Vec3>& path, double maxT, double advancedTime, double dt) const;
    // same spline, times from a per-sample accelerate/cruise profile (src/TrajInterpolation.cpp:96-133)
    Matrix interpolateTrajMaxVel(const std::vector<Vec3>& path, double v_start, double v_max, double a_max,
                                 double advancedTime, double dt) const;
};

}  // namespace epp

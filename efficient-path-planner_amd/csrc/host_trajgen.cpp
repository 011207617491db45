// host_trajgen.cpp — poly_traj::generateTrajectory over the HIP min-snap path.
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "epp.h"
#include "epp/trajectory_generator.h"

namespace poly_traj {

bool generateTrajectory(const std::vector<epp::Vec3>& waypoints, double v_max, double a_max,
                        double sampling_intervall, double startTimeOffset, const epp::Vec3& v0,
                        const epp::Vec3& a0, epp::Matrix& result) {
    if (waypoints.size() < 2) throw std::invalid_argument("At least two waypoints are required");
    std::vector<double> wp(waypoints.size() * 3);
    for (size_t i = 0; i < waypoints.size(); ++i) {
        wp[3 * i] = waypoints[i].x;
        wp[3 * i + 1] = waypoints[i].y;
        wp[3 * i + 2] = waypoints[i].z;
    }
    const double v[3] = {v0.x, v0.y, v0.z}, a[3] = {a0.x, a0.y, a0.z};
    double* rows = nullptr;
    int64_t n = 0;
    const epp_status rc = epp_generate_trajectory_host(wp.data(), (int32_t)waypoints.size(), v_max, a_max,
                                                       sampling_intervall, startTimeOffset, v, a, &rows, &n);
    if (rc == EPP_ERR_INVALID_ARGUMENT) throw std::invalid_argument(epp_last_error());
    if (rc != EPP_OK) throw std::runtime_error(std::string("generateTrajectory: ") + epp_last_error());
    result = epp::Matrix((size_t)n, 10);
    if (n) std::memcpy(result.data.data(), rows, (size_t)n * 10 * sizeof(double));
    epp_host_free(rows);
    return true;
}

}  // namespace poly_traj

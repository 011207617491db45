// host_trajgen.cpp — poly_traj::generateTrajectory over the HIP min-snap path.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "epp.h"
#include "epp_internal.h"
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
    // the rows go straight from the kernel's pinned output into `result` (its storage is
    // reused when the caller passes the previous trajectory back, as a 50 Hz loop does)
    epp::Matrix tmp;
    auto into = [](void* ctx, int64_t R) -> double* {
        epp::Matrix& m = *static_cast<epp::Matrix*>(ctx);
        m.rows = (size_t)R;
        m.cols = 10;
        m.data.resize((size_t)std::max<int64_t>(R, 1) * 10);
        return m.data.data();
    };
    std::swap(tmp, result);  // (result keeps its old value if the call throws)
    int64_t n = 0;
    const epp_status rc = epp::generate_trajectory_into(wp.data(), (int32_t)waypoints.size(), nullptr, v_max, a_max,
                                                        sampling_intervall, startTimeOffset, v, a, into, &tmp, &n);
    if (rc != EPP_OK) {
        std::swap(tmp, result);
        if (rc == EPP_ERR_INVALID_ARGUMENT) throw std::invalid_argument(epp_last_error());
        throw std::runtime_error(std::string("generateTrajectory: ") + epp_last_error());
    }
    tmp.data.resize((size_t)n * 10);
    std::swap(tmp, result);
    return true;
}

}  // namespace poly_traj

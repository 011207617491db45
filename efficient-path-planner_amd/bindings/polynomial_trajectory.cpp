// polynomial_trajectory — the documented Python surface of the reference's min-snap
// wrapper (external/poly_traj/README.md:79, `polynomial_trajectory.generate_trajectory`;
// the reference ships no binding source for it).  Backed by the HIP kernels through
// the C ABI; returns the real 10-column layout of poly_traj::generateTrajectory
// ([x, vx, ax, y, vy, ay, z, vz, az, t], src/trajectory_generator.cpp:81-96).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "epp.h"

namespace py = pybind11;

static py::array_t<double> generate_trajectory(py::array_t<double, py::array::c_style | py::array::forcecast> waypoints,
                                               double v_max, double a_max, double sampling_intervall,
                                               double start_time_offset, py::object initial_vel,
                                               py::object initial_acc) {
    if (waypoints.ndim() != 2 || waypoints.shape(1) != 3)
        throw std::invalid_argument("waypoints must be an (n, 3) array");
    double v0[3] = {0, 0, 0}, a0[3] = {0, 0, 0};
    auto read3 = [](py::object o, double* out) {
        if (o.is_none()) return;
        auto a = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(o);
        if (!a || a.size() != 3) throw std::invalid_argument("initial velocity/acceleration must have 3 entries");
        for (int i = 0; i < 3; ++i) out[i] = a.data()[i];
    };
    read3(initial_vel, v0);
    read3(initial_acc, a0);
    double* rows = nullptr;
    int64_t n = 0;
    epp_status rc;
    {
        py::gil_scoped_release release;
        rc = epp_generate_trajectory_host(waypoints.data(), (int32_t)waypoints.shape(0), v_max, a_max,
                                          sampling_intervall, start_time_offset, v0, a0, &rows, &n);
    }
    if (rc == EPP_ERR_INVALID_ARGUMENT) throw std::invalid_argument(epp_last_error());
    if (rc != EPP_OK) throw std::runtime_error(epp_last_error());
    py::array_t<double> out({(py::ssize_t)n, (py::ssize_t)10});
    if (n) std::memcpy(out.mutable_data(), rows, (size_t)n * 10 * sizeof(double));
    epp_host_free(rows);
    return out;
}

PYBIND11_MODULE(polynomial_trajectory, m) {
    m.doc() = "MI355X min-snap trajectory generation (drop-in for poly_traj::generateTrajectory)";
    m.def("generate_trajectory", &generate_trajectory, py::arg("waypoints"), py::arg("v_max"), py::arg("a_max"),
          py::arg("sampling_intervall"), py::arg("startTimeOffset") = 0.0, py::arg("initialVel") = py::none(),
          py::arg("initialAcc") = py::none());
}

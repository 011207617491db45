// online_traj_planner — drop-in for the reference's pybind module (src/pybind.cpp:10-27):
// the OnlineTrajGenerator class with the same method names, argument names and return
// shapes (numpy arrays where the reference returns Eigen objects), plus the Vector3d /
// MatrixXd helper classes.  Every call releases the GIL while the GPU path runs.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "epp/ConfigParser.h"
#include "epp/MultiTrackPlanner.h"
#include "epp/OnlineTrajGenerator.h"

namespace py = pybind11;
using epp::Matrix;
using epp::Vec3;

using DArr = py::array_t<double, py::array::c_style | py::array::forcecast>;

static Vec3 to_vec3(const py::object& o) {
    if (py::isinstance<Vec3>(o)) return o.cast<Vec3>();
    DArr a = DArr::ensure(o);
    if (!a || a.size() != 3) throw std::invalid_argument("expected 3 values");
    return Vec3(a.data()[0], a.data()[1], a.data()[2]);
}

static Matrix to_matrix(const py::object& o) {
    if (py::isinstance<Matrix>(o)) return o.cast<Matrix>();
    DArr a = DArr::ensure(o);
    if (!a) throw std::invalid_argument("expected a 2-D array");
    if (a.ndim() == 1 && a.size() == 0) return Matrix();
    if (a.ndim() != 2) throw std::invalid_argument("expected a 2-D array");
    Matrix m((size_t)a.shape(0), (size_t)a.shape(1));
    if (a.size()) std::memcpy(m.data.data(), a.data(), (size_t)a.size() * sizeof(double));
    return m;
}

static py::array_t<double> from_matrix(const Matrix& m) {
    py::array_t<double> out({(py::ssize_t)m.rows, (py::ssize_t)m.cols});
    if (!m.data.empty()) std::memcpy(out.mutable_data(), m.data.data(), m.data.size() * sizeof(double));
    return out;
}

PYBIND11_MODULE(online_traj_planner, m) {
    m.doc() = "MI355X drop-in of the online_traj_planner module (OnlineTrajGenerator)";

    py::class_<Vec3>(m, "Vector3d")
        .def(py::init([](const py::object& o) { return to_vec3(o); }))
        .def("__array__", [](const Vec3& v, py::args, py::kwargs) {
            py::array_t<double> a(3);
            a.mutable_data()[0] = v.x;
            a.mutable_data()[1] = v.y;
            a.mutable_data()[2] = v.z;
            return a;
        })
        .def("__repr__", [](const Vec3& v) {
            return "Vector3d(" + std::to_string(v.x) + ", " + std::to_string(v.y) + ", " + std::to_string(v.z) + ")";
        });

    py::class_<Matrix>(m, "MatrixXd")
        .def(py::init([](const py::object& o) { return to_matrix(o); }))
        .def("__array__", [](const Matrix& mat, py::args, py::kwargs) { return from_matrix(mat); })
        .def_property_readonly("shape", [](const Matrix& mat) { return py::make_tuple(mat.rows, mat.cols); });

    // PathPlanner (include/PathPlanner.h:30-80) — not bound by the reference, exposed here
    // so its planner, pruning and trajectory check can be driven and tested from Python.
    py::class_<epp::PathPlanner>(m, "PathPlanner")
        .def(py::init([](const py::object& gates, const py::object& obstacles, const std::string& configPath) {
                 Matrix gm = to_matrix(gates), om = to_matrix(obstacles);
                 auto cfg = std::make_shared<epp::ConfigParser>(configPath);
                 py::gil_scoped_release release;
                 return new epp::PathPlanner(gm, om, cfg);
             }),
             py::arg("nominalGatePositionAndType"), py::arg("nominalObstaclePosition"), py::arg("configPath"))
        .def(
            "plan_path",
            [](const epp::PathPlanner& self, const py::object& start, const py::object& goal,
               double timeLimit) -> py::object {
                Vec3 s = to_vec3(start), g = to_vec3(goal);
                std::vector<Vec3> path;
                bool ok;
                {
                    py::gil_scoped_release release;
                    ok = self.planPath(s, g, timeLimit, path);
                }
                if (!ok) return py::none();
                py::array_t<double> out({(py::ssize_t)path.size(), (py::ssize_t)3});
                for (size_t i = 0; i < path.size(); ++i)
                    for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = path[i][k];
                return out;
            },
            py::arg("start"), py::arg("goal"), py::arg("timeLimit") = 1.0)
        .def(
            "include_gates2",
            [](const epp::PathPlanner& self, const py::list& segments) {
                std::vector<std::vector<Vec3>> wp;
                for (const auto& s : segments) {
                    Matrix m = to_matrix(py::reinterpret_borrow<py::object>(s));
                    if (m.cols != 3) throw std::invalid_argument("segments must be (n, 3) arrays");
                    std::vector<Vec3> seg;
                    for (size_t i = 0; i < m.rows; ++i) seg.emplace_back(m(i, 0), m(i, 1), m(i, 2));
                    if (seg.empty()) throw std::invalid_argument("empty segment");
                    wp.push_back(std::move(seg));
                }
                if (wp.empty()) throw std::invalid_argument("no segments");
                std::vector<Vec3> flat;
                {
                    py::gil_scoped_release release;
                    flat = self.includeGates2(wp);
                }
                py::array_t<double> out({(py::ssize_t)flat.size(), (py::ssize_t)3});
                for (size_t i = 0; i < flat.size(); ++i)
                    for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = flat[i][k];
                return out;
            },
            py::arg("waypoints"))
        .def(
            "check_trajectory_validity",
            [](const epp::PathPlanner& self, const py::object& traj, double minDistance) {
                Matrix m = to_matrix(traj);
                py::gil_scoped_release release;
                return self.checkTrajectoryValidity(m, minDistance);
            },
            py::arg("trajectory"), py::arg("minDistance"))
        .def(
            "check_trajectory_validity_and_generate",  // the C5 online step in one launch (this build)
            [](const epp::PathPlanner& self, const py::object& traj, double minDistance, const py::object& waypoints,
               double vMax, double aMax, double samplingInterval, double startTimeOffset, const py::object& v0,
               const py::object& a0) {
                Matrix m = to_matrix(traj), w = to_matrix(waypoints);
                if (w.cols != 3) throw std::invalid_argument("waypoints must be an (n, 3) array");
                std::vector<Vec3> wp;
                for (size_t i = 0; i < w.rows; ++i) wp.emplace_back(w(i, 0), w(i, 1), w(i, 2));
                const Vec3 v = to_vec3(v0), a = to_vec3(a0);
                Matrix out;
                bool valid;
                {
                    py::gil_scoped_release release;
                    valid = self.checkTrajectoryValidityAndGenerate(m, minDistance, wp, vMax, aMax, samplingInterval,
                                                                    startTimeOffset, v, a, out);
                }
                return py::make_tuple(valid, from_matrix(out));
            },
            py::arg("trajectory"), py::arg("minDistance"), py::arg("waypoints"), py::arg("v_max"), py::arg("a_max"),
            py::arg("sampling_interval"), py::arg("startTimeOffset") = 0.0,
            py::arg("v0") = py::make_tuple(0.0, 0.0, 0.0), py::arg("a0") = py::make_tuple(0.0, 0.0, 0.0))
        .def(
            "check_point_validity",
            [](const epp::PathPlanner& self, const py::object& p, bool canPassGate) {
                return self.worldPtr->checkPointValidity(to_vec3(p), canPassGate);
            },
            py::arg("point"), py::arg("canPassGate"))
        .def(
            "check_ray_valid",
            [](const epp::PathPlanner& self, const py::object& a, const py::object& b, bool canPassGate) {
                return self.worldPtr->checkRayValid(to_vec3(a), to_vec3(b), canPassGate);
            },
            py::arg("start"), py::arg("end"), py::arg("canPassGate") = false)
        .def("update_gate_pos",
             [](epp::PathPlanner& self, int gateId, const std::vector<double>& pose) { self.updateGatePos(gateId, pose); })
        .def(
            "plan_paths",  // concurrent planPath over independent (start, goal) pairs
            [](const epp::PathPlanner& self, const std::vector<std::pair<py::object, py::object>>& problems,
               double timeLimit) {
                std::vector<std::pair<Vec3, Vec3>> pr;
                for (const auto& p : problems) pr.emplace_back(to_vec3(p.first), to_vec3(p.second));
                std::vector<std::vector<Vec3>> paths;
                std::vector<char> ok;
                {
                    py::gil_scoped_release release;
                    self.planPaths(pr, timeLimit, paths, ok);
                }
                py::list out;
                for (size_t i = 0; i < pr.size(); ++i) {
                    py::array_t<double> a({(py::ssize_t)paths[i].size(), (py::ssize_t)3});
                    for (size_t j = 0; j < paths[i].size(); ++j)
                        for (int k = 0; k < 3; ++k) a.mutable_data()[j * 3 + k] = paths[i][j][k];
                    out.append(py::make_tuple((bool)ok[i], a));
                }
                return out;
            },
            py::arg("problems"), py::arg("timeLimit"))
        .def(
            "plan_paths_include_gates2",  // planPaths of a chain of segments + includeGates2 in one call
            [](const epp::PathPlanner& self, const std::vector<std::pair<py::object, py::object>>& problems,
               double timeLimit) -> py::object {
                std::vector<std::pair<Vec3, Vec3>> pr;
                for (const auto& p : problems) pr.emplace_back(to_vec3(p.first), to_vec3(p.second));
                std::vector<std::vector<Vec3>> paths;
                std::vector<char> ok;
                std::vector<Vec3> flat;
                bool all;
                {
                    py::gil_scoped_release release;
                    all = self.planPathsIncludeGates2(pr, timeLimit, paths, ok, flat);
                }
                py::list segs;
                for (size_t i = 0; i < pr.size(); ++i) {
                    py::array_t<double> a({(py::ssize_t)paths[i].size(), (py::ssize_t)3});
                    for (size_t j = 0; j < paths[i].size(); ++j)
                        for (int k = 0; k < 3; ++k) a.mutable_data()[j * 3 + k] = paths[i][j][k];
                    segs.append(py::make_tuple((bool)ok[i], a));
                }
                if (!all) return py::make_tuple(segs, py::none());
                py::array_t<double> out({(py::ssize_t)flat.size(), (py::ssize_t)3});
                for (size_t i = 0; i < flat.size(); ++i)
                    for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = flat[i][k];
                return py::make_tuple(segs, out);
            },
            py::arg("problems"), py::arg("timeLimit"))
        .def(
            "check_rays_both",  // World::checkRaysBoth: bit 0 canPassGate = false, bit 1 true
            [](const epp::PathPlanner& self, const py::object& s1, const py::object& s2) {
                Matrix a = to_matrix(s1), b = to_matrix(s2);
                if (a.cols != 3 || b.cols != 3 || a.rows != b.rows)
                    throw std::invalid_argument("s1 and s2 must be (n, 3) arrays of one length");
                py::array_t<uint8_t> out((py::ssize_t)a.rows);
                {
                    py::gil_scoped_release release;
                    self.worldPtr->checkRaysBoth(a.data.data(), b.data.data(), (int64_t)a.rows, out.mutable_data());
                }
                return out;
            },
            py::arg("s1"), py::arg("s2"))
        .def(
            "plan_once",  // one batch-planner attempt with an explicit sample count and seed
            [](const epp::PathPlanner& self, const py::object& start, const py::object& goal, int64_t samples,
               uint64_t seed) -> py::object {
                Vec3 s = to_vec3(start), g = to_vec3(goal);
                std::vector<Vec3> path;
                bool ok;
                {
                    py::gil_scoped_release release;
                    ok = self.planOnce(s, g, samples, seed, path);
                }
                if (!ok) return py::none();
                py::array_t<double> out({(py::ssize_t)path.size(), (py::ssize_t)3});
                for (size_t i = 0; i < path.size(); ++i)
                    for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = path[i][k];
                return out;
            },
            py::arg("start"), py::arg("goal"), py::arg("samples"), py::arg("seed"))
        .def(
            "world_obbs",  // the world's OBBs as built (center xyz, half sizes): (n, 6)
            [](const epp::PathPlanner& self) {
                (void)self.worldPtr->device();  // the flattened table is rebuilt lazily
                const auto& o = self.worldPtr->obbs();
                py::array_t<double> out({(py::ssize_t)o.size(), (py::ssize_t)6});
                for (size_t i = 0; i < o.size(); ++i)
                    for (int k = 0; k < 3; ++k) {
                        out.mutable_data()[i * 6 + k] = o[i].center[k];
                        out.mutable_data()[i * 6 + 3 + k] = o[i].half[k];
                    }
                return out;
            })
        .def("set_seed", &epp::PathPlanner::setSeed)
        .def("set_neighbours", &epp::PathPlanner::setNeighbours)
        .def("last_stats", [](const epp::PathPlanner& self) {
            const auto& s = self.lastStats();
            py::dict d;
            if (s.size != sizeof(epp::PlannerStats) || s.version != epp::kPlannerAbiVersion)
                throw std::runtime_error("PlannerStats: the library's layout differs from this module's header");
            d["size"] = s.size;
            d["version"] = s.version;
            d["states_sampled"] = s.states_sampled;
            d["states_valid"] = s.states_valid;
            d["edges_checked"] = s.edges_checked;
            d["edges_valid"] = s.edges_valid;
            d["attempts"] = s.attempts;
            d["rows_downloaded"] = s.rows_downloaded;
            d["restricted_rows"] = s.restricted_rows;
            d["fallbacks"] = s.fallbacks;
            d["fallback_why"] = std::vector<int64_t>(s.fallback_why, s.fallback_why + 7);
            d["restricted_symmetrised"] = s.restricted_symmetrised;
            d["symmetrised_after_census"] = s.symmetrised_after_census;
            d["astar_pops"] = s.astar_pops;
            d["restricted_nodes"] = s.restricted_nodes;
            d["ms_restricted_max"] = s.ms_restricted_max;
            d["ms_copy_of_max"] = s.ms_copy_of_max;
            d["ms_batch"] = s.ms_batch;
            d["ms_enqueue"] = s.ms_enqueue;
            d["ms_solve"] = s.ms_solve;
            d["ms_shortcut"] = s.ms_shortcut;
            d["ms"] = s.ms;
            d["ms_device"] = s.ms_device;
            d["ms_search"] = s.ms_search;
            return d;
        });

    // ConfigParser (src/ConfigParserYAML.cpp:10-118): the parsed configuration as a dict
    // (JSON or block-YAML file, as YAML::LoadFile reads either); no GPU involved
    m.def(
        "load_config",
        [](const std::string& configPath) {
            epp::ConfigParser c(configPath);
            auto v3 = [](const Vec3& v) { return py::make_tuple(v[0], v[1], v[2]); };
            auto obbs = [&](const std::vector<epp::OBBDescription>& ds) {
                py::list l;
                for (const auto& d : ds) {
                    py::dict o;
                    o["center"] = v3(d.center);
                    o["half_size"] = v3(d.halfSize);
                    o["type"] = d.type;
                    o["name"] = d.name;
                    l.append(o);
                }
                return l;
            };
            py::dict out, gates, heights;
            for (int t = 0; t < c.numGateTypes(); ++t) {
                gates[py::int_(t)] = obbs(c.getGateGeometryByTypeId(t));
                heights[py::int_(t)] = c.getObjectPropertiesByTypeId(t).height;
            }
            out["gate_geometry"] = gates;
            out["gate_height"] = heights;
            out["obstacle_geometry"] = obbs(c.getObstacleGeometry());
            const auto& w = c.getWorldProperties();
            py::dict wd;
            wd["lower_bound"] = v3(w.lowerBound);
            wd["upper_bound"] = v3(w.upperBound);
            wd["inflate_radius"] = w.inflateRadius;
            out["world"] = wd;
            const auto& p = c.getPathPlannerProperties();
            py::dict pd;
            pd["optimality_threshold_percentage"] = p.optimalityThresholdPercentage;
            pd["time_limit_online"] = p.timeLimitOnline;
            pd["time_limit_offline"] = p.timeLimitOffline;
            pd["checkpoint_gate_offset"] = p.checkpointGateOffset;
            pd["range"] = p.range;
            pd["min_dist_check_traj_collision"] = p.minDistCheckTrajCollision;
            pd["path_simplification"] = p.pathSimplification;
            pd["recalculate_online"] = p.recalculateOnline;
            pd["can_pass_gate"] = p.canPassGate;
            pd["advance_for_calculation"] = p.advanceForCalculation;
            pd["planner"] = p.planner;
            pd["samples_fmt"] = p.samplesFMT;
            out["path_planner"] = pd;
            const auto& g = c.getTrajectoryGeneratorProperties();
            py::dict gd;
            gd["max_velocity"] = g.maxVelocity;
            gd["max_acceleration"] = g.maxAcceleration;
            gd["sampling_interval"] = g.samplingInterval;
            gd["type"] = g.type;
            gd["max_time"] = g.maxTime;
            gd["prepend_traj_time"] = g.prependTrajTime;
            gd["max_traj_divergence"] = g.maxTrajDivergence;
            out["trajectory_generator"] = gd;
            return out;
        },
        py::arg("configPath"));

    // planTracks (include/epp/MultiTrackPlanner.h): independent tracks across GPUs of this
    // node, one host thread per device, waypoint sets all-gathered over RCCL
    m.def(
        "plan_tracks",
        [](const py::list& problems, const std::string& configPath, const std::vector<int>& devices,
           double takeoffTime) {
            std::vector<epp::TrackProblem> tp;
            for (const auto& item : problems) {
                py::tuple t = py::reinterpret_borrow<py::tuple>(item);
                if (t.size() != 4) throw std::invalid_argument("problems: (start, goal, gates, obstacles) tuples");
                tp.push_back({to_vec3(t[0]), to_vec3(t[1]), to_matrix(t[2]), to_matrix(t[3])});
            }
            std::vector<epp::TrackResult> res;
            {
                py::gil_scoped_release release;
                res = epp::planTracks(tp, configPath, devices, takeoffTime);
            }
            py::list out;
            for (const auto& r : res) {
                py::array_t<double> wp({(py::ssize_t)r.waypoints.size(), (py::ssize_t)3});
                for (size_t i = 0; i < r.waypoints.size(); ++i)
                    for (int k = 0; k < 3; ++k) wp.mutable_data()[i * 3 + k] = r.waypoints[i][k];
                out.append(py::make_tuple(wp, from_matrix(r.trajectory), r.device));
            }
            return out;
        },
        py::arg("problems"), py::arg("configPath"), py::arg("devices"), py::arg("takeoffTime") = 0.0);

    py::class_<epp::OnlineTrajGenerator>(m, "OnlineTrajGenerator")
        .def(py::init([](const py::object& start, const py::object& goal, const py::object& gates,
                         const py::object& obstacles, const std::string& configPath) {
                 Vec3 s = to_vec3(start), g = to_vec3(goal);
                 Matrix gm = to_matrix(gates), om = to_matrix(obstacles);
                 py::gil_scoped_release release;
                 return new epp::OnlineTrajGenerator(s, g, gm, om, configPath);
             }),
             py::arg("start"), py::arg("goal"), py::arg("nominalGatePositionAndType"),
             py::arg("nominalObstaclePosition"), py::arg("configPath"))
        .def("pre_compute_traj", &epp::OnlineTrajGenerator::preComputeTraj, py::arg("takeoffTime"),
             py::call_guard<py::gil_scoped_release>())
        .def(
            "update_gate_pos",
            [](epp::OnlineTrajGenerator& self, int gateId, const py::object& newPose, const py::object& dronePos,
               bool nextGateWithinRange, double flightTime) {
                DArr p = DArr::ensure(newPose);
                if (!p || p.size() < 6) throw std::invalid_argument("newPose needs 6 values");
                std::vector<double> pose(p.data(), p.data() + p.size());
                Vec3 d = to_vec3(dronePos);
                py::gil_scoped_release release;
                return self.updateGatePos(gateId, pose, d, nextGateWithinRange, flightTime);
            },
            py::arg("gateId"), py::arg("newPose"), py::arg("dronePos"), py::arg("nextGateWithinRange"),
            py::arg("flightTime"))
        .def(
            "sample_traj",
            [](const epp::OnlineTrajGenerator& self, double t) {
                std::vector<double> r = self.sampleTraj(t);
                py::array_t<double> out((py::ssize_t)r.size());
                std::memcpy(out.mutable_data(), r.data(), r.size() * sizeof(double));
                return out;
            },
            py::arg("currentTime"))
        .def("get_traj_end_time", &epp::OnlineTrajGenerator::getTrajEndTime)
        .def("get_planned_traj", [](const epp::OnlineTrajGenerator& self) { return from_matrix(self.getPlannedTraj()); })
        // additions of this build
        .def("wait_for_update", &epp::OnlineTrajGenerator::waitForUpdate, py::call_guard<py::gil_scoped_release>())
        .def("recompute_counts",
             [](const epp::OnlineTrajGenerator& self) {
                 const auto c = self.recomputeCounts();
                 py::dict d;
                 d["planned"] = c.planned;
                 d["skipped_invalid_start"] = c.skippedInvalidStart;
                 d["failed"] = c.failed;
                 return d;
             })
        .def(
            "planner", [](epp::OnlineTrajGenerator& self) -> epp::PathPlanner& { return self.planner(); },
            py::return_value_policy::reference_internal)
        .def("get_waypoints", [](const epp::OnlineTrajGenerator& self) {
            const auto c = self.getWaypoints();
            py::array_t<double> out({(py::ssize_t)c.size(), (py::ssize_t)3});
            for (size_t i = 0; i < c.size(); ++i)
                for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = c[i][k];
            return out;
        })
        .def("planner_stats", [](epp::OnlineTrajGenerator& self) {
            const auto& s = self.planner().lastStats();
            py::dict d;
            if (s.size != sizeof(epp::PlannerStats) || s.version != epp::kPlannerAbiVersion)
                throw std::runtime_error("PlannerStats: the library's layout differs from this module's header");
            d["size"] = s.size;
            d["version"] = s.version;
            d["states_sampled"] = s.states_sampled;
            d["edges_checked"] = s.edges_checked;
            d["ms"] = s.ms;
            d["ms_device"] = s.ms_device;
            d["ms_search"] = s.ms_search;
            d["attempts"] = s.attempts;
            d["rows_downloaded"] = s.rows_downloaded;
            d["restricted_rows"] = s.restricted_rows;
            d["fallbacks"] = s.fallbacks;
            d["fallback_why"] = std::vector<int64_t>(s.fallback_why, s.fallback_why + 7);
            d["restricted_symmetrised"] = s.restricted_symmetrised;
            d["symmetrised_after_census"] = s.symmetrised_after_census;
            d["astar_pops"] = s.astar_pops;
            d["restricted_nodes"] = s.restricted_nodes;
            d["ms_restricted_max"] = s.ms_restricted_max;
            d["ms_copy_of_max"] = s.ms_copy_of_max;
            d["ms_batch"] = s.ms_batch;
            d["ms_enqueue"] = s.ms_enqueue;
            d["ms_solve"] = s.ms_solve;
            d["ms_shortcut"] = s.ms_shortcut;
            return d;
        })
        .def("get_checkpoints", [](const epp::OnlineTrajGenerator& self) {
            const auto& c = self.getCheckpoints();
            py::array_t<double> out({(py::ssize_t)c.size(), (py::ssize_t)3});
            for (size_t i = 0; i < c.size(); ++i)
                for (int k = 0; k < 3; ++k) out.mutable_data()[i * 3 + k] = c[i][k];
            return out;
        });
}

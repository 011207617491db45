// host_objects.cpp — world construction from gate / obstacle poses (host side).
//
// Reference: World::addGatePrivateOperation / addObstacle (src/World.cpp:13-55),
// Object::createFromDescription / translate / rotateZ (src/Object.cpp:11-85).
// The arithmetic order is the reference's: centre = (desc + g) - g rotated by
// Rz(yaw), plus g; rotation = Rz(yaw) * I.  Rz has exact zeros off its xy block, so
// the 3x3 products reduce to two rounded products and one rounded sum per axis no
// matter how Eigen orders the sum.
#include <cmath>
#include <cstring>
#include <string>

#include "epp_internal.h"

namespace {

int add_object(const double g_in[3], const double rot[3], const epp_obb_desc* d, int nd,
               int is_gate, epp_obb* out, int capacity, int* count) {
    if (std::fabs(rot[0]) > 1e-6) {
        epp::set_error("Rotation around x axis is not supported");  // Object.cpp:38-42
        return EPP_ERR_UNSUPPORTED;
    }
    if (std::fabs(rot[1]) > 1e-6) {
        epp::set_error("Rotation around y axis is not supported");  // Object.cpp:43-47
        return EPP_ERR_UNSUPPORTED;
    }
    if (g_in[2] > 1e-6) {
        epp::set_error("Center z position must be zero");  // Object.cpp:16-20
        return EPP_ERR_RUNTIME;
    }
    const double gc[3] = {0.0 + g_in[0], 0.0 + g_in[1], 0.0 + g_in[2]};  // globalCenter += t
    const double c = std::cos(rot[2]), s = std::sin(rot[2]);            // Object.cpp:69-70
    for (int k = 0; k < nd; ++k) {
        const int idx = (*count)++;
        if (idx >= capacity) continue;  // counted, reported as EPP_ERR_CAPACITY
        epp_obb& o = out[idx];
        std::memset(&o, 0, sizeof(o));
        double ctr[3];
        for (int i = 0; i < 3; ++i) {
            o.half[i] = d[k].size[i] / 2;       // ConfigParserYAML.cpp:63
            ctr[i] = d[k].pos[i] + g_in[i];     // translate (Object.cpp:57)
        }
        const double rx = ctr[0] - gc[0], ry = ctr[1] - gc[1], rz = ctr[2] - gc[2];  // :81
        o.center[0] = (c * rx - s * ry) + gc[0];  // rotation * relativeCenter + globalCenter  :82
        o.center[1] = (s * rx + c * ry) + gc[1];
        o.center[2] = rz + gc[2];
        const double R[9] = {c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0};  // Object.cpp:72-75, :83
        std::memcpy(o.rot, R, sizeof(R));
        o.filling = d[k].filling ? 1 : 0;
        o.is_gate = is_gate;
    }
    return EPP_OK;
}

}  // namespace

extern "C" epp_status epp_build_obbs(const epp_obb_desc* gate_desc, const int32_t* gate_desc_off,
                                     int32_t n_gate_types, const epp_obb_desc* obst_desc,
                                     int32_t n_obst_desc, const double* gates, int32_t n_gates,
                                     const double* obstacles, int32_t n_obstacles, epp_obb* out,
                                     int32_t capacity, int32_t* n_out) {
    if (!n_out || n_gates < 0 || n_obstacles < 0 || (n_gates > 0 && (!gates || !gate_desc_off)) ||
        (n_obstacles > 0 && !obstacles) || (capacity > 0 && !out)) {
        epp::set_error("epp_build_obbs: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    int count = 0;
    for (int g = 0; g < n_gates; ++g) {
        const double* row = gates + 7 * g;
        const double pos[3] = {row[0], row[1], 0.0};  // gate(2) = 0  PathPlanner.cpp:68
        const double rot[3] = {row[3], row[4], row[5]};
        const int type = (int)row[6];                  // World.cpp:18
        if (type < 0 || type >= n_gate_types) {
            epp::set_error("unknown gate type " + std::to_string(type));
            return EPP_ERR_RUNTIME;
        }
        const int rc = add_object(pos, rot, gate_desc + gate_desc_off[type],
                                  gate_desc_off[type + 1] - gate_desc_off[type], 1, out, capacity, &count);
        if (rc) return rc;
    }
    for (int k = 0; k < n_obstacles; ++k) {
        const double* row = obstacles + 6 * k;
        const double pos[3] = {row[0], row[1], row[2]};
        const double rot[3] = {row[3], row[4], row[5]};
        const int rc = add_object(pos, rot, obst_desc, n_obst_desc, 0, out, capacity, &count);
        if (rc) return rc;
    }
    *n_out = count;
    if (count > capacity) {
        epp::set_error("epp_build_obbs: output capacity too small");
        return EPP_ERR_CAPACITY;
    }
    return EPP_OK;
}

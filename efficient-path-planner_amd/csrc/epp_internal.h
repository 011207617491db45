// epp_internal.h — layouts shared by the host library and the HIP kernels.
//
// The world lives in HBM as one contiguous blob so that a workgroup can stage it
// into LDS with straight 16-byte copies:
//
//   double  soa[EPP_NF][n_pad]   field-major OBB table (see enum below)
//   uint32  meta[n_pad]          bit0 filling, bit1 gate, bits 8-15/16-23/24-31 = first
//                                cull-grid cell (x, y, z) the OBB's AABB touches
//   uint32  cell_start[ncell+1]  CSR offsets of the cull grid
//   uint16  cell_obb[...]        OBB ids per cell
//
// n_pad rounds n_obbs up to a multiple of 2 so every array stays 16-byte aligned.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "epp.h"

namespace epp {

// field index into the SoA table
enum Field : int {
    F_LOX = 0, F_LOY, F_LOZ, F_HIX, F_HIY, F_HIZ,  // AABB (rtree box, World.cpp:57-67)
    F_CX, F_CY, F_CZ,                              // OBB centre
    F_COS, F_SIN,                                  // R = [[c,-s,0],[s,c,0],[0,0,1]]
    F_HX, F_HY, F_HZ,                              // half sizes
    F_R,                                           // owner inflate radius (gate/obstacle)
    EPP_NF
};

constexpr uint32_t META_FILLING = 1u;
constexpr uint32_t META_GATE = 2u;
constexpr int kMaxGridAxis = 255;

// Passed to kernels by value.
struct WorldView {
    const unsigned char* blob;  // device pointer
    uint32_t blob_bytes;
    int32_t n_obb;
    int32_t n_pad;
    int32_t nx, ny, nz;
    uint32_t off_meta;        // byte offsets inside the blob
    uint32_t off_cell_start;
    uint32_t off_cell_obb;
    double gx0, gy0, gz0;     // grid origin = min AABB lo
    double gx1, gy1, gz1;     // grid far corner = max AABB hi
    double icx, icy, icz;     // 1 / cell size
};

// Host-side world: the upload plus host copies (for AABB introspection and rebuilds).
struct HostWorld {
    WorldView view{};
    double r_gate = 0, r_obst = 0;
    int device = 0;
    void* d_blob = nullptr;
    size_t d_capacity = 0;
    std::string blob;            // host image of the device blob
    std::vector<double> aabbs;   // n x 6
};

// Cell index along one axis: same double operations on host and device, so the
// candidate lists are exact (no rounding slack needed: floor(fl((p-o)*inv)) is
// monotone in p).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline int cell_of(double p, double o, double inv, int n) {
    double f = (p - o) * inv;
    int c;
    if (!(f >= 0.0)) c = 0;                    // also catches NaN
    else if (f >= (double)n) c = n - 1;
    else c = (int)f;                           // f >= 0: truncation == floor
    return c < n ? c : n - 1;
}

void set_error(const std::string& msg);

}  // namespace epp

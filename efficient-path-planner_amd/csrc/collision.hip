// collision.hip — batched OBB validity kernels for gfx950 (MI355X).
//
//   k_states  : World::checkPointValidity(p, canPassGate)  src/World.cpp:80-104
//               World::checkPointValidity(p, minDistance)  src/World.cpp:106-128  (MINDIST)
//               + optional wave-ballot compaction of the valid states
//   k_motions : World::checkRayValid(s, e, canPassGate)     src/World.cpp:130-162
//               discrete32 mode: 32 point checks along the edge
//
// Layout: one lane owns 4 consecutive states (96 B, six 16-B loads) or 4 edges, and
// writes their 4 flag bytes with one 32-bit store, so a wavefront streams 6 KB in and
// 256 B out per item group.  The world blob (OBB SoA + cull grid, epp_internal.h) is
// staged once per workgroup into LDS; grids are persistent (grid-stride) so the
// staging is amortised.  All decision arithmetic is IEEE fp64 with contraction
// disabled (-ffp-contract=off): booleans match the reference bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "epp_internal.h"

namespace epp {
const WorldView& world_view(const epp_world* w);

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kLdsBudget = 64 * 1024;

struct Acc {
    const double* f;
    int n_pad;
    const uint32_t* meta;
    const uint32_t* cs;
    const uint16_t* co;
    __device__ __forceinline__ double g(int field, int i) const { return f[field * n_pad + i]; }
};

__device__ __forceinline__ Acc make_acc(const unsigned char* base, const WorldView& w) {
    Acc a;
    a.f = reinterpret_cast<const double*>(base);
    a.n_pad = w.n_pad;
    a.meta = reinterpret_cast<const uint32_t*>(base + w.off_meta);
    a.cs = reinterpret_cast<const uint32_t*>(base + w.off_cell_start);
    a.co = reinterpret_cast<const uint16_t*>(base + w.off_cell_obb);
    return a;
}

// OBB::checkCollisionWithPoint — src/OBB.cpp:63-91.  R = Rz, so
// R^T (p - c) = (c*dx + s*dy, c*dy - s*dx, dz) exactly as Eigen evaluates it.
__device__ __forceinline__ bool obb_point_hit(const Acc& a, int i, uint32_t m, double px,
                                              double py, double pz, double r) {
    const double c = a.g(F_COS, i), s = a.g(F_SIN, i);
    const double dx = px - a.g(F_CX, i), dy = py - a.g(F_CY, i), dz = pz - a.g(F_CZ, i);
    const double lx = c * dx + s * dy;
    const double ly = c * dy - s * dx;
    double tx = a.g(F_HX, i), ty = a.g(F_HY, i), tz = a.g(F_HZ, i);
    if (!(m & META_FILLING)) {  // shouldBeInflated()  include/OBB.h:54-57
        tx = tx + r;
        ty = ty + r;
        tz = tz + r;
    }
    return fabs(lx) <= tx && fabs(ly) <= ty && fabs(dz) <= tz;
}

// OBB::checkCollisionWithRay — src/OBB.cpp:10-61
__device__ __forceinline__ bool obb_ray_hit(const Acc& a, int i, uint32_t m, const double s[3],
                                            const double e[3], double r) {
    if (obb_point_hit(a, i, m, s[0], s[1], s[2], r) || obb_point_hit(a, i, m, e[0], e[1], e[2], r))
        return true;  // :13-18
    const double c = a.g(F_COS, i), sn = a.g(F_SIN, i);
    const double cx = a.g(F_CX, i), cy = a.g(F_CY, i), cz = a.g(F_CZ, i);
    double ls[3], ld[3];
    {
        const double dx = s[0] - cx, dy = s[1] - cy, dz = s[2] - cz;
        ls[0] = c * dx + sn * dy;
        ls[1] = c * dy - sn * dx;
        ls[2] = dz;
        const double ex = e[0] - cx, ey = e[1] - cy, ez = e[2] - cz;
        ld[0] = (c * ex + sn * ey) - ls[0];  // localEnd - localStart  :23
        ld[1] = (c * ey - sn * ex) - ls[1];
        ld[2] = ez - ls[2];
    }
    const double h[3] = {a.g(F_HX, i), a.g(F_HY, i), a.g(F_HZ, i)};
    double tMin = 0.0, tMax = 1.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double ih = h[k] + r;  // always inflated  :28
        const double bmin = -ih, bmax = ih;
        if (fabs(ld[k]) < 1e-6) {  // :34
            if (ls[k] < bmin || ls[k] > bmax) return false;
        } else {
            const double invD = 1.0 / ld[k];  // :44
            const double t1 = (bmin - ls[k]) * invD;
            const double t2 = (bmax - ls[k]) * invD;
            const double tEntry = (t2 < t1) ? t2 : t1;  // std::min
            const double tExit = (t1 < t2) ? t2 : t1;   // std::max
            tMin = (tMin < tEntry) ? tEntry : tMin;     // std::max
            tMax = (tExit < tMax) ? tExit : tMax;       // std::min
            if (tMin > tMax) return false;
        }
    }
    return 0 <= tMin && tMin <= 1 && 0 <= tMax && tMax <= 1;  // :60
}

// World::checkPointValidity — src/World.cpp:80-128.  The rtree query
// contains(point) == strict interior of the AABB.
template <bool MINDIST>
__device__ __forceinline__ bool point_valid(const Acc& a, const WorldView& w, double px, double py,
                                            double pz, bool can_pass, double md) {
    if (!(w.gx0 < px && px < w.gx1 && w.gy0 < py && py < w.gy1 && w.gz0 < pz && pz < w.gz1))
        return true;  // outside every AABB
    const int cx = cell_of(px, w.gx0, w.icx, w.nx);
    const int cy = cell_of(py, w.gy0, w.icy, w.ny);
    const int cz = cell_of(pz, w.gz0, w.icz, w.nz);
    const int cell = (cz * w.ny + cy) * w.nx + cx;
    const uint32_t b = a.cs[cell], e = a.cs[cell + 1];
    for (uint32_t k = b; k < e; ++k) {
        const int i = a.co[k];
        if (!(a.g(F_LOX, i) < px && px < a.g(F_HIX, i) && a.g(F_LOY, i) < py && py < a.g(F_HIY, i) &&
              a.g(F_LOZ, i) < pz && pz < a.g(F_HIZ, i)))
            continue;
        const uint32_t m = a.meta[i];
        if (MINDIST) {
            if (m & META_FILLING) continue;  // :116-119
            if (obb_point_hit(a, i, m, px, py, pz, md)) return false;
        } else {
            if ((m & META_FILLING) && can_pass) continue;  // :92-95
            if (obb_point_hit(a, i, m, px, py, pz, a.g(F_R, i))) return false;
        }
    }
    return true;
}

// World::checkRayValid — src/World.cpp:130-162.  rtree intersects(rayBox) == closed
// AABB overlap.  Every candidate is tested in exactly one cell (the first cell the
// OBB's and the ray's cell ranges share).
__device__ __forceinline__ bool ray_valid(const Acc& a, const WorldView& w, const double s[3],
                                          const double e[3], bool can_pass) {
    double lo[3], hi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        lo[k] = (e[k] < s[k]) ? e[k] : s[k];
        hi[k] = (s[k] < e[k]) ? e[k] : s[k];
    }
    if (hi[0] < w.gx0 || w.gx1 < lo[0] || hi[1] < w.gy0 || w.gy1 < lo[1] || hi[2] < w.gz0 ||
        w.gz1 < lo[2])
        return true;
    const int x0 = cell_of(lo[0], w.gx0, w.icx, w.nx), x1 = cell_of(hi[0], w.gx0, w.icx, w.nx);
    const int y0 = cell_of(lo[1], w.gy0, w.icy, w.ny), y1 = cell_of(hi[1], w.gy0, w.icy, w.ny);
    const int z0 = cell_of(lo[2], w.gz0, w.icz, w.nz), z1 = cell_of(hi[2], w.gz0, w.icz, w.nz);
    for (int z = z0; z <= z1; ++z)
        for (int y = y0; y <= y1; ++y)
            for (int x = x0; x <= x1; ++x) {
                const int cell = (z * w.ny + y) * w.nx + x;
                const uint32_t b = a.cs[cell], en = a.cs[cell + 1];
                for (uint32_t k = b; k < en; ++k) {
                    const int i = a.co[k];
                    const uint32_t m = a.meta[i];
                    const int ox = (m >> 8) & 255, oy = (m >> 16) & 255, oz = m >> 24;
                    if (x != (ox > x0 ? ox : x0) || y != (oy > y0 ? oy : y0) ||
                        z != (oz > z0 ? oz : z0))
                        continue;  // visited in an earlier cell
                    if (a.g(F_HIX, i) < lo[0] || hi[0] < a.g(F_LOX, i) || a.g(F_HIY, i) < lo[1] ||
                        hi[1] < a.g(F_LOY, i) || a.g(F_HIZ, i) < lo[2] || hi[2] < a.g(F_LOZ, i))
                        continue;
                    if ((m & META_FILLING) && can_pass) continue;  // :150-153
                    if (obb_ray_hit(a, i, m, s, e, a.g(F_R, i))) return false;
                }
            }
    return true;
}

// discrete32: x = s + (e - s) * (k/32), k = 1..32 (RealVectorStateSpace::interpolate)
__device__ __forceinline__ bool ray_valid_d32(const Acc& a, const WorldView& w, const double s[3],
                                              const double e[3], bool can_pass) {
    for (int k = 1; k <= 32; ++k) {
        const double t = (double)k / 32.0;
        const double px = s[0] + (e[0] - s[0]) * t;
        const double py = s[1] + (e[1] - s[1]) * t;
        const double pz = s[2] + (e[2] - s[2]) * t;
        if (!point_valid<false>(a, w, px, py, pz, can_pass, 0.0)) return false;
    }
    return true;
}

__device__ __forceinline__ const unsigned char* stage_world(const WorldView& w, unsigned char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(w.blob);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const uint32_t n16 = w.blob_bytes / 16;
    for (uint32_t o = threadIdx.x; o < n16; o += blockDim.x) dst[o] = src[o];
    __syncthreads();
    return lds;
}

// Loads 4 consecutive xyz triples (96 B) owned by this lane.
__device__ __forceinline__ void load4(const double* __restrict__ p, int64_t first, int64_t n,
                                      bool aligned, double v[12]) {
    if (aligned && first + 4 <= n) {
        const double2* q = reinterpret_cast<const double2*>(p + 3 * first);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double2 t = q[k];
            v[2 * k] = t.x;
            v[2 * k + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) v[k] = (first + k / 3 < n) ? p[3 * first + k] : 0.0;
    }
}

__device__ __forceinline__ void store4(uint8_t* __restrict__ out, int64_t first, int64_t n,
                                       const uint32_t f[4]) {
    if (first + 4 <= n && ((reinterpret_cast<uintptr_t>(out + first) & 3) == 0)) {
        *reinterpret_cast<uint32_t*>(out + first) = f[0] | (f[1] << 8) | (f[2] << 16) | (f[3] << 24);
    } else {
        for (int k = 0; k < 4; ++k)
            if (first + k < n) out[first + k] = (uint8_t)f[k];
    }
}

template <bool LDS, bool MINDIST>
__global__ __launch_bounds__(kBlock) void k_states(WorldView w, const double* __restrict__ xyz,
                                                   int64_t n, int can_pass, double md,
                                                   uint8_t* __restrict__ valid,
                                                   int32_t* __restrict__ compact_idx,
                                                   unsigned long long* __restrict__ n_valid,
                                                   int aligned) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const unsigned char* base = LDS ? stage_world(w, lds) : w.blob;
    const Acc a = make_acc(base, w);
    const int64_t groups = (n + 3) / 4;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    // wave-uniform trip count: every lane of a wave runs every iteration (ballot/shfl)
    for (int64_t g0 = (int64_t)blockIdx.x * kBlock; g0 < groups; g0 += stride) {
        const int64_t g = g0 + threadIdx.x;
        const int64_t first = 4 * g;
        uint32_t f[4] = {0, 0, 0, 0};
        if (g < groups) {
            double v[12];
            load4(xyz, first, n, aligned != 0, v);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (first + k < n)
                    f[k] = point_valid<MINDIST>(a, w, v[3 * k], v[3 * k + 1], v[3 * k + 2],
                                                can_pass != 0, md)
                               ? 1u
                               : 0u;
            store4(valid, first, n, f);
        }
        if (compact_idx) {  // wave-ballot compaction (uniform branch)
            const int lane = threadIdx.x & 63;
            const uint32_t cnt = f[0] + f[1] + f[2] + f[3];
            uint32_t incl = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = __shfl_up(incl, d, 64);
                if (lane >= d) incl += t;
            }
            const uint32_t total = __shfl(incl, 63, 64);
            unsigned long long wbase = 0;
            if (lane == 0 && total) wbase = atomicAdd(n_valid, (unsigned long long)total);
            wbase = __shfl(wbase, 0, 64);
            uint64_t pos = wbase + incl - cnt;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (f[k]) compact_idx[pos++] = (int32_t)(first + k);
        }
    }
}

template <bool LDS, int MODE>
__global__ __launch_bounds__(kBlock) void k_motions(WorldView w, const double* __restrict__ s1,
                                                    const double* __restrict__ s2, int64_t n,
                                                    int can_pass, uint8_t* __restrict__ valid,
                                                    int aligned) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const unsigned char* base = LDS ? stage_world(w, lds) : w.blob;
    const Acc a = make_acc(base, w);
    const int64_t groups = (n + 3) / 4;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += stride) {
        const int64_t first = 4 * g;
        double vs[12], ve[12];
        load4(s1, first, n, aligned != 0, vs);
        load4(s2, first, n, aligned != 0, ve);
        uint32_t f[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (first + k < n) {
                const double* s = vs + 3 * k;
                const double* e = ve + 3 * k;
                f[k] = (MODE == 0 ? ray_valid(a, w, s, e, can_pass != 0)
                                  : ray_valid_d32(a, w, s, e, can_pass != 0))
                           ? 1u
                           : 0u;
            }
        store4(valid, first, n, f);
    }
}

struct DevInfo {
    int cus = 256;
    bool init = false;
};
DevInfo g_dev[64];

int cu_count() {
    int d = 0;
    (void)hipGetDevice(&d);
    if (d < 0 || d >= 64) return 256;
    if (!g_dev[d].init) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && c > 0)
            g_dev[d].cus = c;
        g_dev[d].init = true;
    }
    return g_dev[d].cus;
}

int grid_for(int64_t groups, uint32_t lds_bytes) {
    const int64_t need = (groups + kBlock - 1) / kBlock;
    int per_cu = 8;
    if (lds_bytes > 0) per_cu = (int)std::max<uint32_t>(1u, std::min<uint32_t>(8u, (160u * 1024u) / lds_bytes));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
}

epp_status launch_error(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    return EPP_OK;
}

}  // namespace
}  // namespace epp

using namespace epp;

extern "C" {

epp_status epp_check_states(const epp_world* world, const double* xyz, int64_t n,
                            int32_t can_pass_gate, uint8_t* valid, int32_t* compact_idx,
                            int64_t* n_valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid)) || (compact_idx && !n_valid)) {
        set_error("epp_check_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const WorldView& w = world_view(world);
    const int aligned = (reinterpret_cast<uintptr_t>(xyz) & 15) == 0;
    const int64_t groups = (n + 3) / 4;
    const bool lds = w.blob_bytes <= kLdsBudget;
    const uint32_t shm = lds ? w.blob_bytes : 0;
    const int grid = grid_for(groups, shm);
    if (lds)
        hipLaunchKernelGGL((k_states<true, false>), dim3(grid), dim3(kBlock), shm, (hipStream_t)stream, w,
                           xyz, n, can_pass_gate, 0.0, valid, compact_idx,
                           reinterpret_cast<unsigned long long*>(n_valid), aligned);
    else
        hipLaunchKernelGGL((k_states<false, false>), dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, w,
                           xyz, n, can_pass_gate, 0.0, valid, compact_idx,
                           reinterpret_cast<unsigned long long*>(n_valid), aligned);
    return launch_error("epp_check_states");
}

epp_status epp_check_states_mindist(const epp_world* world, const double* xyz, int64_t n,
                                    double min_distance, uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid))) {
        set_error("epp_check_states_mindist: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const WorldView& w = world_view(world);
    const int aligned = (reinterpret_cast<uintptr_t>(xyz) & 15) == 0;
    const int64_t groups = (n + 3) / 4;
    const bool lds = w.blob_bytes <= kLdsBudget;
    const uint32_t shm = lds ? w.blob_bytes : 0;
    const int grid = grid_for(groups, shm);
    if (lds)
        hipLaunchKernelGGL((k_states<true, true>), dim3(grid), dim3(kBlock), shm, (hipStream_t)stream, w,
                           xyz, n, 0, min_distance, valid, nullptr, nullptr, aligned);
    else
        hipLaunchKernelGGL((k_states<false, true>), dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, w,
                           xyz, n, 0, min_distance, valid, nullptr, nullptr, aligned);
    return launch_error("epp_check_states_mindist");
}

epp_status epp_check_motions(const epp_world* world, const double* s1, const double* s2, int64_t n,
                             int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!s1 || !s2 || !valid)) || (mode != 0 && mode != 1)) {
        set_error("epp_check_motions: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const WorldView& w = world_view(world);
    const int aligned =
        ((reinterpret_cast<uintptr_t>(s1) | reinterpret_cast<uintptr_t>(s2)) & 15) == 0;
    const int64_t groups = (n + 3) / 4;
    const bool lds = w.blob_bytes <= kLdsBudget;
    const uint32_t shm = lds ? w.blob_bytes : 0;
    const int grid = grid_for(groups, shm);
    hipStream_t st = (hipStream_t)stream;
    if (lds) {
        if (mode == 0)
            hipLaunchKernelGGL((k_motions<true, 0>), dim3(grid), dim3(kBlock), shm, st, w, s1, s2, n,
                               can_pass_gate, valid, aligned);
        else
            hipLaunchKernelGGL((k_motions<true, 1>), dim3(grid), dim3(kBlock), shm, st, w, s1, s2, n,
                               can_pass_gate, valid, aligned);
    } else {
        if (mode == 0)
            hipLaunchKernelGGL((k_motions<false, 0>), dim3(grid), dim3(kBlock), 0, st, w, s1, s2, n,
                               can_pass_gate, valid, aligned);
        else
            hipLaunchKernelGGL((k_motions<false, 1>), dim3(grid), dim3(kBlock), 0, st, w, s1, s2, n,
                               can_pass_gate, valid, aligned);
    }
    return launch_error("epp_check_motions");
}

}  // extern "C"

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
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>

#include "epp_internal.h"

namespace epp {
const WorldView& world_view(const epp_world* w);
const WorldView* world_dview(const epp_world* w);

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kLdsBudget = 150 * 1024;

struct Acc {
    const double* f;
    int n_pad;
    const uint32_t* meta;
    const unsigned long long* mask;
    const uint32_t* cs;
    const uint16_t* co;
    __device__ __forceinline__ double g(int field, int i) const { return f[field * n_pad + i]; }
};

// `front` holds cell_mask + cell_start (LDS or HBM), `base` the whole blob.
__device__ __forceinline__ Acc make_acc(const unsigned char* front, const unsigned char* base,
                                        const WorldView& w) {
    Acc a;
    a.f = reinterpret_cast<const double*>(base + w.off_soa);
    a.n_pad = w.n_pad;
    a.meta = reinterpret_cast<const uint32_t*>(base + w.off_meta);
    a.mask = reinterpret_cast<const unsigned long long*>(front + w.off_cell_mask);
    a.cs = reinterpret_cast<const uint32_t*>(front + w.off_cell_start);
    a.co = reinterpret_cast<const uint16_t*>(base + w.off_cell_obb);
    return a;
}

__device__ __forceinline__ double owner_r(const WorldView& w, uint32_t m) {
    return (m & META_GATE) ? w.r_gate : w.r_obst;  // src/World.cpp:89-90
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

// Occupancy test of a state's fine sub-cell; returns the number of candidate OBBs (its
// coarse cell's list, starting at `start`), 0 if no AABB can contain the state.
// Branch-free: every lane reads the (clamped) cell, so the four states of a lane
// interleave and no exec-mask juggling is needed.
__device__ __forceinline__ uint32_t classify(const Acc& a, const WorldView& w, double px, double py,
                                             double pz, uint32_t& start) {
    const float fx = fine_coord(px, w.ofx, w.i4x);
    const float fy = fine_coord(py, w.ofy, w.i4y);
    const float fz = fine_coord(pz, w.ofz, w.i4z);
    // outside the union of the AABBs (conservative, see epp_internal.h); NaN -> outside
    const bool in = (fx >= 0.0f) & (fx <= w.limx) & (fy >= 0.0f) & (fy <= w.limy) & (fz >= 0.0f) &
                    (fz <= w.limz);
    const int ix = (int)fminf(fmaxf(fx, 0.0f), w.fmaxx);
    const int iy = (int)fminf(fmaxf(fy, 0.0f), w.fmaxy);
    const int iz = (int)fminf(fmaxf(fz, 0.0f), w.fmaxz);
    const int cell = ((iz >> 2) * w.ny + (iy >> 2)) * w.nx + (ix >> 2);
    const uint32_t bit = (uint32_t)((((iz & 3) << 2) + (iy & 3)) * 4 + (ix & 3));
    const unsigned long long m = a.mask[cell];
    const uint32_t word = (bit & 32u) ? (uint32_t)(m >> 32) : (uint32_t)m;
    const bool occ = in & (((word >> (bit & 31u)) & 1u) != 0u);
    const uint32_t s0 = a.cs[cell], s1 = a.cs[cell + 1];
    start = s0;
    return occ ? s1 - s0 : 0u;
}

// World::checkPointValidity — src/World.cpp:80-128.  The rtree query
// contains(point) == strict interior of the AABB.
template <bool MINDIST>
__device__ __forceinline__ bool point_valid(const Acc& a, const WorldView& w, double px, double py,
                                            double pz, bool can_pass, double md) {
    uint32_t b = 0;
    const uint32_t c = classify(a, w, px, py, pz, b);
    const uint32_t e = b + c;
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
            if (obb_point_hit(a, i, m, px, py, pz, owner_r(w, m))) return false;
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
    const int x0 = fine_index(fine_coord(lo[0], w.ofx, w.i4x), w.nx) >> 2;
    const int x1 = fine_index(fine_coord(hi[0], w.ofx, w.i4x), w.nx) >> 2;
    const int y0 = fine_index(fine_coord(lo[1], w.ofy, w.i4y), w.ny) >> 2;
    const int y1 = fine_index(fine_coord(hi[1], w.ofy, w.i4y), w.ny) >> 2;
    const int z0 = fine_index(fine_coord(lo[2], w.ofz, w.i4z), w.nz) >> 2;
    const int z1 = fine_index(fine_coord(hi[2], w.ofz, w.i4z), w.nz) >> 2;
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
                    if (obb_ray_hit(a, i, m, s, e, owner_r(w, m))) return false;
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

// Copies the first `bytes` of the blob into LDS (block-wide, ends with a barrier).
__device__ __forceinline__ const unsigned char* stage_world(const WorldView& w, unsigned char* lds,
                                                            uint32_t bytes) {
    const uint4* src = reinterpret_cast<const uint4*>(w.blob);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    const uint32_t n16 = bytes / 16;
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

// ---- k_states: wave-cooperative candidate testing ----------------------------------
// Phase 1 (per lane, 4 states): bounds + fine-mask test.  A state whose sub-cell is
// occupied owns a segment of (state, candidate OBB) pairs: its coarse cell's list.
// Phase 2 (per wave): the segments are compacted into LDS (wave prefix sums) and the 64
// lanes take one pair each (a binary search over the segment offsets finds the pair's
// state), setting per-state "hit" bits with LDS atomics.  Only ~6% of uniform samples
// have candidates; without this a wavefront would run its slowest lane's candidate loop
// for every state slot.
constexpr int kSegCap = 96;     // needy states a wave handles cooperatively per group
constexpr int kPairCap = 512;   // (state, candidate) pairs a wave handles cooperatively
struct WaveScratch {
    double xyz[kSegCap][3];        // coordinates of the needy states
    uint32_t seg_start[kSegCap];   // exclusive prefix of pair counts
    uint32_t seg_state[kSegCap];   // sid (8 bits) | first candidate entry << 8
    uint8_t head[kPairCap];        // segment index at its first pair, 0 elsewhere
    uint32_t bits[8];              // hit bits of the 256 states of the wave's group
};
constexpr uint32_t kScratchBytes = (kBlock / 64) * ((sizeof(WaveScratch) + 15) & ~15u);

__device__ __forceinline__ void wave_lds_sync() {
    // LDS operations of one wavefront complete in order; this only stops the compiler
    // from moving memory accesses across the point (no vmcnt drain: the prefetched
    // loads of the next group stay in flight).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-wide inclusive scans with DPP (GFX9 row_shr / row_bcast): six cross-lane
// adds, no LDS round trips.  Lanes without a source read `old` = identity.
__device__ __forceinline__ uint32_t dpp_incl_add(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t dpp_incl_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return x;
}
// Exclusive prefix sum over the wave and the wave total.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, int /*lane*/, uint32_t& total) {
    const uint32_t incl = dpp_incl_add(x);
    total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    return incl - x;
}

template <bool MINDIST>
__device__ __forceinline__ bool pair_hit_r(const Acc& a, double r_gate, double r_obst, int i, double px, double py,
                                           double pz, bool can_pass, double md) {
    if (!(a.g(F_LOX, i) < px && px < a.g(F_HIX, i) && a.g(F_LOY, i) < py && py < a.g(F_HIY, i) &&
          a.g(F_LOZ, i) < pz && pz < a.g(F_HIZ, i)))
        return false;  // rtree contains(point): strict  src/World.cpp:83
    const uint32_t m = a.meta[i];
    if (MINDIST) return !(m & META_FILLING) && obb_point_hit(a, i, m, px, py, pz, md);  // :116-125
    return !((m & META_FILLING) && can_pass) &&
           obb_point_hit(a, i, m, px, py, pz, (m & META_GATE) ? r_gate : r_obst);  // :89-100
}
template <bool MINDIST>
__device__ __forceinline__ bool pair_hit(const Acc& a, const WorldView& w, int i, double px, double py,
                                         double pz, bool can_pass, double md) {
    return pair_hit_r<MINDIST>(a, w.r_gate, w.r_obst, i, px, py, pz, can_pass, md);
}

// Candidate walk of one state by its own lane (tail states and overflow).
template <bool MINDIST>
__device__ __forceinline__ bool state_valid_scalar(const Acc& a, const WorldView& w, double px,
                                                   double py, double pz, bool can_pass, double md) {
    uint32_t st = 0;
    const uint32_t c = classify(a, w, px, py, pz, st);
    for (uint32_t j = 0; j < c; ++j)
        if (pair_hit<MINDIST>(a, w, a.co[st + j], px, py, pz, can_pass, md)) return false;
    return true;
}

// STAGE: 0 = world read from HBM/L2, 1 = front (masks, cell starts) in LDS, 2 = all in LDS
template <int STAGE, bool MINDIST, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void k_states(WorldView w, const double* __restrict__ xyz,
                                                   int64_t n, int can_pass, double md,
                                                   uint8_t* __restrict__ valid,
                                                   int32_t* __restrict__ compact_idx,
                                                   unsigned long long* __restrict__ n_valid,
                                                   uint32_t stage_bytes, unsigned long long* __restrict__ tl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63;
    // optional per-wave timeline (debug entry epp_dbg_states_timeline): s_memrealtime
    // (100 MHz, chip-wide) at entry, data arrival, after staging, after the groups
    const int gwave = (int)((blockIdx.x * kBlock + threadIdx.x) >> 6);
    auto mark = [&](int k) {
        if (tl) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tl[gwave * 8 + k] = t;
        }
    };
    mark(0);
    // full groups of 4 states; the (< 4) tail states are handled after the main loop
    const int64_t groups = n / 4;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    // Loads are unconditional (clamped to the last full group) so the compiler keeps
    // the next group's six loads in flight with a counted vmcnt.
    auto load = [&](int64_t grp, double (&dst)[12]) {
        grp = grp < groups ? grp : groups - 1;
        if (ALIGNED) {
            const double2* q = reinterpret_cast<const double2*>(xyz + 12 * grp);
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const double2 t = q[k];
                dst[2 * k] = t.x;
                dst[2 * k + 1] = t.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) dst[k] = xyz[12 * grp + k];
        }
    };
    int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double va[12], vb[12];
    if (groups > 0) load(g, va);  // first loads before the world staging
    if (tl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        mark(1);
    }
    WaveScratch* ws = reinterpret_cast<WaveScratch*>(lds + (threadIdx.x >> 6) * ((sizeof(WaveScratch) + 15) & ~15u));
    const unsigned char* staged = STAGE ? stage_world(w, lds + kScratchBytes, stage_bytes) : w.blob;
    const Acc a = make_acc(staged, STAGE == 2 ? staged : w.blob, w);
    mark(2);

    auto process = [&](int64_t gg, const double (&v)[12]) {
        const bool live = gg < groups;
        const int64_t first = 4 * gg;
        // phase 1
        uint32_t cst[4], cnt[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = classify(a, w, v[3 * k], v[3 * k + 1], v[3 * k + 2], cst[k]);
            cnt[k] = live ? c : 0u;
        }
        const uint32_t mine = cnt[0] + cnt[1] + cnt[2] + cnt[3];
        const uint32_t nseg = (cnt[0] > 0) + (cnt[1] > 0) + (cnt[2] > 0) + (cnt[3] > 0);
        uint32_t total, S;
        const uint32_t pexcl = wave_excl_scan(mine, lane, total);
        const uint32_t sexcl = wave_excl_scan(nseg, lane, S);
        uint32_t hits = 0;
        if (total && S <= (uint32_t)kSegCap && total <= (uint32_t)kPairCap) {
            // wave-uniform: cooperative pair testing.  Pair p belongs to the last segment
            // starting at or before p: heads are scattered to LDS and propagated with a
            // wave max-scan (carried across rounds), no search.
            if (lane < 8) ws->bits[lane] = 0;
            for (uint32_t p = lane; p < total; p += 64) ws->head[p] = 0;
            wave_lds_sync();
            uint32_t si = sexcl, pp = pexcl;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (cnt[k]) {
                    ws->seg_start[si] = pp;
                    ws->seg_state[si] = (uint32_t)(lane * 4 + k) | (cst[k] << 8);
                    ws->xyz[si][0] = v[3 * k];
                    ws->xyz[si][1] = v[3 * k + 1];
                    ws->xyz[si][2] = v[3 * k + 2];
                    ws->head[pp] = (uint8_t)si;
                    ++si;
                    pp += cnt[k];
                }
            wave_lds_sync();
            uint32_t carry = 0;
            for (uint32_t r = 0; r < total; r += 64) {  // wave-uniform rounds
                const uint32_t p = r + lane;
                const uint32_t hd = p < total ? (uint32_t)ws->head[p] : 0u;
                const uint32_t j = max(dpp_incl_max(hd), carry);
                carry = (uint32_t)__builtin_amdgcn_readlane((int)j, 63);
                if (p < total) {
                    const uint32_t e = ws->seg_state[j];
                    const int i = a.co[(e >> 8) + (p - ws->seg_start[j])];
                    if (pair_hit<MINDIST>(a, w, i, ws->xyz[j][0], ws->xyz[j][1], ws->xyz[j][2],
                                          can_pass != 0, md)) {
                        const uint32_t sid = e & 255u;
                        atomicOr(&ws->bits[sid >> 5], 1u << (sid & 31));
                    }
                }
            }
            wave_lds_sync();
            hits = (ws->bits[lane >> 3] >> ((lane & 7) * 4)) & 15u;
            wave_lds_sync();  // scratch is rewritten by the next group
        } else if (total) {  // rare: too many needy states, every lane walks its own lists
#pragma unroll
            for (int k = 0; k < 4; ++k)
                for (uint32_t j = 0; j < cnt[k]; ++j)
                    if (pair_hit<MINDIST>(a, w, a.co[cst[k] + j], v[3 * k], v[3 * k + 1], v[3 * k + 2],
                                          can_pass != 0, md)) {
                        hits |= 1u << k;
                        break;
                    }
        }
        const uint32_t fl = live ? (~hits & 15u) : 0u;  // bit k: state first+k valid
        if (live) {
            if (ALIGNED)
                *reinterpret_cast<uint32_t*>(valid + first) =
                    (fl & 1u) | ((fl & 2u) << 7) | ((fl & 4u) << 14) | ((fl & 8u) << 21);
            else
                for (int k = 0; k < 4; ++k) valid[first + k] = (uint8_t)((fl >> k) & 1u);
        }
        if (compact_idx) {  // wave-ballot compaction (uniform branch)
            const uint32_t c = (uint32_t)__popc(fl);
            uint32_t ctot;
            const uint32_t cex = wave_excl_scan(c, lane, ctot);
            unsigned long long wbase = 0;
            if (lane == 0 && ctot) wbase = atomicAdd(n_valid, (unsigned long long)ctot);
            wbase = __shfl(wbase, 0, 64);
            uint64_t pos = wbase + cex;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((fl >> k) & 1u) compact_idx[pos++] = (int32_t)(first + k);
        }
    };
    // block-uniform trip count: every lane runs every iteration (ballots, wave scratch);
    // ping-pong register buffers: the next group loads while this one is processed
    for (int64_t g0 = (int64_t)blockIdx.x * kBlock; g0 < groups; g0 += 2 * stride, g += 2 * stride) {
        load(g + stride, vb);
        process(g, va);
        if (g0 + stride >= groups) break;
        load(g + 2 * stride, va);
        process(g + stride, vb);
    }
    mark(3);
    if (tl && lane == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        tl[gwave * 8 + 4] = hw;
        tl[gwave * 8 + 5] = xcc;
        tl[gwave * 8 + 6] = __builtin_amdgcn_s_memtime();
    }
    // tail: the last n % 4 states, one lane each
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - 4 * groups)) {
        const int64_t i = 4 * groups + threadIdx.x;
        const bool ok = state_valid_scalar<MINDIST>(a, w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2],
                                                    can_pass != 0, md);
        valid[i] = ok ? 1 : 0;
        if (compact_idx && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

// ---- k_states_bm: flat-bitmap fast path ----------------------------------------------
// Per state: three float cell coordinates and ONE bitmap word (global, L1/L2 resident);
// a clear bit proves the state lies outside every inflated AABB (valid, no OBB test).
// The few states on set bits are compacted per wave (ballots) into an LDS queue; one
// lane per queued state walks its coarse-cell candidate list with the exact fp64
// rtree-prefilter + OBB tests, and the hit flags are read back from LDS.
constexpr int kQueueCap = 256;  // a wave's whole group (64 lanes x 4 states)
struct StateQueue {
    double xyz[kQueueCap][3];
    uint32_t cls[kQueueCap];
    uint8_t hit[kQueueCap];
};

// Fast-path parameters of the bitmap (kept in SGPRs; the rest of the WorldView is read
// through the scalar cache only on the rare exact path).
typedef const __attribute__((address_space(1))) uint16_t* gptr_u16;  // global, not flat

struct BmParams {
    gptr_u16 cls;
    float ox, oy, oz, ix, iy, iz;
    uint32_t nx, ny, nz, sentinel;
};

// index of the fine cell of p in cls[] (the zero sentinel when p is outside the grid)
__device__ __forceinline__ uint32_t cls_index(const BmParams& p, double px, double py, double pz) {
    const int ix = bm_axis(px, p.ox, p.ix), iy = bm_axis(py, p.oy, p.iy), iz = bm_axis(pz, p.oz, p.iz);
    const bool in = (unsigned)ix < p.nx && (unsigned)iy < p.ny && (unsigned)iz < p.nz;
    // dims <= 4096 per axis, so the products fit 24-bit multiplies
    const uint32_t c = __umul24(__umul24((uint32_t)iz, p.ny) + (uint32_t)iy, p.nx) + (uint32_t)ix;
    return in ? c : p.sentinel;
}

// Exact test of one queued state: rtree prefilter + OBB tests on its coarse-cell list.
// The WorldView pointer is laundered through an empty asm so the compiler cannot hoist
// the field loads into the streaming loop: the rare path reads them through the scalar
// cache instead of pinning ~50 SGPRs for the whole kernel.
// `base` is the blob: its LDS copy (STAGE) or the HBM original.  `cls` is the state's
// fine-cell class: the first chunk of its candidate list.
template <bool MINDIST>
__device__ __forceinline__ bool states_exact_hit(const WorldView* wvp, const unsigned char* base, double px,
                                                 double py, double pz, uint32_t cls, int can_pass, double md) {
    // constant address space: the fields come in by scalar loads (lgkmcnt), not flat
    // loads that would also wait for the in-flight prefetch
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass only parses device bodies)
    typedef const __attribute__((address_space(4))) WorldView* cwv_ptr;
    cwv_ptr p = (cwv_ptr)wvp;
    asm volatile("" : "+s"(p));
#else
    const WorldView* p = wvp;
#endif
    // list path: only the few fields it needs (keeps SGPR pressure low)
    Acc a;
    a.f = reinterpret_cast<const double*>(base + p->off_soa);
    a.n_pad = p->n_pad;
    a.meta = reinterpret_cast<const uint32_t*>(base + p->off_meta);
    const double rg = p->r_gate, ro = p->r_obst;
    const uint32_t hd = reinterpret_cast<const uint32_t*>(base + p->off_lists)[cls];
    const uint16_t* ids = reinterpret_cast<const uint16_t*>(base + p->off_ids) + (hd >> 12);
    const uint32_t cnt = hd & 4095u;
    for (uint32_t j = 0; j < cnt; ++j)
        if (pair_hit_r<MINDIST>(a, rg, ro, ids[j], px, py, pz, can_pass != 0, md)) return true;
    return false;
}

// Same predicate as pair_hit_r on one AoS record (rec: kRecDoubles doubles), written
// branch-free: all fields are read up front (one LDS round trip instead of a
// short-circuit chain of dependent read -> compare -> branch steps) and the outcome is
// a conjunction of the same fp64 comparisons, so the booleans are unchanged.
template <bool MINDIST>
__device__ __forceinline__ bool rec_hit(const double* rec, double rg, double ro, double px, double py, double pz,
                                        bool can_pass, double md) {
    double f[kRecDoubles];
#pragma unroll
    for (int k = 0; k <= F_HZ; ++k) f[k] = rec[k];
    f[R_META] = rec[R_META];  // (the two padding doubles are not read)
    const uint32_t m = (uint32_t)__double_as_longlong(f[R_META]);
    // rtree contains(point): strict  src/World.cpp:83
    const bool in = (f[F_LOX] < px) & (px < f[F_HIX]) & (f[F_LOY] < py) & (py < f[F_HIY]) & (f[F_LOZ] < pz) &
                    (pz < f[F_HIZ]);
    const bool fill = (m & META_FILLING) != 0u;
    // MINDIST skips every filling OBB (:116-118), else only with canPassGate (:92-95)
    const bool skip = MINDIST ? fill : (fill & can_pass);
    const double r = MINDIST ? md : ((m & META_GATE) ? rg : ro);  // :89-90
    // OBB::checkCollisionWithPoint — src/OBB.cpp:63-91 (same evaluation as obb_point_hit)
    const double c = f[F_COS], s = f[F_SIN];
    const double dx = px - f[F_CX], dy = py - f[F_CY], dz = pz - f[F_CZ];
    const double lx = c * dx + s * dy;
    const double ly = c * dy - s * dx;
    const double ix = f[F_HX] + r, iy = f[F_HY] + r, iz = f[F_HZ] + r;  // shouldBeInflated()
    const double tx = fill ? f[F_HX] : ix, ty = fill ? f[F_HY] : iy, tz = fill ? f[F_HZ] : iz;
    return in & !skip & (fabs(lx) <= tx) & (fabs(ly) <= ty) & (fabs(dz) <= tz);
}

// Exact test on the AoS records + the cell's candidate list (no early exit: the lists
// are short and straight-line control flow keeps the wave converged).  `sbase` points
// at the records (LDS copy or HBM); `lists_off` / `ids_off` are relative to it.
template <bool MINDIST>
__device__ __forceinline__ bool states_exact_rec(const unsigned char* sbase, uint32_t lists_off, uint32_t ids_off,
                                                 double rg, double ro, double px, double py, double pz, uint32_t cls,
                                                 int can_pass, double md) {
    const double* recs = reinterpret_cast<const double*>(sbase);
    const uint32_t h = reinterpret_cast<const uint32_t*>(sbase + lists_off)[cls];
    const uint16_t* ids = reinterpret_cast<const uint16_t*>(sbase + ids_off) + (h >> 12);
    const uint32_t cnt = h & 4095u;
    bool hit = false;
    for (uint32_t j = 0; j < cnt; ++j)
        hit |= rec_hit<MINDIST>(recs + (size_t)ids[j] * kRecDoubles, rg, ro, px, py, pz, can_pass != 0, md);
    return hit;
}

// STAGE: the blob up to the bitmap (cull grid, lists, OBB table) is copied into LDS once
// per workgroup, so the exact path runs on LDS reads (lgkmcnt) and never waits behind
// the in-flight prefetch of the next group (vmcnt counts in order).
template <bool MINDIST, bool ALIGNED, bool STAGE>
__global__ __launch_bounds__(kBlock) void k_states_bm(const WorldView* __restrict__ wv, const double* __restrict__ xyz,
                                                      int64_t n, int can_pass, double md,
                                                      uint8_t* __restrict__ valid,
                                                      int32_t* __restrict__ compact_idx,
                                                      unsigned long long* __restrict__ n_valid,
                                                      unsigned long long* __restrict__ tl, uint32_t stage_bytes) {
    __shared__ StateQueue queues[kBlock / 64];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_blob[];
    const int lane = threadIdx.x & 63;
    StateQueue* qu = &queues[threadIdx.x >> 6];
    const int gwave = (int)((blockIdx.x * kBlock + threadIdx.x) >> 6);
    auto mark = [&](int k) {
        if (tl) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tl[gwave * 8 + k] = t;
        }
    };
    mark(0);
    BmParams bp;
    bp.cls = (gptr_u16)(wv->blob + wv->off_bitmap);
    bp.ox = wv->bofx; bp.oy = wv->bofy; bp.oz = wv->bofz;
    bp.ix = wv->bix; bp.iy = wv->biy; bp.iz = wv->biz;
    bp.nx = (uint32_t)wv->bnx; bp.ny = (uint32_t)wv->bny; bp.nz = (uint32_t)wv->bnz;
    bp.sentinel = wv->bm_words;
    const unsigned char* xbase = nullptr;
    uint32_t total_needy_dbg = 0;  // blob for the exact path: LDS copy or HBM (set below)
    const int64_t groups = n / 4;  // full groups of 4; the n % 4 tail states come last
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    auto load = [&](int64_t grp, double (&dst)[12]) {
        grp = grp < groups ? grp : groups - 1;  // unconditional (clamped): no branch, counted vmcnt
        if (ALIGNED) {
            const double2* q = reinterpret_cast<const double2*>(xyz + 12 * grp);
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const double2 t = q[k];
                dst[2 * k] = t.x;
                dst[2 * k + 1] = t.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 12; ++k) dst[k] = xyz[12 * grp + k];
        }
    };
    // the current group's four cell classes are requested BEFORE the next group's
    // prefetch, so waiting for them (vmcnt counts in order) leaves the prefetch in flight
    auto words = [&](const double (&v)[12], uint32_t (&wd)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) wd[k] = bp.cls[cls_index(bp, v[3 * k], v[3 * k + 1], v[3 * k + 2])];
    };
    auto finish = [&](int64_t gg, const double (&v)[12], const uint32_t (&wd)[4]) {
        const int64_t first = 4 * gg;
        const bool live = gg < groups;
        bool needy[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) needy[k] = live & (wd[k] != 0u);
        unsigned long long bal[4];
        uint32_t total = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bal[k] = __ballot(needy[k]);
            total += (uint32_t)__popcll(bal[k]);
        }
        mark(4);
        total_needy_dbg += total;
        uint32_t hits = 0;
        if (total > 0) {  // wave-uniform: queue the needy states, one lane per state
            uint32_t pos[4];
            uint32_t base = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                pos[k] = base + lanes_below(bal[k]);
                base += (uint32_t)__popcll(bal[k]);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (needy[k]) {
                    qu->xyz[pos[k]][0] = v[3 * k];
                    qu->xyz[pos[k]][1] = v[3 * k + 1];
                    qu->xyz[pos[k]][2] = v[3 * k + 2];
                    qu->cls[pos[k]] = wd[k];
                }
            wave_lds_sync();
            for (uint32_t e = lane; e < total; e += 64)  // rounds of 64 (almost always one)
                qu->hit[e] = states_exact_hit<MINDIST>(wv, xbase, qu->xyz[e][0], qu->xyz[e][1], qu->xyz[e][2],
                                                       qu->cls[e], can_pass, md)
                                 ? 1
                                 : 0;
            wave_lds_sync();
            mark(5);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (needy[k] && qu->hit[pos[k]]) hits |= 1u << k;
            wave_lds_sync();  // the queue is rewritten by the next group
        }
        const uint32_t fl = live ? (~hits & 15u) : 0u;  // bit k: state first+k valid
        if (live) {
            if (ALIGNED)
                *reinterpret_cast<uint32_t*>(valid + first) =
                    (fl & 1u) | ((fl & 2u) << 7) | ((fl & 4u) << 14) | ((fl & 8u) << 21);
            else
                for (int k = 0; k < 4; ++k) valid[first + k] = (uint8_t)((fl >> k) & 1u);
        }
        if (compact_idx) {  // wave-ballot compaction (uniform branch)
            const uint32_t c = (uint32_t)__popc(fl);
            uint32_t ctot;
            const uint32_t cex = wave_excl_scan(c, lane, ctot);
            unsigned long long wbase = 0;
            if (lane == 0 && ctot) wbase = atomicAdd(n_valid, (unsigned long long)ctot);
            wbase = __shfl(wbase, 0, 64);
            uint64_t p = wbase + cex;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((fl >> k) & 1u) compact_idx[p++] = (int32_t)(first + k);
        }
    };
    int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double va[12], vb[12];
    uint32_t wd[4];
    if (groups > 0) load(g, va);
    if (tl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        mark(1);
    }
    if (STAGE) {
        const uint4* src = reinterpret_cast<const uint4*>(wv->blob);
        uint4* dst = reinterpret_cast<uint4*>(lds_blob);
        for (uint32_t o = threadIdx.x; o < stage_bytes / 16; o += kBlock) dst[o] = src[o];
        __syncthreads();
        xbase = lds_blob;
    } else {
        xbase = wv->blob;
    }
    mark(2);
    // block-uniform trip count: every lane runs every iteration (ballots, wave queue)
    for (int64_t g0 = (int64_t)blockIdx.x * kBlock; g0 < groups; g0 += 2 * stride, g += 2 * stride) {
        words(va, wd);
        load(g + stride, vb);
        finish(g, va, wd);
        if (g0 + stride >= groups) break;
        words(vb, wd);
        load(g + 2 * stride, va);
        finish(g + stride, vb, wd);
    }
    mark(3);
    if (tl && lane == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        tl[gwave * 8 + 6] = hw;
        tl[gwave * 8 + 7] = xcc | ((unsigned long long)total_needy_dbg << 32);
    }
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - 4 * groups)) {  // tail: the last n % 4 states
        const int64_t i = 4 * groups + threadIdx.x;
        const double px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
        const uint32_t c = bp.cls[cls_index(bp, px, py, pz)];
        const bool ok = !(c != 0u && states_exact_hit<MINDIST>(wv, xbase, px, py, pz, c, can_pass, md));
        valid[i] = ok ? 1 : 0;
        if (compact_idx && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

// ---- k_states_v3: occupancy instead of software prefetch --------------------------
// 512-thread workgroups, <= 64 VGPRs (8 waves per SIMD), two states per lane (48 B, three
// 16-B loads) and no double buffer: at 1M states every wave of the chip holds exactly one
// item and the latency chains (state load -> cell class -> LDS candidate tests) of 32
// waves per CU overlap.  Same fast path / queue / exact path as k_states_bm.
constexpr int kBlock3 = 512;
constexpr int kQueue3 = 128;  // a wave's item: 64 lanes x 2 states
struct StateQueue3 {
    double xyz[kQueue3][3];
    uint16_t cls[kQueue3];
    uint8_t hit[kQueue3];
};

// COMPACT: also append the valid indices; TL: per-wave timeline (debug entry only)
template <bool MINDIST, bool STAGE, bool COMPACT, bool TL>
__global__ __launch_bounds__(kBlock3) void k_states_v3(const WorldView* __restrict__ wv,
                                                          const double* __restrict__ xyz, int64_t n, int can_pass,
                                                          double md, uint8_t* __restrict__ valid,
                                                          int32_t* __restrict__ compact_idx,
                                                          unsigned long long* __restrict__ n_valid,
                                                          unsigned long long* __restrict__ tl, uint32_t stage_bytes) {
    __shared__ StateQueue3 queues[kBlock3 / 64];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_blob[];
    const int lane = threadIdx.x & 63;
    StateQueue3* qu = &queues[threadIdx.x >> 6];
    const int gwave = (int)((blockIdx.x * kBlock3 + threadIdx.x) >> 6);
    auto mark = [&](int k) {
        if (TL) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tl[gwave * 8 + k] = t;
        }
    };
    mark(0);
    BmParams bp;
    bp.cls = (gptr_u16)(wv->blob + wv->off_bitmap);
    bp.ox = wv->bofx; bp.oy = wv->bofy; bp.oz = wv->bofz;
    bp.ix = wv->bix; bp.iy = wv->biy; bp.iz = wv->biz;
    bp.nx = (uint32_t)wv->bnx; bp.ny = (uint32_t)wv->bny; bp.nz = (uint32_t)wv->bnz;
    bp.sentinel = wv->bm_words;
    const int64_t items = n / 2;  // pairs of states; an odd last state comes after the loop
    const int64_t stride = (int64_t)gridDim.x * kBlock3;
    int64_t it = (int64_t)blockIdx.x * kBlock3 + threadIdx.x;
    double v[6];
    auto load = [&](int64_t i) {
        i = i < items ? i : items - 1;
        const double2* q = reinterpret_cast<const double2*>(xyz + 6 * i);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double2 t = q[k];
            v[2 * k] = t.x;
            v[2 * k + 1] = t.y;
        }
    };
    if (items > 0) load(it);
    // records + lists: [off_aos, off_bitmap) of the blob, staged into LDS
    const uint32_t lists_off = wv->off_lists - wv->off_aos, ids_off = wv->off_ids - wv->off_aos;
    const double rg = wv->r_gate, ro = wv->r_obst;
    const unsigned char* xbase;
    if (STAGE) {
        const uint4* src = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds_blob);
        for (uint32_t o = threadIdx.x; o < stage_bytes / 16; o += kBlock3) dst[o] = src[o];
        __syncthreads();
        xbase = lds_blob;
    } else {
        xbase = wv->blob + wv->off_aos;
    }
    mark(2);
    uint32_t total_needy_dbg = 0;
    // block-uniform trip count: every lane runs every iteration (ballots, wave queue)
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock3; i0 < items; i0 += stride, it += stride) {
        if (i0 != (int64_t)blockIdx.x * kBlock3) load(it);
        const bool live = it < items;
        const uint32_t c0 = bp.cls[cls_index(bp, v[0], v[1], v[2])];
        const uint32_t c1 = bp.cls[cls_index(bp, v[3], v[4], v[5])];
        const bool n0 = live & (c0 != 0u), n1 = live & (c1 != 0u);
        const unsigned long long b0 = __ballot(n0), b1 = __ballot(n1);
        const uint32_t t0 = (uint32_t)__popcll(b0), total = t0 + (uint32_t)__popcll(b1);
        mark(4);
        if (TL) total_needy_dbg += total;
        uint32_t hits = 0;
        if (total > 0) {  // wave-uniform
            const uint32_t p0 = lanes_below(b0), p1 = t0 + lanes_below(b1);
            if (n0) {
                qu->xyz[p0][0] = v[0];
                qu->xyz[p0][1] = v[1];
                qu->xyz[p0][2] = v[2];
                qu->cls[p0] = (uint16_t)c0;
            }
            if (n1) {
                qu->xyz[p1][0] = v[3];
                qu->xyz[p1][1] = v[4];
                qu->xyz[p1][2] = v[5];
                qu->cls[p1] = (uint16_t)c1;
            }
            wave_lds_sync();
            for (uint32_t e = lane; e < total; e += 64)
                qu->hit[e] = states_exact_rec<MINDIST>(xbase, lists_off, ids_off, rg, ro, qu->xyz[e][0], qu->xyz[e][1],
                                                       qu->xyz[e][2], qu->cls[e], can_pass, md)
                                 ? 1
                                 : 0;
            wave_lds_sync();
            mark(5);
            hits = (n0 && qu->hit[p0] ? 1u : 0u) | (n1 && qu->hit[p1] ? 2u : 0u);
            wave_lds_sync();  // the queue is rewritten next
        }
        const uint32_t fl = live ? (~hits & 3u) : 0u;
        if (live) *reinterpret_cast<uint16_t*>(valid + 2 * it) = (uint16_t)((fl & 1u) | ((fl & 2u) << 7));
        if (COMPACT) {  // wave-ballot compaction
            const uint32_t c = (uint32_t)__popc(fl);
            uint32_t ctot;
            const uint32_t cex = wave_excl_scan(c, lane, ctot);
            unsigned long long wbase = 0;
            if (lane == 0 && ctot) wbase = atomicAdd(n_valid, (unsigned long long)ctot);
            wbase = __shfl(wbase, 0, 64);
            uint64_t p = wbase + cex;
            if (fl & 1u) compact_idx[p++] = (int32_t)(2 * it);
            if (fl & 2u) compact_idx[p] = (int32_t)(2 * it + 1);
        }
    }
    mark(3);
    if (TL && lane == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        tl[gwave * 8 + 6] = hw;
        tl[gwave * 8 + 7] = xcc | ((unsigned long long)total_needy_dbg << 32);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {  // odd last state
        const int64_t i = n - 1;
        const double px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
        const uint32_t c = bp.cls[cls_index(bp, px, py, pz)];
        const bool ok = !(c != 0u && states_exact_rec<MINDIST>(xbase, lists_off, ids_off, rg, ro, px, py, pz, c, can_pass, md));
        valid[i] = ok ? 1 : 0;
        if (COMPACT && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

// ---- k_states_v4: workgroup-wide queue of the exact tests -------------------------
// As k_states_v3 (512 threads, two states per lane, high occupancy), but the states on
// occupied cells of the whole workgroup (~9% of 1024) are gathered into ONE LDS queue
// and tested by the first ceil(T/64) waves only, so the exact path runs on full
// wavefronts instead of ~10 active lanes in each of 8 waves.  Three barriers per item.
constexpr int kBlock4 = 512;
constexpr int kQueue4 = 2 * kBlock4;
struct StateQueue4 {
    double x[kQueue4], y[kQueue4], z[kQueue4];
    uint16_t cls[kQueue4];
    uint8_t hit[kQueue4];
    uint32_t wcnt[kBlock4 / 64];
};

// Block-wide copy of `bytes` (16-byte multiple) HBM -> LDS with global (not flat) loads,
// so waiting for the copy never waits on LDS traffic or vice versa.  No barrier.
__device__ __forceinline__ void stage_copy(unsigned char* dst, const unsigned char* src, uint32_t bytes,
                                           uint32_t nthreads) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(1))) uint4* gptr_u4;
    const gptr_u4 s = (gptr_u4)src;
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (uint32_t o = threadIdx.x; o < bytes / 16; o += nthreads) d[o] = s[o];
#endif
}

template <bool MINDIST, bool STAGE, bool COMPACT>
__global__ __launch_bounds__(kBlock4) void k_states_v4(const WorldView* __restrict__ wv,
                                                       const double* __restrict__ xyz, uint32_t items,
                                                       int64_t n, int can_pass, double md,
                                                       uint8_t* __restrict__ valid,
                                                       int32_t* __restrict__ compact_idx,
                                                       unsigned long long* __restrict__ n_valid,
                                                       uint32_t stage_bytes) {
    __shared__ StateQueue4 q;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_blob[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
    BmParams bp;
    bp.cls = (gptr_u16)(wv->blob + wv->off_bitmap);
    bp.ox = wv->bofx; bp.oy = wv->bofy; bp.oz = wv->bofz;
    bp.ix = wv->bix; bp.iy = wv->biy; bp.iz = wv->biz;
    bp.nx = (uint32_t)wv->bnx; bp.ny = (uint32_t)wv->bny; bp.nz = (uint32_t)wv->bnz;
    bp.sentinel = wv->bm_words;
    const uint32_t stride = gridDim.x * kBlock4;
    uint32_t it = blockIdx.x * kBlock4 + threadIdx.x;
    double v[6];
    auto load = [&](uint32_t i) {
        i = i < items ? i : items - 1;
        const double2* p = reinterpret_cast<const double2*>(xyz) + 3 * (size_t)i;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double2 t = p[k];
            v[2 * k] = t.x;
            v[2 * k + 1] = t.y;
        }
    };
    if (items > 0) load(it);
    // records + lists: [off_aos, off_bitmap) of the blob, staged into LDS
    const uint32_t lists_off = wv->off_lists - wv->off_aos, ids_off = wv->off_ids - wv->off_aos;
    const double rg = wv->r_gate, ro = wv->r_obst;
    const unsigned char* xbase;
    if (STAGE) {
        stage_copy(lds_blob, wv->blob + wv->off_aos, stage_bytes, kBlock4);
        xbase = lds_blob;  // (the first barrier below orders the copy before any use)
    } else {
        xbase = wv->blob + wv->off_aos;
    }
    // block-uniform trip count: every thread runs every iteration (barriers)
    for (uint32_t i0 = blockIdx.x * kBlock4; i0 < items; i0 += stride, it += stride) {
        if (i0 != blockIdx.x * kBlock4) load(it);
        const bool live = it < items;
        const uint32_t c0 = bp.cls[cls_index(bp, v[0], v[1], v[2])];
        const uint32_t c1 = bp.cls[cls_index(bp, v[3], v[4], v[5])];
        const bool n0 = live & (c0 != 0u), n1 = live & (c1 != 0u);
        const unsigned long long b0 = __ballot(n0), b1 = __ballot(n1);
        const uint32_t t0 = (uint32_t)__popcll(b0), tw = t0 + (uint32_t)__popcll(b1);
        if (lane == 0) q.wcnt[wave] = tw;
        __syncthreads();
        // wave offset and block total (scalar loops over the 8 counters: no per-wave masks)
        uint32_t off = 0, T = 0;
        for (int w = 0; w < wave; ++w) off += q.wcnt[w];
        T = off;
        for (int w = wave; w < kBlock4 / 64; ++w) T += q.wcnt[w];
        uint32_t hits = 0;
        if (T > 0) {  // block-uniform
            const uint32_t p0 = off + lanes_below(b0), p1 = off + t0 + lanes_below(b1);
            if (n0) {
                q.x[p0] = v[0];
                q.y[p0] = v[1];
                q.z[p0] = v[2];
                q.cls[p0] = (uint16_t)c0;
            }
            if (n1) {
                q.x[p1] = v[3];
                q.y[p1] = v[4];
                q.z[p1] = v[5];
                q.cls[p1] = (uint16_t)c1;
            }
            __syncthreads();
            for (uint32_t e = threadIdx.x; e < T; e += kBlock4)  // only the first ceil(T/64) waves
                q.hit[e] = states_exact_rec<MINDIST>(xbase, lists_off, ids_off, rg, ro, q.x[e], q.y[e], q.z[e], q.cls[e],
                                                     can_pass, md)
                               ? 1
                               : 0;
            __syncthreads();
            hits = (n0 && q.hit[p0] ? 1u : 0u) | (n1 && q.hit[p1] ? 2u : 0u);
        }
        const uint32_t fl = live ? (~hits & 3u) : 0u;
        if (live) *reinterpret_cast<uint16_t*>(valid + 2 * (size_t)it) = (uint16_t)((fl & 1u) | ((fl & 2u) << 7));
        if (COMPACT) {  // wave-ballot compaction
            const uint32_t c = (uint32_t)__popc(fl);
            uint32_t ctot;
            const uint32_t cex = wave_excl_scan(c, lane, ctot);
            unsigned long long wbase = 0;
            if (lane == 0 && ctot) wbase = atomicAdd(n_valid, (unsigned long long)ctot);
            wbase = __shfl(wbase, 0, 64);
            uint64_t p = wbase + cex;
            if (fl & 1u) compact_idx[p++] = (int32_t)(2 * (size_t)it);
            if (fl & 2u) compact_idx[p] = (int32_t)(2 * (size_t)it + 1);
        }
    }
    if (STAGE && items == 0) __syncthreads();  // (no loop ran: nothing read the copy)
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {  // odd last state
        const int64_t i = n - 1;
        const double px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
        const uint32_t c = bp.cls[cls_index(bp, px, py, pz)];
        const bool ok = !(c != 0u && states_exact_rec<MINDIST>(xbase, lists_off, ids_off, rg, ro, px, py, pz, c, can_pass, md));
        valid[i] = ok ? 1 : 0;
        if (COMPACT && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

// ---- k_states_v5: the whole decision runs out of LDS ------------------------------
// Persistent workgroups (one per CU), four states per lane (96 B = six 16-B loads),
// the next group prefetched while the current one is classified.  The world's
// records, candidate lists and fine-cell class table are staged into LDS once per
// workgroup while the first group's HBM loads are in flight.  Per state: class lookup
// (LDS, ~15 VALU: the class grid's empty margin cells make a clamp do the bounds test)
// -> ballot; a group with needy states queues them in the wave's LDS queue and, in the
// common case (<= 64 needy states and <= 64 candidate pairs), tests each (state,
// candidate) pair on its own lane with the hits returned by one ballot; otherwise each
// queued state walks its own list.  One 32-bit store writes a lane's four flags.
// The per-state VALU count matters: at 1M states/launch the kernel's critical path is
// the last-arriving data plus the VALU work behind it (PMC: SQ_INSTS_VALU).
struct WaveQueue5 {
    double x[64], y[64], z[64];
    uint32_t pair[128];  // segment heads of the (state, candidate) pairs
    uint16_t cls[64];
    uint8_t hit[64];
};
template <int BLOCK>
constexpr uint32_t queue5_bytes() { return (BLOCK / 64) * sizeof(WaveQueue5); }

// hardware f32 -> i32 conversion (NaN -> 0, saturating), then clamp to [0, n-1]
__device__ __forceinline__ uint32_t cell_axis5(double p, float off, float inv, uint32_t nm1) {
    const float f = fmaf((float)p, inv, off);
    int i;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(i) : "v"(f));
    return min((uint32_t)i, nm1);  // negative -> huge -> last (empty) cell
}

// TL: per-wave timeline (debug entry only; 8 u64 per wave: entry, data + staging
// arrived, -, end, first group classified, first group's exact path done, HW_ID,
// XCC_ID | needy states << 32)
// PREFETCH: groups per lane > 1 (the next group's loads overlap this one's work);
// single-pass launches (e.g. 1M states on 256 CUs) drop the second buffer's registers.
// SPL: states per lane and group (4: 96 B = six 16-B loads, 8: 192 B = twelve); one
// flag store of SPL bytes.  More states per lane = fewer waves, i.e. fewer executions
// of the per-wave fixed costs (setup, staging, the exact path).
template <bool MINDIST, bool COMPACT, bool TL, int BLOCK, bool PREFETCH, int SPL>
__global__ __launch_bounds__(BLOCK) void k_states_v5(const WorldView* __restrict__ wv,
                                                     const double* xyz, int64_t groups, int64_t n,
                                                     int can_pass, double md, uint8_t* __restrict__ valid,
                                                     int32_t* __restrict__ compact_idx,
                                                     unsigned long long* __restrict__ n_valid, uint32_t stage_bytes,
                                                     int fast, unsigned long long* __restrict__ tl) {
    __shared__ WaveQueue5 queues[BLOCK / 64];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_blob[];
    const int lane = threadIdx.x & 63;
    const int gwave = (int)((blockIdx.x * BLOCK + threadIdx.x) >> 6);
    uint32_t tl_needy = 0, tl_item = 0;
    auto mark = [&](int k) {
        if (TL) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (lane == 0) tl[gwave * 8 + k] = t;
        }
    };
    mark(0);
    WaveQueue5* qu = &queues[threadIdx.x >> 6];
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    const int64_t gfirst = (int64_t)blockIdx.x * BLOCK;
    int64_t g = gfirst + threadIdx.x;
    constexpr int NV = 3 * SPL;  // doubles per group
    double va[NV], vb[NV];
    // (no full group: loads read the WorldView instead, >= 96 bytes, ignored)
    const double* xyzb = groups > 0 ? xyz : reinterpret_cast<const double*>(wv);
    auto load = [&](int64_t grp, double (&dst)[NV]) {
        grp = grp < groups ? grp : groups - 1;
        grp = grp < 0 ? 0 : grp;
        const double2* q = reinterpret_cast<const double2*>(xyzb) + (NV / 2) * grp;
#pragma unroll
        for (int k = 0; k < NV / 2; ++k) {
            const double2 t = q[k];
            dst[2 * k] = t.x;
            dst[2 * k + 1] = t.y;
        }
    };
    // [off_aos, blob_bytes): records, list headers, list ids, class table.  The copy's
    // loads are issued BEFORE the group's loads and stored after them, so the stores
    // wait on a counted vmcnt that leaves the group's HBM loads in flight, and the
    // barrier below never waits on HBM.  Every lane loads and stores every chunk slot
    // (clamped source; out-of-range chunks go to a dummy LDS slot): no branches.  xyz
    // is not __restrict__ so its loads cannot be sunk past the LDS stores.
    // (LDS-DMA variants were tried: hipcc then drains vmcnt at the first use of any
    // group, prefetched ones included.)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 struct ends up on the stack)
    constexpr int kStageChunks = (int)(kStageBudget / (BLOCK * 16));
    u32x4 stg[kStageChunks];
    const uint32_t n16 = stage_bytes / 16u;  // >= 1 (the class table's sentinel)
#if defined(__HIP_DEVICE_COMPILE__)  // global (not flat) loads: flat ones would also count lgkmcnt and force vmcnt(0)
    typedef const __attribute__((address_space(1))) u32x4* gptr_stage;
    const gptr_stage ssrc = (gptr_stage)(wv->blob + wv->off_aos);
#else
    const u32x4* ssrc = reinterpret_cast<const u32x4*>(wv->blob + wv->off_aos);
#endif
#pragma unroll
    for (int i = 0; i < kStageChunks; ++i) {
        const uint32_t o = (uint32_t)(i * BLOCK) + threadIdx.x;
        stg[i] = ssrc[o < n16 ? o : n16 - 1u];
    }
    load(g, va);  // unconditional (clamped): a branch here would make hipcc's vmcnt counts conservative
#pragma unroll
    for (int i = 0; i < kStageChunks; ++i) {
        const uint32_t o = (uint32_t)(i * BLOCK) + threadIdx.x;
        // (the launch allocates 16 spare bytes after the copy: the dummy slot)
        *reinterpret_cast<u32x4*>(lds_blob + 16u * (o < n16 ? o : n16)) = stg[i];
    }
    const uint32_t lists_off = wv->off_lists - wv->off_aos, ids_off = wv->off_ids - wv->off_aos;
    const uint16_t* cls_tab = reinterpret_cast<const uint16_t*>(lds_blob + (wv->off_bitmap - wv->off_aos));
    const uint32_t* hdrs = reinterpret_cast<const uint32_t*>(lds_blob + lists_off);
    const uint16_t* ids_all = reinterpret_cast<const uint16_t*>(lds_blob + ids_off);
    const double* recs = reinterpret_cast<const double*>(lds_blob);
    const float ox = wv->bofx, oy = wv->bofy, oz = wv->bofz, ix = wv->bix, iy = wv->biy, iz = wv->biz;
    const uint32_t nx = (uint32_t)wv->bnx, ny = (uint32_t)wv->bny, nz = (uint32_t)wv->bnz;
    const double rg = wv->r_gate, ro = wv->r_obst;
    __syncthreads();
    mark(1);
    mark(2);
    auto cls_of = [&](double px, double py, double pz) -> uint32_t {
        const uint32_t cx = cell_axis5(px, ox, ix, nx - 1), cy = cell_axis5(py, oy, iy, ny - 1),
                       cz = cell_axis5(pz, oz, iz, nz - 1);
        return (uint32_t)cls_tab[__umul24(__umul24(cz, ny) + cy, nx) + cx];
    };
    auto process = [&](int64_t gg, const double (&v)[NV]) {
        const bool live = gg < groups;
        uint32_t c[SPL];
        bool needy[SPL];
        unsigned long long b[SPL];
        uint32_t base[SPL], total = 0;
#pragma unroll
        for (int k = 0; k < SPL; ++k) c[k] = cls_of(v[3 * k], v[3 * k + 1], v[3 * k + 2]);
#pragma unroll
        for (int k = 0; k < SPL; ++k) {
            needy[k] = live & (c[k] != 0u);
            b[k] = __ballot(needy[k]);
            base[k] = total;
            total += (uint32_t)__popcll(b[k]);
        }
        if (TL) {
            tl_needy += total;
            if (tl_item == 0) mark(4);
        }
        uint32_t hits = 0;
        if (fast == 2) {  // ablation (diagnostics only, wrong answers): needy states count as hits
#pragma unroll
            for (int k = 0; k < SPL; ++k) hits |= needy[k] ? 1u << k : 0u;
        } else if (total > 0) {  // wave-uniform
            uint32_t pos[SPL];
#pragma unroll
            for (int k = 0; k < SPL; ++k) pos[k] = base[k] + lanes_below(b[k]);
            // queue the needy states (slot = rank in the wave), rounds of 64
            for (uint32_t r0 = 0; r0 < total; r0 += 64) {
#pragma unroll
                for (int k = 0; k < SPL; ++k) {
                    const uint32_t slot = pos[k] - r0;
                    if (needy[k] && slot < 64u) {
                        qu->x[slot] = v[3 * k];
                        qu->y[slot] = v[3 * k + 1];
                        qu->z[slot] = v[3 * k + 2];
                        qu->cls[slot] = (uint16_t)c[k];
                    }
                }
                wave_lds_sync();
                const uint32_t tq = min(total - r0, 64u);
                // lane e < tq owns queued state e: its candidate list
                const bool act = (uint32_t)lane < tq;
                const uint32_t hd = hdrs[act ? (uint32_t)qu->cls[lane] : 0u];  // list 0 is empty
                const uint32_t cnt = hd & 4095u, first = hd >> 12;
                uint32_t ptot;
                const uint32_t poff = wave_excl_scan(cnt, lane, ptot);
                bool hit_e = false;
                if (fast && ptot <= 128u) {
                    // one (state, candidate) pair per lane and round (two rounds at most):
                    // pair q finds its state as the max-scan of segment heads (state e
                    // marks position poff_e); hits come back by ballot
                    qu->pair[lane] = 0u;
                    qu->pair[64 + lane] = 0u;
                    if (act) qu->pair[poff] = (uint32_t)lane;  // cnt >= 1 for queued states
                    wave_lds_sync();
                    const uint32_t e0 = dpp_incl_max(qu->pair[lane]);
                    auto test = [&](uint32_t e, uint32_t q) {
                        const uint32_t pe = (uint32_t)__shfl((int)poff, (int)e, 64);
                        const uint32_t fe = (uint32_t)__shfl((int)first, (int)e, 64);
                        return q < ptot && rec_hit<MINDIST>(recs + (size_t)ids_all[fe + q - pe] * kRecDoubles, rg, ro,
                                                            qu->x[e], qu->y[e], qu->z[e], can_pass != 0, md);
                    };
                    const unsigned long long m0 = __ballot(test(e0, (uint32_t)lane));
                    unsigned long long m1 = 0ull;
                    if (ptot > 64u) {  // wave-uniform
                        const uint32_t carry = (uint32_t)__builtin_amdgcn_readlane((int)e0, 63);
                        const uint32_t e1 = max(dpp_incl_max(qu->pair[64 + lane]), carry);
                        m1 = __ballot(test(e1, 64u + (uint32_t)lane));
                    }
                    // any hit among this state's pairs [poff, poff + cnt) of the 128-bit mask
                    auto bits = [](unsigned long long m, uint32_t from, uint32_t len) {
                        const unsigned long long msk = len >= 64u ? ~0ull : ((1ull << len) - 1ull);
                        return ((m >> from) & msk) != 0ull;
                    };
                    const uint32_t end = poff + cnt;
                    const bool lo = poff < 64u && bits(m0, poff, min(end, 64u) - poff);
                    const bool hi = end > 64u && bits(m1, poff > 64u ? poff - 64u : 0u, end - max(poff, 64u));
                    hit_e = act && (lo || hi);
                } else if (act) {  // long lists: each queued state walks its own
                    hit_e = states_exact_rec<MINDIST>(lds_blob, lists_off, ids_off, rg, ro, qu->x[lane], qu->y[lane],
                                                      qu->z[lane], qu->cls[lane], can_pass, md);
                }
                // back to the owners: state slot r0 + e lives on lane e
                const unsigned long long hm = __ballot(hit_e);
#pragma unroll
                for (int k = 0; k < SPL; ++k) {
                    const uint32_t slot = pos[k] - r0;
                    if (needy[k] && slot < 64u && ((hm >> slot) & 1ull)) hits |= 1u << k;
                }
                wave_lds_sync();  // the queue is rewritten next
            }
            if (TL && tl_item == 0) mark(5);
        }
        if (TL) ++tl_item;
        const uint32_t fl = live ? (~hits & ((1u << SPL) - 1u)) : 0u;  // bit k: state SPL gg + k valid
        if (live) {
            if (SPL == 4) {
                *reinterpret_cast<uint32_t*>(valid + 4 * gg) =
                    (fl & 1u) | ((fl & 2u) << 7) | ((fl & 4u) << 14) | ((fl & 8u) << 21);
            } else {
                unsigned long long w = 0ull;
#pragma unroll
                for (int k = 0; k < SPL; ++k) w |= (unsigned long long)((fl >> k) & 1u) << (8 * k);
                *reinterpret_cast<unsigned long long*>(valid + SPL * gg) = w;
            }
        }
        if (COMPACT) {  // wave-ballot compaction
            const uint32_t cnt = (uint32_t)__popc(fl);
            uint32_t ctot;
            const uint32_t cex = wave_excl_scan(cnt, lane, ctot);
            unsigned long long wbase = 0;
            if (lane == 0 && ctot) wbase = atomicAdd(n_valid, (unsigned long long)ctot);
            wbase = __shfl(wbase, 0, 64);
            uint64_t p = wbase + cex;
#pragma unroll
            for (int k = 0; k < SPL; ++k)
                if ((fl >> k) & 1u) compact_idx[p++] = (int32_t)(SPL * gg + k);
        }
    };
    // block-uniform trip count; the next group's loads are issued before this one is
    // classified (vmcnt counts in order: the class lookups never wait on them)
    if (PREFETCH) {  // prefetch loads unconditional (clamped): counted vmcnt, no merge points
        for (int64_t g0 = gfirst; g0 < groups; g0 += 2 * stride, g += 2 * stride) {
            load(g + stride, vb);
            process(g, va);
            if (g0 + stride >= groups) break;
            load(g + 2 * stride, va);
            process(g + stride, vb);
        }
    } else {
        for (int64_t g0 = gfirst; g0 < groups; g0 += stride, g += stride) {
            if (g0 != gfirst) load(g, va);
            process(g, va);
        }
    }
    if (TL) {
        mark(3);
        if (lane == 0) {
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            tl[gwave * 8 + 6] = hw;
            tl[gwave * 8 + 7] = xcc | ((unsigned long long)tl_needy << 32);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - SPL * groups)) {  // tail: the last n % SPL states
        const int64_t i = SPL * groups + threadIdx.x;
        const double px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
        const uint32_t c = cls_of(px, py, pz);
        const bool ok = !(c != 0u && states_exact_rec<MINDIST>(lds_blob, lists_off, ids_off, rg, ro, px, py, pz, c,
                                                               can_pass, md));
        valid[i] = ok ? 1 : 0;
        if (COMPACT && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

template <bool LDS, int MODE>
__global__ __launch_bounds__(kBlock) void k_motions(WorldView w, const double* __restrict__ s1,
                                                    const double* __restrict__ s2, int64_t n,
                                                    int can_pass, uint8_t* __restrict__ valid,
                                                    int aligned) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const unsigned char* base = LDS ? stage_world(w, lds, w.blob_bytes) : w.blob;
    const Acc a = make_acc(base, base, w);
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

// ---- k_motions_v2: motion checks out of LDS ----------------------------------------
// The coarse grid (occupancy masks, cell starts, cell lists) and the AoS OBB records are
// staged into LDS once per persistent workgroup; one edge per lane per iteration.  Every
// candidate test is branch-free on LDS data: all record fields are read up front, so a
// candidate costs one LDS round trip instead of the short-circuit chain of dependent
// global loads of k_motions.  Same candidate order, de-duplication (first common cell)
// and predicates as ray_valid / ray_valid_d32 (src/World.cpp:130-162, src/OBB.cpp:10-91).

// OBB::checkCollisionWithRay (src/OBB.cpp:10-61) on one AoS record, branch-free.  `r` is
// the owner's inflation radius; the endpoint tests inflate only collision OBBs (:13-14),
// the slab test always (:28).  Axes are processed in order with the reference's min /
// max selects; an axis after a rejection cannot undo it, so evaluating every axis and
// combining the rejections gives the reference's early-return answer.
__device__ __forceinline__ bool rec_ray_hit(const double* rec, const double s[3], const double e[3], double r) {
    double f[kRecDoubles];
#pragma unroll
    for (int k = 0; k <= F_HZ; ++k) f[k] = rec[k];
    f[R_META] = rec[R_META];
    const uint32_t m = (uint32_t)__double_as_longlong(f[R_META]);
    const bool fill = (m & META_FILLING) != 0u;
    const double c = f[F_COS], sn = f[F_SIN];
    const double cx = f[F_CX], cy = f[F_CY], cz = f[F_CZ];
    const double h[3] = {f[F_HX], f[F_HY], f[F_HZ]};
    // endpoint tests  :13-18 (OBB::checkCollisionWithPoint, inflated iff collision)
    const double ph0 = fill ? h[0] : h[0] + r, ph1 = fill ? h[1] : h[1] + r, ph2 = fill ? h[2] : h[2] + r;
    double ls[3], ld[3];
    bool end_hit;
    {
        const double dx = s[0] - cx, dy = s[1] - cy, dz = s[2] - cz;
        ls[0] = c * dx + sn * dy;
        ls[1] = c * dy - sn * dx;
        ls[2] = dz;
        const double ex = e[0] - cx, ey = e[1] - cy, ez = e[2] - cz;
        const double le0 = c * ex + sn * ey, le1 = c * ey - sn * ex;
        end_hit = ((fabs(ls[0]) <= ph0) & (fabs(ls[1]) <= ph1) & (fabs(dz) <= ph2)) |
                  ((fabs(le0) <= ph0) & (fabs(le1) <= ph1) & (fabs(ez) <= ph2));
        ld[0] = le0 - ls[0];  // localEnd - localStart  :23
        ld[1] = le1 - ls[1];
        ld[2] = ez - ls[2];
    }
    double tMin = 0.0, tMax = 1.0;
    bool rejected = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double ih = h[k] + r;  // always inflated  :28
        const double bmin = -ih, bmax = ih;
        const bool par = fabs(ld[k]) < 1e-6;  // :34
        const bool outside = (ls[k] < bmin) | (ls[k] > bmax);
        const double invD = 1.0 / ld[k];  // :44 (unused when par)
        const double t1 = (bmin - ls[k]) * invD;
        const double t2 = (bmax - ls[k]) * invD;
        const double tEntry = (t2 < t1) ? t2 : t1;  // std::min
        const double tExit = (t1 < t2) ? t2 : t1;   // std::max
        const double nMin = (tMin < tEntry) ? tEntry : tMin;
        const double nMax = (tExit < tMax) ? tExit : tMax;
        rejected = rejected | (par & outside) | (!par & (nMin > nMax));
        tMin = par ? tMin : nMin;
        tMax = par ? tMax : nMax;
    }
    const bool slab_hit = !rejected & (0 <= tMin) & (tMin <= 1) & (0 <= tMax) & (tMax <= 1);  // :60
    return end_hit | slab_hit;
}

template <int MODE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_motions_v2(const WorldView* __restrict__ wv, const double* __restrict__ s1,
                                                        const double* __restrict__ s2, int64_t n, int can_pass,
                                                        uint8_t* __restrict__ valid, uint32_t front_bytes,
                                                        uint32_t rec_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // [0, front_bytes): masks, cell starts, cell lists (the blob up to `meta`);
    // [front_bytes, + rec_bytes): the AoS records
    {
        const uint4* src0 = reinterpret_cast<const uint4*>(wv->blob);
        const uint4* src1 = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t o = threadIdx.x; o < front_bytes / 16; o += BLOCK) dst[o] = src0[o];
        uint4* dst1 = reinterpret_cast<uint4*>(lds + front_bytes);
        for (uint32_t o = threadIdx.x; o < rec_bytes / 16; o += BLOCK) dst1[o] = src1[o];
    }
    const unsigned long long* mask = reinterpret_cast<const unsigned long long*>(lds + wv->off_cell_mask);
    const uint32_t* cs = reinterpret_cast<const uint32_t*>(lds + wv->off_cell_start);
    const uint16_t* co = reinterpret_cast<const uint16_t*>(lds + wv->off_cell_obb);
    const double* recs = reinterpret_cast<const double*>(lds + front_bytes);
    const int nx = wv->nx, ny = wv->ny, nz = wv->nz;
    const double gx0 = wv->gx0, gy0 = wv->gy0, gz0 = wv->gz0, gx1 = wv->gx1, gy1 = wv->gy1, gz1 = wv->gz1;
    const float ofx = wv->ofx, ofy = wv->ofy, ofz = wv->ofz, i4x = wv->i4x, i4y = wv->i4y, i4z = wv->i4z;
    const float limx = wv->limx, limy = wv->limy, limz = wv->limz;
    const float fmx = wv->fmaxx, fmy = wv->fmaxy, fmz = wv->fmaxz;
    const double rg = wv->r_gate, ro = wv->r_obst;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
        const double s[3] = {s1[3 * i], s1[3 * i + 1], s1[3 * i + 2]};
        const double e[3] = {s2[3 * i], s2[3 * i + 1], s2[3 * i + 2]};
        bool ok = true;
        if (MODE == 0) {
            // World::checkRayValid — rtree intersects(rayBox): closed AABB overlap
            double lo[3], hi[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                lo[k] = (e[k] < s[k]) ? e[k] : s[k];
                hi[k] = (s[k] < e[k]) ? e[k] : s[k];
            }
            if (!(hi[0] < gx0 || gx1 < lo[0] || hi[1] < gy0 || gy1 < lo[1] || hi[2] < gz0 || gz1 < lo[2])) {
                const int x0 = fine_index(fine_coord(lo[0], ofx, i4x), nx) >> 2;
                const int x1 = fine_index(fine_coord(hi[0], ofx, i4x), nx) >> 2;
                const int y0 = fine_index(fine_coord(lo[1], ofy, i4y), ny) >> 2;
                const int y1 = fine_index(fine_coord(hi[1], ofy, i4y), ny) >> 2;
                const int z0 = fine_index(fine_coord(lo[2], ofz, i4z), nz) >> 2;
                const int z1 = fine_index(fine_coord(hi[2], ofz, i4z), nz) >> 2;
                for (int z = z0; z <= z1 && ok; ++z)
                    for (int y = y0; y <= y1 && ok; ++y)
                        for (int x = x0; x <= x1 && ok; ++x) {
                            const int cell = (z * ny + y) * nx + x;
                            const uint32_t b = cs[cell], en = cs[cell + 1];
                            for (uint32_t k = b; k < en; ++k) {
                                const double* rec = recs + (size_t)co[k] * kRecDoubles;
                                const uint32_t m = (uint32_t)__double_as_longlong(rec[R_META]);
                                const int ox = (m >> 8) & 255, oy = (m >> 16) & 255, oz = m >> 24;
                                // tested once: in the first cell its and the ray's ranges share
                                const bool first = x == (ox > x0 ? ox : x0) && y == (oy > y0 ? oy : y0) &&
                                                   z == (oz > z0 ? oz : z0);
                                const bool overlap = !(rec[F_HIX] < lo[0] || hi[0] < rec[F_LOX] || rec[F_HIY] < lo[1] ||
                                                       hi[1] < rec[F_LOY] || rec[F_HIZ] < lo[2] || hi[2] < rec[F_LOZ]);
                                const bool skip = (m & META_FILLING) && can_pass;  // :150-153
                                if (first && overlap && !skip &&
                                    rec_ray_hit(rec, s, e, (m & META_GATE) ? rg : ro)) {
                                    ok = false;
                                    break;
                                }
                            }
                        }
            }
        } else {
            // discrete32: x = s + (e - s) * (k/32), k = 1..32 (World::checkPointValidity each)
            for (int k = 1; k <= 32 && ok; ++k) {
                const double t = (double)k / 32.0;
                const double px = s[0] + (e[0] - s[0]) * t;
                const double py = s[1] + (e[1] - s[1]) * t;
                const double pz = s[2] + (e[2] - s[2]) * t;
                const float fx = fine_coord(px, ofx, i4x), fy = fine_coord(py, ofy, i4y), fz = fine_coord(pz, ofz, i4z);
                const bool in = (fx >= 0.0f) & (fx <= limx) & (fy >= 0.0f) & (fy <= limy) & (fz >= 0.0f) & (fz <= limz);
                const int ix = (int)fminf(fmaxf(fx, 0.0f), fmx);
                const int iy = (int)fminf(fmaxf(fy, 0.0f), fmy);
                const int iz = (int)fminf(fmaxf(fz, 0.0f), fmz);
                const int cell = ((iz >> 2) * ny + (iy >> 2)) * nx + (ix >> 2);
                const uint32_t bit = (uint32_t)((((iz & 3) << 2) + (iy & 3)) * 4 + (ix & 3));
                const bool occ = in && ((mask[cell] >> bit) & 1ull);
                if (!occ) continue;
                const uint32_t b = cs[cell], en = cs[cell + 1];
                for (uint32_t q = b; q < en; ++q)
                    if (rec_hit<false>(recs + (size_t)co[q] * kRecDoubles, rg, ro, px, py, pz, can_pass != 0, 0.0)) {
                        ok = false;
                        break;
                    }
            }
        }
        valid[i] = ok ? 1 : 0;
    }
}

// ---- k_motions_v3: analytic motion checks with a per-wave candidate queue ------------
// k_motions_v2's analytic mode pays the divergent per-lane walk AND, whenever any lane of
// the wave reaches a surviving candidate, the ~200-instruction slab test with most lanes
// idle (C3: ~0.9 candidates per edge on average, ~5 for the wave's worst lane).  Here the
// walk only filters (first common cell, closed AABB overlap, filling skip — the rtree
// prefilter of src/World.cpp:143-153) and pushes (lane, OBB) pairs into the wave's LDS
// queue; the wave then runs the exact test over the queue 64 pairs at a time with every
// lane busy, the pair's edge fetched from its owner lane by ds_bpermute.  Any hit clears
// the owner's flag.  An edge is invalid iff some candidate hits, so testing every
// candidate (no early exit) gives the reference's answer.  A full queue makes the
// pushing lane test inline (same predicate).
constexpr int kQueueM = 256;  // queued pairs per wave

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_motions_v3(const WorldView* __restrict__ wv, const double* __restrict__ s1,
                                                      const double* __restrict__ s2, int64_t n, int can_pass,
                                                      uint8_t* __restrict__ valid, uint32_t front_bytes,
                                                      uint32_t rec_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    {
        const uint4* src0 = reinterpret_cast<const uint4*>(wv->blob);
        const uint4* src1 = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t o = threadIdx.x; o < front_bytes / 16; o += BLOCK) dst[o] = src0[o];
        uint4* dst1 = reinterpret_cast<uint4*>(lds + front_bytes);
        for (uint32_t o = threadIdx.x; o < rec_bytes / 16; o += BLOCK) dst1[o] = src1[o];
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* queue = reinterpret_cast<uint32_t*>(lds + front_bytes + rec_bytes) + wave * (kQueueM + 1);
    uint32_t* qcount = queue + kQueueM;
    uint8_t* flags = lds + front_bytes + rec_bytes + (BLOCK / 64) * (kQueueM + 1) * 4 + wave * 64;
    // walk filter table: per OBB {float lo[3], meta, float hi[3], pad} (32 B, two LDS
    // reads), the AABB rounded outward, so the float overlap test passes every pair the
    // double test passes; the double test is redone on the queued pairs
    float4* filt = reinterpret_cast<float4*>(lds + front_bytes + rec_bytes + (BLOCK / 64) * ((kQueueM + 1) * 4 + 64));
    const uint32_t* cs = reinterpret_cast<const uint32_t*>(lds + wv->off_cell_start);
    const uint16_t* co = reinterpret_cast<const uint16_t*>(lds + wv->off_cell_obb);
    const double* recs = reinterpret_cast<const double*>(lds + front_bytes);
    __syncthreads();  // records staged
    for (int o = threadIdx.x; o < wv->n_obb; o += BLOCK) {
        const double* r = recs + (size_t)o * kRecDoubles;
        filt[2 * o] = make_float4(__double2float_rd(r[F_LOX]), __double2float_rd(r[F_LOY]), __double2float_rd(r[F_LOZ]),
                                  __uint_as_float((uint32_t)__double_as_longlong(r[R_META])));
        filt[2 * o + 1] = make_float4(__double2float_ru(r[F_HIX]), __double2float_ru(r[F_HIY]),
                                      __double2float_ru(r[F_HIZ]), 0.0f);
    }
    const int nx = wv->nx, ny = wv->ny, nz = wv->nz;
    const double gx0 = wv->gx0, gy0 = wv->gy0, gz0 = wv->gz0, gx1 = wv->gx1, gy1 = wv->gy1, gz1 = wv->gz1;
    const float ofx = wv->ofx, ofy = wv->ofy, ofz = wv->ofz, i4x = wv->i4x, i4y = wv->i4y, i4z = wv->i4z;
    const double rg = wv->r_gate, ro = wv->r_obst;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    // wave-uniform loop: every lane of the wave runs every iteration (ds_bpermute below)
    for (int64_t i0 = (int64_t)blockIdx.x * BLOCK + wave * 64; i0 < n; i0 += stride) {
        const int64_t i = i0 + lane;
        const bool act = i < n;
        double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
        if (act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s[k] = s1[3 * i + k];
                e[k] = s2[3 * i + k];
            }
        }
        if (lane == 0) *qcount = 0u;
        flags[lane] = 1;
        wave_lds_sync();
        bool ok = true;
        double lo[3], hi[3];
        float flo[3], fhi[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = (e[k] < s[k]) ? e[k] : s[k];
            hi[k] = (s[k] < e[k]) ? e[k] : s[k];
            flo[k] = __double2float_rd(lo[k]);
            fhi[k] = __double2float_ru(hi[k]);
        }
        // World::checkRayValid — rtree intersects(rayBox): closed AABB overlap
        if (act && !(hi[0] < gx0 || gx1 < lo[0] || hi[1] < gy0 || gy1 < lo[1] || hi[2] < gz0 || gz1 < lo[2])) {
            const int x0 = fine_index(fine_coord(lo[0], ofx, i4x), nx) >> 2;
            const int x1 = fine_index(fine_coord(hi[0], ofx, i4x), nx) >> 2;
            const int y0 = fine_index(fine_coord(lo[1], ofy, i4y), ny) >> 2;
            const int y1 = fine_index(fine_coord(hi[1], ofy, i4y), ny) >> 2;
            const int z0 = fine_index(fine_coord(lo[2], ofz, i4z), nz) >> 2;
            const int z1 = fine_index(fine_coord(hi[2], ofz, i4z), nz) >> 2;
            for (int z = z0; z <= z1; ++z)
                for (int y = y0; y <= y1; ++y)
                    for (int x = x0; x <= x1; ++x) {
                        const int cell = (z * ny + y) * nx + x;
                        const uint32_t b = cs[cell], en = cs[cell + 1];
                        for (uint32_t k = b; k < en; ++k) {
                            const uint32_t id = co[k];
                            const float4 fa = filt[2 * id], fb = filt[2 * id + 1];
                            const uint32_t m = __float_as_uint(fa.w);
                            const int ox = (m >> 8) & 255, oy = (m >> 16) & 255, oz = m >> 24;
                            const bool first = (x == (ox > x0 ? ox : x0)) & (y == (oy > y0 ? oy : y0)) &
                                               (z == (oz > z0 ? oz : z0));
                            const bool may = !((fb.x < flo[0]) | (fhi[0] < fa.x) | (fb.y < flo[1]) | (fhi[1] < fa.y) |
                                               (fb.z < flo[2]) | (fhi[2] < fa.z));
                            const bool skip = (m & META_FILLING) && can_pass;  // :150-153
                            if (first & may & !skip) {
                                const uint32_t slot = atomicAdd(qcount, 1u);
                                if (slot < (uint32_t)kQueueM) {
                                    queue[slot] = (id << 6) | (uint32_t)lane;
                                } else {
                                    const double* rec = recs + (size_t)id * kRecDoubles;
                                    const bool overlap =
                                        !((rec[F_HIX] < lo[0]) | (hi[0] < rec[F_LOX]) | (rec[F_HIY] < lo[1]) |
                                          (hi[1] < rec[F_LOY]) | (rec[F_HIZ] < lo[2]) | (hi[2] < rec[F_LOZ]));
                                    if (overlap && rec_ray_hit(rec, s, e, (m & META_GATE) ? rg : ro)) ok = false;
                                }
                            }
                        }
                    }
        }
        wave_lds_sync();
        const uint32_t total = min(*qcount, (uint32_t)kQueueM);
        for (uint32_t base = 0; base < total; base += 64) {
            const uint32_t j = base + lane;
            const bool has = j < total;
            const uint32_t q = has ? queue[j] : 0u;
            const int owner = (int)(q & 63u);
            double ps[3], pe[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                ps[k] = __shfl(s[k], owner);
                pe[k] = __shfl(e[k], owner);
            }
            if (has) {
                const double* rec = recs + (size_t)(q >> 6) * kRecDoubles;
                const uint32_t m = (uint32_t)__double_as_longlong(rec[R_META]);
                // the exact rtree prefilter: closed overlap of the OBB's AABB and the ray box
                double plo[3], phi[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    plo[k] = (pe[k] < ps[k]) ? pe[k] : ps[k];
                    phi[k] = (ps[k] < pe[k]) ? pe[k] : ps[k];
                }
                const bool overlap = !((rec[F_HIX] < plo[0]) | (phi[0] < rec[F_LOX]) | (rec[F_HIY] < plo[1]) |
                                       (phi[1] < rec[F_LOY]) | (rec[F_HIZ] < plo[2]) | (phi[2] < rec[F_LOZ]));
                if (overlap && rec_ray_hit(rec, ps, pe, (m & META_GATE) ? rg : ro)) flags[owner] = 0;
            }
        }
        wave_lds_sync();
        if (act) valid[i] = (ok && flags[lane]) ? 1 : 0;
        wave_lds_sync();  // flags / count are reset by the next iteration
    }
}

// ---- k_motions_v4: analytic motion checks, lane-balanced candidate walk ---------------
// v3's walk is per lane, so a wave pays its worst lane's list length (C3: 28.5 entries
// against a wave average of 6.7).  v4 expands the work over the whole wave in two
// levels, all in wave-uniform control flow:
//   1. (edge, coarse cell) pairs: each lane's cell box has nc cells; an exclusive scan of
//      nc lays the pairs out, 64 per chunk; a lane finds the pair's owner edge by a DPP
//      max-scan of segment heads (LDS `heads`) and decodes the cell from the owner's box;
//   2. (pair, list entry): the chunk's list lengths are scanned the same way; each lane
//      takes one entry, reads the OBB's 32-byte filter record (outward-rounded float
//      AABB + meta) and applies the first-common-cell rule, the overlap test and the
//      filling skip (src/World.cpp:143-153); survivors go to the wave's queue.
// The queue is flushed (exact double overlap + OBB::checkCollisionWithRay on 64 pairs at
// a time, as in v3) whenever it could not take another chunk, and at the end, so it never
// overflows.  Same answers as the reference: an edge is invalid iff some candidate hits.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_motions_v4(const WorldView* __restrict__ wv, const double* __restrict__ s1,
                                                      const double* __restrict__ s2, int64_t n, int can_pass,
                                                      uint8_t* __restrict__ valid, uint32_t front_bytes,
                                                      uint32_t rec_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    {
        const uint4* src0 = reinterpret_cast<const uint4*>(wv->blob);
        const uint4* src1 = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t o = threadIdx.x; o < front_bytes / 16; o += BLOCK) dst[o] = src0[o];
        uint4* dst1 = reinterpret_cast<uint4*>(lds + front_bytes);
        for (uint32_t o = threadIdx.x; o < rec_bytes / 16; o += BLOCK) dst1[o] = src1[o];
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // per wave: queue[kQueueM], count, flags[64] (bytes), heads[64] (u32)
    constexpr uint32_t kWaveBytes = (kQueueM + 1) * 4 + 64 + 256;
    unsigned char* wbase = lds + front_bytes + rec_bytes + wave * kWaveBytes;
    uint32_t* queue = reinterpret_cast<uint32_t*>(wbase);
    uint32_t* qcount = queue + kQueueM;
    uint8_t* flags = wbase + (kQueueM + 1) * 4;
    uint32_t* heads = reinterpret_cast<uint32_t*>(wbase + (kQueueM + 1) * 4 + 64);
    float4* filt = reinterpret_cast<float4*>(lds + front_bytes + rec_bytes + (BLOCK / 64) * kWaveBytes);
    const uint32_t* cs = reinterpret_cast<const uint32_t*>(lds + wv->off_cell_start);
    const uint16_t* co = reinterpret_cast<const uint16_t*>(lds + wv->off_cell_obb);
    const double* recs = reinterpret_cast<const double*>(lds + front_bytes);
    __syncthreads();  // records staged
    for (int o = threadIdx.x; o < wv->n_obb; o += BLOCK) {
        const double* r = recs + (size_t)o * kRecDoubles;
        filt[2 * o] = make_float4(__double2float_rd(r[F_LOX]), __double2float_rd(r[F_LOY]), __double2float_rd(r[F_LOZ]),
                                  __uint_as_float((uint32_t)__double_as_longlong(r[R_META])));
        filt[2 * o + 1] = make_float4(__double2float_ru(r[F_HIX]), __double2float_ru(r[F_HIY]),
                                      __double2float_ru(r[F_HIZ]), 0.0f);
    }
    const int nx = wv->nx, ny = wv->ny, nz = wv->nz;
    const double gx0 = wv->gx0, gy0 = wv->gy0, gz0 = wv->gz0, gx1 = wv->gx1, gy1 = wv->gy1, gz1 = wv->gz1;
    const float ofx = wv->ofx, ofy = wv->ofy, ofz = wv->ofz, i4x = wv->i4x, i4y = wv->i4y, i4z = wv->i4z;
    const double rg = wv->r_gate, ro = wv->r_obst;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    for (int64_t i0 = (int64_t)blockIdx.x * BLOCK + wave * 64; i0 < n; i0 += stride) {
        const int64_t i = i0 + lane;
        const bool act = i < n;
        double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
        if (act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s[k] = s1[3 * i + k];
                e[k] = s2[3 * i + k];
            }
        }
        if (lane == 0) *qcount = 0u;
        flags[lane] = 1;
        double lo[3], hi[3];
        float flo[3], fhi[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = (e[k] < s[k]) ? e[k] : s[k];
            hi[k] = (s[k] < e[k]) ? e[k] : s[k];
            flo[k] = __double2float_rd(lo[k]);
            fhi[k] = __double2float_ru(hi[k]);
        }
        // World::checkRayValid — rtree intersects(rayBox): closed AABB overlap with the grid
        const bool in = act && !(hi[0] < gx0 || gx1 < lo[0] || hi[1] < gy0 || gy1 < lo[1] || hi[2] < gz0 || gz1 < lo[2]);
        const int x0 = fine_index(fine_coord(lo[0], ofx, i4x), nx) >> 2;
        const int x1 = fine_index(fine_coord(hi[0], ofx, i4x), nx) >> 2;
        const int y0 = fine_index(fine_coord(lo[1], ofy, i4y), ny) >> 2;
        const int y1 = fine_index(fine_coord(hi[1], ofy, i4y), ny) >> 2;
        const int z0 = fine_index(fine_coord(lo[2], ofz, i4z), nz) >> 2;
        const int z1 = fine_index(fine_coord(hi[2], ofz, i4z), nz) >> 2;
        const uint32_t wx = (uint32_t)(x1 - x0 + 1), wy = (uint32_t)(y1 - y0 + 1);
        const uint32_t nc = in ? wx * wy * (uint32_t)(z1 - z0 + 1) : 0u;
        const uint32_t box0 = (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)z0 << 16);
        const uint32_t boxw = wx | (wy << 8);
        uint32_t total_c;
        const uint32_t offc = wave_excl_scan(nc, lane, total_c);
        wave_lds_sync();

        // exact tests of the queued pairs (wave-uniform call sites only)
        auto flush = [&]() {
            const uint32_t total = *qcount;
            for (uint32_t base = 0; base < total; base += 64) {
                const uint32_t j = base + lane;
                const bool has = j < total;
                const uint32_t q = has ? queue[j] : 0u;
                const int owner = (int)(q & 63u);
                double ps[3], pe[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ps[k] = __shfl(s[k], owner);
                    pe[k] = __shfl(e[k], owner);
                }
                if (has) {
                    const double* rec = recs + (size_t)(q >> 6) * kRecDoubles;
                    const uint32_t m = (uint32_t)__double_as_longlong(rec[R_META]);
                    double plo[3], phi[3];
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        plo[k] = (pe[k] < ps[k]) ? pe[k] : ps[k];
                        phi[k] = (ps[k] < pe[k]) ? pe[k] : ps[k];
                    }
                    const bool overlap = !((rec[F_HIX] < plo[0]) | (phi[0] < rec[F_LOX]) | (rec[F_HIY] < plo[1]) |
                                           (phi[1] < rec[F_LOY]) | (rec[F_HIZ] < plo[2]) | (phi[2] < rec[F_LOZ]));
                    if (overlap && rec_ray_hit(rec, ps, pe, (m & META_GATE) ? rg : ro)) flags[owner] = 0;
                }
            }
            wave_lds_sync();
            if (lane == 0) *qcount = 0u;
            wave_lds_sync();
        };

        uint32_t carry_owner = 0u;
        for (uint32_t cb = 0; cb < total_c; cb += 64) {
            // level 1: lane -> (owner edge, cell)
            heads[lane] = 0u;
            wave_lds_sync();
            if (nc > 0u && offc >= cb && offc < cb + 64u) heads[offc - cb] = (uint32_t)lane + 1u;
            wave_lds_sync();
            const uint32_t hm = dpp_incl_max(heads[lane]);
            const uint32_t owner = hm ? hm - 1u : carry_owner;
            carry_owner = (uint32_t)__builtin_amdgcn_readlane((int)owner, 63);
            const bool has_c = cb + (uint32_t)lane < total_c;
            const uint32_t ooff = (uint32_t)__shfl((int)offc, (int)owner);
            const uint32_t ob = (uint32_t)__shfl((int)box0, (int)owner);
            const uint32_t ow = (uint32_t)__shfl((int)boxw, (int)owner);
            const uint32_t c = cb + (uint32_t)lane - ooff;
            const uint32_t owx = ow & 255u, owy = ow >> 8;
            const uint32_t cx = c % owx, t = c / owx, cy = t % owy, cz = t / owy;
            const uint32_t x = (ob & 255u) + cx, y = ((ob >> 8) & 255u) + cy, z = (ob >> 16) + cz;
            const int cell = ((int)z * ny + (int)y) * nx + (int)x;
            const uint32_t b = has_c ? cs[cell] : 0u;
            const uint32_t len = has_c ? cs[cell + 1] - b : 0u;
            const uint32_t seg = x | (y << 8) | (z << 16) | (owner << 24);
            uint32_t total_e;
            const uint32_t offe = wave_excl_scan(len, lane, total_e);
            // level 2: lane -> (segment, list entry)
            uint32_t carry_s = 0u;
            for (uint32_t eb = 0; eb < total_e; eb += 64) {
                if (*qcount > (uint32_t)(kQueueM - 64)) flush();
                heads[lane] = 0u;
                wave_lds_sync();
                if (len > 0u && offe >= eb && offe < eb + 64u) heads[offe - eb] = (uint32_t)lane + 1u;
                wave_lds_sync();
                const uint32_t hs = dpp_incl_max(heads[lane]);
                const uint32_t sidx = hs ? hs - 1u : carry_s;
                carry_s = (uint32_t)__builtin_amdgcn_readlane((int)sidx, 63);
                const bool has = eb + (uint32_t)lane < total_e;
                const uint32_t sb = (uint32_t)__shfl((int)b, (int)sidx);
                const uint32_t soff = (uint32_t)__shfl((int)offe, (int)sidx);
                const uint32_t sp = (uint32_t)__shfl((int)seg, (int)sidx);
                const int own = (int)(sp >> 24);
                const uint32_t obox = (uint32_t)__shfl((int)box0, own);
                float ol[3], oh[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ol[k] = __shfl(flo[k], own);
                    oh[k] = __shfl(fhi[k], own);
                }
                if (has) {
                    const uint32_t id = co[sb + (eb + (uint32_t)lane - soff)];
                    const float4 fa = filt[2 * id], fb = filt[2 * id + 1];
                    const uint32_t m = __float_as_uint(fa.w);
                    const uint32_t ox = (m >> 8) & 255u, oy = (m >> 16) & 255u, oz = m >> 24;
                    const uint32_t ex0 = obox & 255u, ey0 = (obox >> 8) & 255u, ez0 = obox >> 16;
                    const bool first = ((sp & 255u) == max(ox, ex0)) & (((sp >> 8) & 255u) == max(oy, ey0)) &
                                       (((sp >> 16) & 255u) == max(oz, ez0));
                    const bool may = !((fb.x < ol[0]) | (oh[0] < fa.x) | (fb.y < ol[1]) | (oh[1] < fa.y) |
                                       (fb.z < ol[2]) | (oh[2] < fa.z));
                    const bool skip = (m & META_FILLING) && can_pass;  // :150-153
                    if (first & may & !skip) {
                        const uint32_t slot = atomicAdd(qcount, 1u);
                        queue[slot] = (id << 6) | (uint32_t)own;
                    }
                }
                wave_lds_sync();
            }
        }
        flush();
        if (act) valid[i] = flags[lane] ? 1 : 0;
        wave_lds_sync();
    }
}

// ---- k_motions_d32q: discrete32 motion checks with a per-wave candidate queue ---------
// The 32 points s + (e - s)·k/32 (k = 1..32) are stepped wave-uniformly.  At each k a
// lane whose point lies in an occupied fine cell walks its coarse cell's list and pushes
// the OBBs whose AABB strictly contains the point (the rtree `contains` of
// src/World.cpp:83) as (lane, k, OBB) triples; when the queue holds kFlushD32 or more
// (and after k = 32) the wave runs OBB::checkCollisionWithPoint (src/OBB.cpp:63-91, via
// rec_hit) on 64 triples at a time, the point recomputed from the owner's endpoints with
// the same arithmetic as k_motions_v2.  Lanes already invalid stop pushing.  A push past
// the queue's end is tested inline.
constexpr int kQueueD32 = 512;
constexpr uint32_t kFlushD32 = 256;

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_motions_d32q(const WorldView* __restrict__ wv,
                                                        const double* __restrict__ s1, const double* __restrict__ s2,
                                                        int64_t n, int can_pass, uint8_t* __restrict__ valid,
                                                        uint32_t front_bytes, uint32_t rec_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    {
        const uint4* src0 = reinterpret_cast<const uint4*>(wv->blob);
        const uint4* src1 = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t o = threadIdx.x; o < front_bytes / 16; o += BLOCK) dst[o] = src0[o];
        uint4* dst1 = reinterpret_cast<uint4*>(lds + front_bytes);
        for (uint32_t o = threadIdx.x; o < rec_bytes / 16; o += BLOCK) dst1[o] = src1[o];
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* queue = reinterpret_cast<uint32_t*>(lds + front_bytes + rec_bytes) + wave * (kQueueD32 + 1);
    uint32_t* qcount = queue + kQueueD32;
    uint8_t* flags = lds + front_bytes + rec_bytes + (BLOCK / 64) * (kQueueD32 + 1) * 4 + wave * 64;
    const unsigned long long* mask = reinterpret_cast<const unsigned long long*>(lds + wv->off_cell_mask);
    const uint32_t* cs = reinterpret_cast<const uint32_t*>(lds + wv->off_cell_start);
    const uint16_t* co = reinterpret_cast<const uint16_t*>(lds + wv->off_cell_obb);
    const double* recs = reinterpret_cast<const double*>(lds + front_bytes);
    const int nx = wv->nx, ny = wv->ny;
    const float ofx = wv->ofx, ofy = wv->ofy, ofz = wv->ofz, i4x = wv->i4x, i4y = wv->i4y, i4z = wv->i4z;
    const float limx = wv->limx, limy = wv->limy, limz = wv->limz;
    const float fmx = wv->fmaxx, fmy = wv->fmaxy, fmz = wv->fmaxz;
    const double rg = wv->r_gate, ro = wv->r_obst;
    const bool cp = can_pass != 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    for (int64_t i0 = (int64_t)blockIdx.x * BLOCK + wave * 64; i0 < n; i0 += stride) {
        const int64_t i = i0 + lane;
        const bool act = i < n;
        double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
        if (act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s[k] = s1[3 * i + k];
                e[k] = s2[3 * i + k];
            }
        }
        if (lane == 0) *qcount = 0u;
        flags[lane] = act ? 1 : 0;
        wave_lds_sync();
        bool ok = true;
        for (int k = 1; k <= 32; ++k) {
            const double t = (double)k / 32.0;
            const double px = s[0] + (e[0] - s[0]) * t;
            const double py = s[1] + (e[1] - s[1]) * t;
            const double pz = s[2] + (e[2] - s[2]) * t;
            const float fx = fine_coord(px, ofx, i4x), fy = fine_coord(py, ofy, i4y), fz = fine_coord(pz, ofz, i4z);
            const bool in = (fx >= 0.0f) & (fx <= limx) & (fy >= 0.0f) & (fy <= limy) & (fz >= 0.0f) & (fz <= limz);
            const int ix = (int)fminf(fmaxf(fx, 0.0f), fmx);
            const int iy = (int)fminf(fmaxf(fy, 0.0f), fmy);
            const int iz = (int)fminf(fmaxf(fz, 0.0f), fmz);
            const int cell = ((iz >> 2) * ny + (iy >> 2)) * nx + (ix >> 2);
            const uint32_t bit = (uint32_t)((((iz & 3) << 2) + (iy & 3)) * 4 + (ix & 3));
            const bool live = ok && flags[lane];
            if (live && in && ((mask[cell] >> bit) & 1ull)) {
                const uint32_t b = cs[cell], en = cs[cell + 1];
                for (uint32_t q = b; q < en; ++q) {
                    const uint32_t id = co[q];
                    const double* rec = recs + (size_t)id * kRecDoubles;
                    // rtree contains(point): strict  src/World.cpp:83 (rec_hit re-tests it)
                    const bool inside = (rec[F_LOX] < px) & (px < rec[F_HIX]) & (rec[F_LOY] < py) &
                                        (py < rec[F_HIY]) & (rec[F_LOZ] < pz) & (pz < rec[F_HIZ]);
                    if (inside) {
                        const uint32_t slot = atomicAdd(qcount, 1u);
                        if (slot < (uint32_t)kQueueD32)
                            queue[slot] = (id << 11) | ((uint32_t)(k - 1) << 6) | (uint32_t)lane;
                        else if (rec_hit<false>(rec, rg, ro, px, py, pz, cp, 0.0))
                            ok = false;
                    }
                }
            }
            wave_lds_sync();
            const uint32_t cnt = *qcount;  // wave-uniform
            if (cnt >= kFlushD32 || k == 32) {
                const uint32_t total = min(cnt, (uint32_t)kQueueD32);
                for (uint32_t base = 0; base < total; base += 64) {
                    const uint32_t j = base + lane;
                    const bool has = j < total;
                    const uint32_t qe = has ? queue[j] : 0u;
                    const int owner = (int)(qe & 63u);
                    double ps[3], pe[3];
#pragma unroll
                    for (int d = 0; d < 3; ++d) {
                        ps[d] = __shfl(s[d], owner);
                        pe[d] = __shfl(e[d], owner);
                    }
                    if (has) {
                        const double tq = (double)(((qe >> 6) & 31u) + 1u) / 32.0;
                        const double qx = ps[0] + (pe[0] - ps[0]) * tq;
                        const double qy = ps[1] + (pe[1] - ps[1]) * tq;
                        const double qz = ps[2] + (pe[2] - ps[2]) * tq;
                        if (rec_hit<false>(recs + (size_t)(qe >> 11) * kRecDoubles, rg, ro, qx, qy, qz, cp, 0.0))
                            flags[owner] = 0;
                    }
                }
                wave_lds_sync();
                if (lane == 0) *qcount = 0u;
                wave_lds_sync();
            }
        }
        if (act) valid[i] = (ok && flags[lane]) ? 1 : 0;
        wave_lds_sync();
    }
}

// ---- k_motions_d32b: discrete32, lane-balanced list walk ------------------------------
// As k_motions_d32q (wave-uniform steps k = 1..32, queued (lane, k, OBB) triples, the
// exact OBB::checkCollisionWithPoint on flush), but at each step the occupied lanes'
// cell lists are expanded over the whole wave (exclusive scan of the list lengths,
// segment heads, DPP max-scan) instead of each lane walking its own list: the wave pays
// ceil(sum of lengths / 64) rounds instead of the longest list.  The entry filter is the
// rtree `contains` (src/World.cpp:83) against the outward-rounded float AABB (a superset
// of the strict double test, which rec_hit repeats).  The queue is flushed before it
// could overflow.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_motions_d32b(const WorldView* __restrict__ wv,
                                                        const double* __restrict__ s1, const double* __restrict__ s2,
                                                        int64_t n, int can_pass, uint8_t* __restrict__ valid,
                                                        uint32_t front_bytes, uint32_t rec_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    {
        const uint4* src0 = reinterpret_cast<const uint4*>(wv->blob);
        const uint4* src1 = reinterpret_cast<const uint4*>(wv->blob + wv->off_aos);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (uint32_t o = threadIdx.x; o < front_bytes / 16; o += BLOCK) dst[o] = src0[o];
        uint4* dst1 = reinterpret_cast<uint4*>(lds + front_bytes);
        for (uint32_t o = threadIdx.x; o < rec_bytes / 16; o += BLOCK) dst1[o] = src1[o];
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr uint32_t kWaveBytes = (kQueueD32 + 1) * 4 + 64 + 256;
    unsigned char* wbase = lds + front_bytes + rec_bytes + wave * kWaveBytes;
    uint32_t* queue = reinterpret_cast<uint32_t*>(wbase);
    uint32_t* qcount = queue + kQueueD32;
    uint8_t* flags = wbase + (kQueueD32 + 1) * 4;
    uint32_t* heads = reinterpret_cast<uint32_t*>(wbase + (kQueueD32 + 1) * 4 + 64);
    float4* filt = reinterpret_cast<float4*>(lds + front_bytes + rec_bytes + (BLOCK / 64) * kWaveBytes);
    const unsigned long long* mask = reinterpret_cast<const unsigned long long*>(lds + wv->off_cell_mask);
    const uint32_t* cs = reinterpret_cast<const uint32_t*>(lds + wv->off_cell_start);
    const uint16_t* co = reinterpret_cast<const uint16_t*>(lds + wv->off_cell_obb);
    const double* recs = reinterpret_cast<const double*>(lds + front_bytes);
    __syncthreads();  // records staged
    for (int o = threadIdx.x; o < wv->n_obb; o += BLOCK) {
        const double* r = recs + (size_t)o * kRecDoubles;
        filt[2 * o] = make_float4(__double2float_rd(r[F_LOX]), __double2float_rd(r[F_LOY]), __double2float_rd(r[F_LOZ]),
                                  0.0f);
        filt[2 * o + 1] = make_float4(__double2float_ru(r[F_HIX]), __double2float_ru(r[F_HIY]),
                                      __double2float_ru(r[F_HIZ]), 0.0f);
    }
    const int nx = wv->nx, ny = wv->ny;
    const float ofx = wv->ofx, ofy = wv->ofy, ofz = wv->ofz, i4x = wv->i4x, i4y = wv->i4y, i4z = wv->i4z;
    const float limx = wv->limx, limy = wv->limy, limz = wv->limz;
    const float fmx = wv->fmaxx, fmy = wv->fmaxy, fmz = wv->fmaxz;
    const double rg = wv->r_gate, ro = wv->r_obst;
    const bool cp = can_pass != 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    for (int64_t i0 = (int64_t)blockIdx.x * BLOCK + wave * 64; i0 < n; i0 += stride) {
        const int64_t i = i0 + lane;
        const bool act = i < n;
        double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
        if (act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s[k] = s1[3 * i + k];
                e[k] = s2[3 * i + k];
            }
        }
        if (lane == 0) *qcount = 0u;
        flags[lane] = act ? 1 : 0;
        wave_lds_sync();
        auto flush = [&]() {
            const uint32_t total = *qcount;
            for (uint32_t base = 0; base < total; base += 64) {
                const uint32_t j = base + lane;
                const bool has = j < total;
                const uint32_t qe = has ? queue[j] : 0u;
                const int owner = (int)(qe & 63u);
                double ps[3], pe[3];
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    ps[d] = __shfl(s[d], owner);
                    pe[d] = __shfl(e[d], owner);
                }
                if (has) {
                    const double tq = (double)(((qe >> 6) & 31u) + 1u) / 32.0;
                    const double qx = ps[0] + (pe[0] - ps[0]) * tq;
                    const double qy = ps[1] + (pe[1] - ps[1]) * tq;
                    const double qz = ps[2] + (pe[2] - ps[2]) * tq;
                    if (rec_hit<false>(recs + (size_t)(qe >> 11) * kRecDoubles, rg, ro, qx, qy, qz, cp, 0.0))
                        flags[owner] = 0;
                }
            }
            wave_lds_sync();
            if (lane == 0) *qcount = 0u;
            wave_lds_sync();
        };
        for (int k = 1; k <= 32; ++k) {
            const double t = (double)k / 32.0;
            const double px = s[0] + (e[0] - s[0]) * t;
            const double py = s[1] + (e[1] - s[1]) * t;
            const double pz = s[2] + (e[2] - s[2]) * t;
            const float fx = fine_coord(px, ofx, i4x), fy = fine_coord(py, ofy, i4y), fz = fine_coord(pz, ofz, i4z);
            const bool in = (fx >= 0.0f) & (fx <= limx) & (fy >= 0.0f) & (fy <= limy) & (fz >= 0.0f) & (fz <= limz);
            const int ix = (int)fminf(fmaxf(fx, 0.0f), fmx);
            const int iy = (int)fminf(fmaxf(fy, 0.0f), fmy);
            const int iz = (int)fminf(fmaxf(fz, 0.0f), fmz);
            const int cell = ((iz >> 2) * ny + (iy >> 2)) * nx + (ix >> 2);
            const uint32_t bit = (uint32_t)((((iz & 3) << 2) + (iy & 3)) * 4 + (ix & 3));
            const bool live = flags[lane] != 0;
            const bool occ = live && in && ((mask[cell] >> bit) & 1ull);
            const uint32_t b = occ ? cs[cell] : 0u;
            const uint32_t len = occ ? cs[cell + 1] - b : 0u;
            uint32_t total_e;
            const uint32_t offe = wave_excl_scan(len, lane, total_e);
            uint32_t carry_s = 0u;
            for (uint32_t eb = 0; eb < total_e; eb += 64) {
                if (*qcount > (uint32_t)(kQueueD32 - 64)) flush();
                heads[lane] = 0u;
                wave_lds_sync();
                if (len > 0u && offe >= eb && offe < eb + 64u) heads[offe - eb] = (uint32_t)lane + 1u;
                wave_lds_sync();
                const uint32_t hs = dpp_incl_max(heads[lane]);
                const uint32_t own = hs ? hs - 1u : carry_s;
                carry_s = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
                const bool has = eb + (uint32_t)lane < total_e;
                const uint32_t sb = (uint32_t)__shfl((int)b, (int)own);
                const uint32_t soff = (uint32_t)__shfl((int)offe, (int)own);
                const double qx = __shfl(px, (int)own), qy = __shfl(py, (int)own), qz = __shfl(pz, (int)own);
                if (has) {
                    const uint32_t id = co[sb + (eb + (uint32_t)lane - soff)];
                    const float4 fa = filt[2 * id], fb = filt[2 * id + 1];
                    const bool may = ((double)fa.x < qx) & (qx < (double)fb.x) & ((double)fa.y < qy) &
                                     (qy < (double)fb.y) & ((double)fa.z < qz) & (qz < (double)fb.z);
                    if (may) {
                        const uint32_t slot = atomicAdd(qcount, 1u);
                        queue[slot] = (id << 11) | ((uint32_t)(k - 1) << 6) | own;
                    }
                }
                wave_lds_sync();
            }
            if (*qcount >= kFlushD32) flush();
        }
        flush();
        if (act) valid[i] = flags[lane] ? 1 : 0;
        wave_lds_sync();
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

int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// Persistent grid: at most `per_cu` resident 256-thread blocks per CU (LDS permitting),
// each looping over item groups, so the world is staged into LDS once per block.
int grid_for(int64_t groups, uint32_t lds_bytes) {
    const int64_t need = (groups + kBlock - 1) / kBlock;
    int per_cu = env_int("EPP_WG_PER_CU", 4);
    if (lds_bytes > 0)
        per_cu = std::max(1, std::min<int>(per_cu, (int)((160u * 1024u) / lds_bytes)));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
}

bool use_lds(const WorldView& w) {
    return w.blob_bytes <= kLdsBudget && !env_int("EPP_NO_LDS", 0) && !env_int("EPP_RAY_NO_LDS", 1);
}

// Opt a kernel in to more than 64 KB of dynamic LDS (static LDS counts against the same
// 160 KB).  A failure here must not linger as the thread's last HIP error.
template <typename K>
void allow_lds(K kernel, uint32_t static_bytes = 0) {
    // once per kernel and process (kernels of one signature share K, so key by address)
    static std::mutex mu;
    static std::set<const void*> done;
    const void* f = reinterpret_cast<const void*>(kernel);
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert(f).second) {
        const int dyn = (int)std::min<uint32_t>(kLdsBudget, 160u * 1024u - static_bytes);
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, dyn) != hipSuccess)
            (void)hipGetLastError();
    }
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

namespace {
// k_states_v5 stages [off_aos, blob_bytes) next to its wave queues
int v5_block(int dflt) {
    const int b = env_int("EPP_V5_BLOCK", dflt);
    return b == 256 ? 256 : (b == 512 ? 512 : 1024);
}
bool v5_fits(const WorldView& w) {
    const uint32_t q = queue5_bytes<1024>();
    return (w.blob_bytes - w.off_aos) + 16u + q <= 160u * 1024u && (w.blob_bytes - w.off_aos) <= kStageBudget &&
           !env_int("EPP_NO_LDS", 0);
}
int v5_cap() { return cu_count() * std::max(1, env_int("EPP_WG_PER_CU5", 1)); }

// Launch shape of k_states_v5.  Single pass (every lane one group): by default two
// 512-thread workgroups per CU when two staged copies fit in LDS (1M states: 8.3-8.4 us
// vs 8.7-8.8 us for one 1024-thread workgroup — each half of the CU syncs and stages on
// its own), else one 1024-thread workgroup.  More than one pass: 512 threads, the next
// group prefetched.  EPP_WG_PER_CU5 / EPP_V5_BLOCK / EPP_V5_SPL override (diagnostics).
struct V5Shape {
    bool spl8;
    int64_t gN;
    int bs, grid;
    bool pf;
};
V5Shape v5_shape(int64_t n, const uint8_t* valid, uint32_t sb) {
    V5Shape r{};
    const bool forced = env_int("EPP_WG_PER_CU5", 0) > 0 || env_int("EPP_V5_BLOCK", 0) > 0;
    const int64_t cap = v5_cap();
    r.spl8 = env_int("EPP_V5_SPL", 4) == 8 && (reinterpret_cast<uintptr_t>(valid) & 7) == 0 && n / 8 <= cap * 512;
    r.gN = n / (r.spl8 ? 8 : 4);
    const bool two = !forced && !r.spl8 && 2u * (sb + 16u + queue5_bytes<512>()) <= 160u * 1024u &&
                     r.gN <= 2 * (int64_t)cu_count() * 512;
    if (two) {
        r.bs = 512;
        r.grid = (int)std::max<int64_t>(1, (r.gN + 511) / 512);
        r.pf = false;
        return r;
    }
    const bool single = r.gN <= cap * (r.spl8 ? 512 : 1024);
    r.bs = v5_block(r.spl8 ? 512 : (single ? 1024 : 512));
    r.grid = (int)std::max<int64_t>(1, std::min<int64_t>((r.gN + r.bs - 1) / r.bs, cap));
    r.pf = r.gN > (int64_t)r.grid * r.bs;  // more than one group per lane
    return r;
}
bool v4_stage(const WorldView& w) {
    return (w.off_bitmap - w.off_aos) + sizeof(StateQueue4) <= 160u * 1024u && !env_int("EPP_NO_LDS", 0);
}
// resident workgroups only (every block loops): LDS-, register- and env-limited per CU
int v4_grid(const WorldView& w, int64_t n) {
    const int64_t items = std::max<int64_t>(1, n / 2);
    const int64_t need = (items + kBlock4 - 1) / kBlock4;
    const uint32_t lds = sizeof(StateQueue4) + (v4_stage(w) ? w.off_bitmap - w.off_aos : 0u);
    const int per_cu = std::max(1, std::min<int>(env_int("EPP_WG_PER_CU", 3), (int)((160u * 1024u) / lds)));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    return (int)std::max<int64_t>(1, std::min(need, cap));
}
bool v3_stage(const WorldView& w) {
    return (w.off_bitmap - w.off_aos) + (kBlock3 / 64) * sizeof(StateQueue3) <= 160u * 1024u &&
           !env_int("EPP_NO_LDS", 0);
}
// all resident waves at once: up to 4 workgroups of 512 per CU (LDS permitting)
int v3_grid(const WorldView& w, int64_t n) {
    const int64_t items = std::max<int64_t>(1, n / 2);
    const int64_t need = (items + kBlock3 - 1) / kBlock3;
    const uint32_t lds = (kBlock3 / 64) * sizeof(StateQueue3) + (v3_stage(w) ? w.off_bitmap - w.off_aos : 0u);
    const int per_cu = std::max(1, std::min<int>(env_int("EPP_WG_PER_CU", 4), (int)((160u * 1024u) / lds)));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    return (int)std::max<int64_t>(1, std::min(need, cap));
}
bool bm_stage(const WorldView& w) {
    return w.off_bitmap + (kBlock / 64) * sizeof(StateQueue) <= 160u * 1024u && !env_int("EPP_NO_LDS", 0);
}
int bm_grid(const WorldView& w, int64_t groups) {
    const uint32_t queue_bytes = (kBlock / 64) * sizeof(StateQueue);
    return grid_for(groups, bm_stage(w) ? w.off_bitmap + queue_bytes : queue_bytes);
}

template <bool MINDIST>
epp_status launch_states(const WorldView& w, const WorldView* dw, const double* xyz, int64_t n, int32_t can_pass, double md,
                         uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, void* stream,
                         unsigned long long* tl = nullptr) {
    // 16-byte loads and 4-byte flag stores need aligned buffers (hipMalloc gives 256 B)
    const bool aligned = ((reinterpret_cast<uintptr_t>(xyz) & 15) | (reinterpret_cast<uintptr_t>(valid) & 3)) == 0;
    const int64_t groups = std::max<int64_t>(1, n / 4);
    // Stage the whole world when it is small (keeps several blocks per CU), else only
    // the front (occupancy masks + cell starts) and read the OBB table through L1/L2.
    const bool lds = w.front_bytes + kScratchBytes <= kLdsBudget && !env_int("EPP_NO_LDS", 0);
    const uint32_t full_cap = (uint32_t)env_int("EPP_STAGE_FULL_MAX", 40 * 1024);
    const uint32_t stage = !lds ? 0u : (w.blob_bytes <= full_cap ? w.blob_bytes : w.front_bytes);
    const uint32_t shm = kScratchBytes + stage;
    const int grid = grid_for(groups, shm);
    hipStream_t st = (hipStream_t)stream;
    auto nv = reinterpret_cast<unsigned long long*>(n_valid);
#define EPP_LAUNCH_STATES(L, A)                                                                       \
    do {                                                                                              \
        allow_lds(k_states<L, MINDIST, A>);                                                           \
        hipLaunchKernelGGL((k_states<L, MINDIST, A>), dim3(grid), dim3(kBlock), shm, st, w, xyz, n,   \
                           can_pass, md, valid, compact_idx, nv, stage, tl);                          \
    } while (0)
    const int impl = env_int("EPP_STATES_IMPL", 5);
    if (impl == 5 && v5_fits(w) && (reinterpret_cast<uintptr_t>(xyz) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(valid) & 3) == 0) {
        const uint32_t sb = w.blob_bytes - w.off_aos;
        const int fast = env_int("EPP_V5_PAIRS", 1);
        // single pass over the states: 8 states per lane in 512-thread workgroups (half
        // the waves of 4 per lane: fewer executions of the per-wave fixed costs); more
        // than one pass: 4 per lane with the next group prefetched
        const V5Shape sh = v5_shape(n, valid, sb);
        const bool spl8 = sh.spl8, pf = sh.pf;
        const int64_t gN = sh.gN;
        const int bs = sh.bs, grid = sh.grid;
        // dynamic LDS: the staged world, optionally padded (EPP_V5_LDS_MIN bytes) so that
        // no more than the intended number of workgroups can share a CU
        const uint32_t dyn = std::max<uint32_t>(sb + 16, (uint32_t)std::max(0, env_int("EPP_V5_LDS_MIN", 0)));
#define EPP_LAUNCH_V5(C, T, B, P, S)                                                                              \
    do {                                                                                                          \
        allow_lds(k_states_v5<MINDIST, C, T, B, P, S>, queue5_bytes<B>());                                        \
        hipLaunchKernelGGL((k_states_v5<MINDIST, C, T, B, P, S>), dim3(grid), dim3(B), dyn, st, dw, xyz, gN, n,     \
                           can_pass, md, valid, compact_idx, nv, sb, fast, tl);                                   \
    } while (0)
#define EPP_LAUNCH_V5B(B, S)                                          \
    do {                                                              \
        if (pf) {                                                     \
            if (tl) EPP_LAUNCH_V5(false, true, B, true, S);           \
            else if (compact_idx) EPP_LAUNCH_V5(true, false, B, true, S); \
            else EPP_LAUNCH_V5(false, false, B, true, S);             \
        } else {                                                      \
            if (tl) EPP_LAUNCH_V5(false, true, B, false, S);          \
            else if (compact_idx) EPP_LAUNCH_V5(true, false, B, false, S); \
            else EPP_LAUNCH_V5(false, false, B, false, S);            \
        }                                                             \
    } while (0)
        if (spl8) {
            EPP_LAUNCH_V5B(512, 8);
        } else if (bs == 256) {
            EPP_LAUNCH_V5B(256, 4);
        } else if (bs == 512) {
            EPP_LAUNCH_V5B(512, 4);
        } else {
            EPP_LAUNCH_V5B(1024, 4);
        }
#undef EPP_LAUNCH_V5B
#undef EPP_LAUNCH_V5
        return launch_error(MINDIST ? "epp_check_states_mindist" : "epp_check_states");
    }
    if ((impl == 4 || impl == 5) && (reinterpret_cast<uintptr_t>(xyz) & 15) == 0 && (reinterpret_cast<uintptr_t>(valid) & 1) == 0 &&
        n / 2 < 0xFFFFFFFFll && !tl) {
        const uint32_t sb = w.off_bitmap - w.off_aos;
        const bool stg = v4_stage(w);
        const int g4 = v4_grid(w, n);
        const uint32_t items = (uint32_t)(n / 2);
#define EPP_LAUNCH_V4(S, C)                                                                             \
    do {                                                                                                \
        allow_lds(k_states_v4<MINDIST, S, C>, sizeof(StateQueue4));                                     \
        hipLaunchKernelGGL((k_states_v4<MINDIST, S, C>), dim3(g4), dim3(kBlock4), S ? sb : 0, st, dw, xyz, items, \
                           n, can_pass, md, valid, compact_idx, nv, sb);                                \
    } while (0)
        if (compact_idx) {
            if (stg) EPP_LAUNCH_V4(true, true);
            else EPP_LAUNCH_V4(false, true);
        } else {
            if (stg) EPP_LAUNCH_V4(true, false);
            else EPP_LAUNCH_V4(false, false);
        }
#undef EPP_LAUNCH_V4
        return launch_error(MINDIST ? "epp_check_states_mindist" : "epp_check_states");
    }
    if ((impl >= 3) && (reinterpret_cast<uintptr_t>(xyz) & 15) == 0 && (reinterpret_cast<uintptr_t>(valid) & 1) == 0) {
        const uint32_t sb = w.off_bitmap - w.off_aos;
        const bool stg = v3_stage(w);
        const int g3 = v3_grid(w, n);
#define EPP_LAUNCH_V3(S, C, T)                                                                          \
    do {                                                                                                \
        allow_lds(k_states_v3<MINDIST, S, C, T>, sizeof(StateQueue3) * (kBlock3 / 64));                 \
        hipLaunchKernelGGL((k_states_v3<MINDIST, S, C, T>), dim3(g3), dim3(kBlock3), S ? sb : 0, st, dw, xyz, \
                           n, can_pass, md, valid, compact_idx, nv, tl, sb);                            \
    } while (0)
        if (tl) {
            if (stg) EPP_LAUNCH_V3(true, false, true);
            else EPP_LAUNCH_V3(false, false, true);
        } else if (compact_idx) {
            if (stg) EPP_LAUNCH_V3(true, true, false);
            else EPP_LAUNCH_V3(false, true, false);
        } else {
            if (stg) EPP_LAUNCH_V3(true, false, false);
            else EPP_LAUNCH_V3(false, false, false);
        }
#undef EPP_LAUNCH_V3
        return launch_error(MINDIST ? "epp_check_states_mindist" : "epp_check_states");
    }
    if (impl != 0) {  // flat-bitmap kernel with prefetch (also the fallback for unaligned buffers)
        const uint32_t sb = w.off_bitmap;  // everything the exact path reads
        const bool stg = bm_stage(w);
        const int g2 = bm_grid(w, groups);
#define EPP_LAUNCH_BM(A, S)                                                                            \
    do {                                                                                               \
        allow_lds(k_states_bm<MINDIST, A, S>, (kBlock / 64) * sizeof(StateQueue));                    \
        hipLaunchKernelGGL((k_states_bm<MINDIST, A, S>), dim3(g2), dim3(kBlock), S ? sb : 0, st, dw, xyz, n, \
                           can_pass, md, valid, compact_idx, nv, tl, sb);                              \
    } while (0)
        if (aligned && stg) EPP_LAUNCH_BM(true, true);
        else if (aligned) EPP_LAUNCH_BM(true, false);
        else if (stg) EPP_LAUNCH_BM(false, true);
        else EPP_LAUNCH_BM(false, false);
#undef EPP_LAUNCH_BM
        return launch_error(MINDIST ? "epp_check_states_mindist" : "epp_check_states");
    }
    const int mode = stage == 0 ? 0 : (stage == w.blob_bytes ? 2 : 1);
    if (mode == 2 && aligned) EPP_LAUNCH_STATES(2, true);
    else if (mode == 2) EPP_LAUNCH_STATES(2, false);
    else if (mode == 1 && aligned) EPP_LAUNCH_STATES(1, true);
    else if (mode == 1) EPP_LAUNCH_STATES(1, false);
    else if (aligned) EPP_LAUNCH_STATES(0, true);
    else EPP_LAUNCH_STATES(0, false);
#undef EPP_LAUNCH_STATES
    return launch_error(MINDIST ? "epp_check_states_mindist" : "epp_check_states");
}
}  // namespace

extern "C" {

epp_status epp_check_states(const epp_world* world, const double* xyz, int64_t n,
                            int32_t can_pass_gate, uint8_t* valid, int32_t* compact_idx,
                            int64_t* n_valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid)) || (compact_idx && !n_valid)) {
        set_error("epp_check_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    return launch_states<false>(world_view(world), world_dview(world), xyz, n, can_pass_gate, 0.0, valid,
                                compact_idx, n_valid, stream);
}

epp_status epp_check_states_mindist(const epp_world* world, const double* xyz, int64_t n,
                                    double min_distance, uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid))) {
        set_error("epp_check_states_mindist: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    return launch_states<true>(world_view(world), world_dview(world), xyz, n, 0, min_distance, valid, nullptr,
                               nullptr, stream);
}

// Debug entry (not part of include/epp.h): k_states on C ABI arguments plus an 8-word
// per-wave timeline buffer (grid waves x 8 u64; see k_states).  Returns the grid size.
epp_status epp_dbg_states_timeline(const epp_world* world, const double* xyz, int64_t n, uint8_t* valid,
                                   unsigned long long* tl, int32_t* grid_waves, void* stream) {
    if (!world || n <= 0 || !xyz || !valid || !tl || !grid_waves) return EPP_ERR_INVALID_ARGUMENT;
    const WorldView& w = world_view(world);
    const bool lds = w.front_bytes + kScratchBytes <= kLdsBudget && !env_int("EPP_NO_LDS", 0);
    const uint32_t full_cap = (uint32_t)env_int("EPP_STAGE_FULL_MAX", 40 * 1024);
    const uint32_t stage = !lds ? 0u : (w.blob_bytes <= full_cap ? w.blob_bytes : w.front_bytes);
    const int impl = env_int("EPP_STATES_IMPL", 5);
    if (impl == 5 && v5_fits(w) && (reinterpret_cast<uintptr_t>(xyz) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(valid) & 3) == 0)
        *grid_waves = [&] {
            const V5Shape sh = v5_shape(n, valid, w.blob_bytes - w.off_aos);
            return sh.grid * (sh.bs / 64);
        }();
    else if (impl >= 3)  // (the timeline runs k_states_v3 for impl 4 too)
        *grid_waves = v3_grid(w, n) * (kBlock3 / 64);
    else
        *grid_waves = (impl == 1 ? bm_grid(w, std::max<int64_t>(1, n / 4))
                                 : grid_for(std::max<int64_t>(1, n / 4), kScratchBytes + stage)) *
                      (kBlock / 64);
    return launch_states<false>(w, world_dview(world), xyz, n, 0, 0.0, valid, nullptr, nullptr, stream, tl);
}

epp_status epp_check_motions(const epp_world* world, const double* s1, const double* s2, int64_t n,
                             int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!s1 || !s2 || !valid)) || (mode != 0 && mode != 1)) {
        set_error("epp_check_motions: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const WorldView& w = world_view(world);
    hipStream_t st0 = (hipStream_t)stream;
    {
        // LDS-resident variant: coarse grid + lists (blob up to `meta`) and the records
        const uint32_t front = w.off_meta;
        const uint32_t recb = (uint32_t)(((size_t)w.n_obb * kRecDoubles * 8 + 15) & ~size_t(15));
        const int impl = env_int("EPP_MOTIONS_IMPL", 5);  // 5: v4 analytic + d32b discrete32
        // pair-queue kernels (v3/v4 analytic, d32q discrete32) unless v2 is asked for
        const bool v3 = impl == 3 || impl == 4 || impl == 5;
        const bool v4 = (impl == 4 || impl == 5) && mode == 0;
        const bool d32b = impl == 5 && mode == 1;  // (analytic under impl 5: v4)
        auto extra_for = [&](int blk) -> uint32_t {
            return v4     ? (uint32_t)((blk / 64) * ((kQueueM + 1) * 4 + 64 + 256) + (uint32_t)w.n_obb * 32u)
                   : d32b ? (uint32_t)((blk / 64) * ((kQueueD32 + 1) * 4 + 64 + 256) + (uint32_t)w.n_obb * 32u)
                   : v3 ? (uint32_t)((blk / 64) * (((mode == 0 ? kQueueM : kQueueD32) + 1) * 4 + 64) +
                                     (mode == 0 ? (uint32_t)w.n_obb * 32u : 0u))
                        : 0u;
        };
        // Block size: 512 threads when two such blocks fit a CU's LDS (small worlds: C4's
        // 64 OBBs, v4 28 vs 32 us per 1M edges), else 1024 (C3's 512 OBBs stage ~95 KB, one
        // block per CU, and 1024 threads double the waves behind the LDS walk: v4 52 vs 69 us)
        const int eb = env_int("EPP_MOTIONS_BLOCK", 0);
        const int block = eb == 512 ? 512 : eb == 1024 ? 1024
                                           : (2u * (front + recb + extra_for(512)) <= 160u * 1024u ? 512 : 1024);
        const uint32_t extra = extra_for(block);
        if ((impl == 2 || v3) && front % 16 == 0 && front + recb + extra <= 160u * 1024u &&
            !env_int("EPP_NO_LDS", 0)) {
            const uint32_t shm = front + recb + extra;
            const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + block - 1) / block, (int64_t)cu_count() *
                                                    std::max(1, (int)((160u * 1024u) / shm))));
            const WorldView* dw = world_dview(world);
#define EPP_LAUNCH_M(KERNEL)                                                                                  \
    do {                                                                                                      \
        allow_lds(KERNEL);                                                                                    \
        hipLaunchKernelGGL(KERNEL, dim3(grid), dim3(block), shm, st0, dw, s1, s2, n, can_pass_gate, valid, front, \
                           recb);                                                                             \
    } while (0)
            if (v4) {
                if (block == 1024) EPP_LAUNCH_M((k_motions_v4<1024>));
                else EPP_LAUNCH_M((k_motions_v4<512>));
            } else if (d32b) {
                if (block == 1024) EPP_LAUNCH_M((k_motions_d32b<1024>));
                else EPP_LAUNCH_M((k_motions_d32b<512>));
            } else if (v3 && mode == 0) {
                if (block == 1024) EPP_LAUNCH_M((k_motions_v3<1024>));
                else EPP_LAUNCH_M((k_motions_v3<512>));
            } else if (v3) {
                if (block == 1024) EPP_LAUNCH_M((k_motions_d32q<1024>));
                else EPP_LAUNCH_M((k_motions_d32q<512>));
            } else if (mode == 0) {
                if (block == 1024) EPP_LAUNCH_M((k_motions_v2<0, 1024>));
                else EPP_LAUNCH_M((k_motions_v2<0, 512>));
            } else {
                if (block == 1024) EPP_LAUNCH_M((k_motions_v2<1, 1024>));
                else EPP_LAUNCH_M((k_motions_v2<1, 512>));
            }
#undef EPP_LAUNCH_M
            return launch_error("epp_check_motions");
        }
    }
    const int aligned =
        ((reinterpret_cast<uintptr_t>(s1) | reinterpret_cast<uintptr_t>(s2)) & 15) == 0;
    const int64_t groups = (n + 3) / 4;
    const bool lds = use_lds(w);
    const uint32_t shm = lds ? w.blob_bytes : 0;
    const int grid = grid_for(groups, shm);
    hipStream_t st = (hipStream_t)stream;
    if (lds) {
        allow_lds(k_motions<true, 0>);
        allow_lds(k_motions<true, 1>);
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

// collision_common.h — device helpers shared by the OBB validity kernels (states.hip,
// motions.hip) and their host-side launch helpers.
//
// All decision arithmetic is IEEE fp64 with contraction disabled (-ffp-contract=off), in
// the reference's evaluation order, so the booleans match the reference bit for bit:
//   OBB::checkCollisionWithPoint  src/OBB.cpp:63-91   (obb_point_hit, rec_hit)
//   OBB::checkCollisionWithRay    src/OBB.cpp:10-61   (obb_ray_hit, rec_ray_hit)
//   World::checkPointValidity     src/World.cpp:80-128 (point_valid, states_exact_rec)
//   World::checkRayValid          src/World.cpp:130-162 (ray_valid)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>

#include "epp_internal.h"

namespace epp {
SmallWorld small_world(const epp_world* w);
epp_status note_record_reader(const epp_world* w, const SmallWorld& sw, hipStream_t st);  // async reader of sw.recs

// small.hip: brute-force kernels for small queries (no index needed)
constexpr int64_t kSmallStates = 4096;   // states per call
constexpr int64_t kSmallMotions = 1024;  // edges per call
constexpr int kSmallMaxObbs = 256;       // OBBs (records staged in LDS: 34 KB)
bool small_states(const SmallWorld& sw, int64_t n);
bool small_motions(const SmallWorld& sw, int64_t n);
// done != NULL: each workgroup publishes seq in done[blockIdx.x] when its flags are visible
epp_status launch_states_small(const SmallWorld& sw, bool mindist, const double* xyz, int64_t n, int32_t can_pass,
                               double md, uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, hipStream_t st,
                               uint32_t* done = nullptr, uint32_t seq = 0);
epp_status launch_motions_small(const SmallWorld& sw, int32_t mode, const double* s1, const double* s2, int64_t n,
                                int32_t can_pass, uint8_t* valid, hipStream_t st, uint32_t* done = nullptr,
                                uint32_t seq = 0);

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

// The 32-step discretised motion check against ONE OBB record: does some point
// s + (e - s) k/32, k = 1..32, lie strictly inside the OBB's AABB (rtree contains,
// src/World.cpp:83) and collide with it (OBB::checkCollisionWithPoint, src/OBB.cpp:63-91;
// filling boxes skipped with can_pass, :92-95)?  Every one of those tests is |a + b t| <= h
// (or lo < a + b t < hi) along the edge, so the t that can hit lie in an interval; it is
// computed with a slack eta (1e-6 m + 1e-12 of the coordinates' magnitude) far above the
// rounding of the points and of the interval itself, and only the k inside it are tested
// exactly (the reference's point evaluation), in order, until one hits.
__device__ __forceinline__ bool d32_pair_hit(const double* rec, const double ps[3], const double pe[3], double rg,
                                             double ro, bool cp) {
    double rr[kRecDoubles];  // the record in registers
#pragma unroll
    for (int k = 0; k <= F_HZ; ++k) rr[k] = rec[k];
    rr[R_META] = rec[R_META];
    const uint32_t m = (uint32_t)__double_as_longlong(rr[R_META]);
    const bool fillb = (m & META_FILLING) != 0u;
    const double r = (m & META_GATE) ? rg : ro;
    const double d[3] = {pe[0] - ps[0], pe[1] - ps[1], pe[2] - ps[2]};
    const double mag = fmax(fmax(fmax(fabs(ps[0]), fabs(ps[1])), fmax(fabs(ps[2]), fabs(pe[0]))),
                            fmax(fmax(fabs(pe[1]), fabs(pe[2])), fmax(fmax(fabs(rr[F_CX]), fabs(rr[F_CY])), fabs(rr[F_CZ]))));
    const double eta = 1e-6 + 1e-12 * mag;
    double t0 = 0.0, t1 = 1.0;
    // lo - eta <= a + b t <= hi + eta
    auto clip = [&](double a, double b, double lo, double hi) {
        const double u0 = lo - eta - a, u1 = hi + eta - a;
        if (b == 0.0) {
            if (!(u0 <= 0.0 && 0.0 <= u1)) t1 = -1.0;
        } else {
            // (a bound, not a decision: the reciprocal by v_rcp_f64 and one Newton step,
            // ~1e-15 relative, far inside the slack eta)
            double ib = __builtin_amdgcn_rcp(b);
            ib = fma(ib, fma(-b, ib, 1.0), ib);
            const double v0 = u0 * ib, v1 = u1 * ib;
            t0 = fmax(t0, fmin(v0, v1));
            t1 = fmin(t1, fmax(v0, v1));
        }
    };
    clip(ps[0], d[0], rr[F_LOX], rr[F_HIX]);  // rtree contains (strict)
    clip(ps[1], d[1], rr[F_LOY], rr[F_HIY]);
    clip(ps[2], d[2], rr[F_LOZ], rr[F_HIZ]);
    const double c = rr[F_COS], sn = rr[F_SIN];  // the OBB frame
    const double ax = ps[0] - rr[F_CX], ay = ps[1] - rr[F_CY];
    const double tx = fillb ? rr[F_HX] : rr[F_HX] + r, ty = fillb ? rr[F_HY] : rr[F_HY] + r,
                 tz = fillb ? rr[F_HZ] : rr[F_HZ] + r;
    clip(c * ax + sn * ay, c * d[0] + sn * d[1], -tx, tx);
    clip(c * ay - sn * ax, c * d[1] - sn * d[0], -ty, ty);
    clip(ps[2] - rr[F_CZ], d[2], -tz, tz);
    int k0 = 33, k1 = 0;
    if (t0 <= t1) {  // (NaN bounds: fmax/fmin drop them -> the whole edge)
        k0 = max(1, (int)ceil(32.0 * t0));
        k1 = min(32, (int)floor(32.0 * t1));
    }
    bool hit = false;
    for (int k = k0; k <= k1 && !hit; ++k) {
        const double t = (double)k / 32.0;
        const double qx = ps[0] + (pe[0] - ps[0]) * t;
        const double qy = ps[1] + (pe[1] - ps[1]) * t;
        const double qz = ps[2] + (pe[2] - ps[2]) * t;
        hit = rec_hit<false>(rr, rg, ro, qx, qy, qz, cp, 0.0);
    }
    return hit;
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
        // std::min / std::max as v_min_f64 / v_max_f64 (one instruction instead of a compare
        // and two 32-bit selects).  Same decisions: t1 and t2 are NaN together (a NaN
        // endpoint or invD) and minNum/maxNum then keep tMin / tMax as the selects do; they
        // may differ only in the sign of a zero, which no comparison below sees.
        const double tEntry = fmin(t1, t2);  // std::min
        const double tExit = fmax(t1, t2);   // std::max
        const double nMin = fmax(tMin, tEntry);
        const double nMax = fmin(tExit, tMax);
        rejected = rejected | (par & outside) | (!par & (nMin > nMax));
        tMin = par ? tMin : nMin;
        tMax = par ? tMax : nMax;
    }
    const bool slab_hit = !rejected & (0 <= tMin) & (tMin <= 1) & (0 <= tMax) & (tMax <= 1);  // :60
    return end_hit | slab_hit;
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

// integer environment variable (test hooks only)
int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// Persistent grid: at most `per_cu` resident 256-thread blocks per CU (LDS permitting),
// each looping over item groups, so the world is staged into LDS once per block.
int grid_for(int64_t groups, uint32_t lds_bytes) {
    const int64_t need = (groups + kBlock - 1) / kBlock;
    int per_cu = 4;
    if (lds_bytes > 0)
        per_cu = std::max(1, std::min<int>(per_cu, (int)((160u * 1024u) / lds_bytes)));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    int64_t g = need < cap ? need : cap;
    return (int)(g < 1 ? 1 : g);
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

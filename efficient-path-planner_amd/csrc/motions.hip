// motions.hip — batched motion (edge) validity checks for gfx950 (MI355X).
//
//   World::checkRayValid(s, e, canPassGate)  src/World.cpp:130-162, via
//   OBB::checkCollisionWithRay               src/OBB.cpp:10-61        (mode 0, analytic)
//   32-step discretised check                BASELINE config 3         (mode 1; points
//   s + (e - s) k/32, k = 1..32, each World::checkPointValidity(p, canPassGate))
//
// Kernels, chosen by what fits (epp_check_motions):
//   k_motions_small  batches of <= 1024 edges on worlds of <= 256 OBBs (small.hip);
//   k_motions_v5     both modes, tile/slab bit-set candidate filter (records and tile rows
//                    in LDS; worlds of <= 1024 OBBs per tile) — the default;
//   k_motions_v4     analytic, coarse grid + records in LDS, lane-balanced list walk;
//   k_motions_d32b   discrete32, same staging, lane-balanced list walk per step;
//   k_motions        generic (worlds too large for LDS): one lane per edge, L2-resident world.
#include "collision_common.h"

namespace epp {
namespace {

// Generic kernel (worlds whose coarse grid + records exceed LDS): one lane per edge, four
// edges per lane and iteration, the world read through L1/L2.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_motions(WorldView w, const double* __restrict__ s1,
                                                    const double* __restrict__ s2, int64_t n,
                                                    int can_pass, uint8_t* __restrict__ valid,
                                                    int aligned) {
    const Acc a = make_acc(w.blob, w.blob, w);
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

constexpr int kQueueM = 256;  // queued (edge, OBB) pairs per wave

// Per-wave time split of k_motions_v4 (diagnostics builds only: -DEPP_MOTIONS_TL, see
// scripts/motions_timeline.py): shader-clock cycles spent in the level-1/2 walk, in the
// flushes, and in total, plus the pairs walked / queued.
#ifdef EPP_MOTIONS_TL
constexpr int kMtlWaves = 1 << 16;
__device__ unsigned long long g_motions_tl[kMtlWaves][6];
#define EPP_MTL_DECL unsigned long long tl_walk = 0, tl_flush = 0, tl_t0 = __builtin_readcyclecounter(), tl_e = 0, tl_q = 0, tl_c = 0
#define EPP_MTL_ADD(v, t) v += __builtin_readcyclecounter() - (t)
#define EPP_MTL_NOW(t) const unsigned long long t = __builtin_readcyclecounter()
#define EPP_MTL_CNT(v, x) v += (x)
#define EPP_MTL_END                                                                                   \
    do {                                                                                              \
        const int w_ = (int)((blockIdx.x * BLOCK + threadIdx.x) >> 6);                               \
        if (lane == 0 && w_ < kMtlWaves) {                                                           \
            g_motions_tl[w_][0] = tl_walk; g_motions_tl[w_][1] = tl_flush;                            \
            g_motions_tl[w_][2] = __builtin_readcyclecounter() - tl_t0; g_motions_tl[w_][3] = tl_e;   \
            g_motions_tl[w_][4] = tl_q; g_motions_tl[w_][5] = tl_c;                                   \
        }                                                                                             \
    } while (0)
#else
#define EPP_MTL_DECL
#define EPP_MTL_ADD(v, t)
#define EPP_MTL_NOW(t)
#define EPP_MTL_CNT(v, x)
#define EPP_MTL_END
#endif

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
    EPP_MTL_DECL;
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
            EPP_MTL_NOW(tf);
            const uint32_t total = *qcount;
            EPP_MTL_CNT(tl_q, total);
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
            EPP_MTL_ADD(tl_flush, tf);
        };

        EPP_MTL_NOW(tw);
        EPP_MTL_CNT(tl_c, total_c);
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
            EPP_MTL_CNT(tl_e, total_e);
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
        EPP_MTL_ADD(tl_walk, tw);
        flush();
        if (act) valid[i] = flags[lane] ? 1 : 0;
        wave_lds_sync();
    }
    EPP_MTL_END;
}

constexpr int kQueueD32 = 512;
constexpr uint32_t kFlushD32 = 256;

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

// ---- k_motions_v5: tile/slab-filtered motion checks ------------------------------------
// The candidate set of an edge is a bit set over a tile's OBBs, computed without walking
// any cell list.  Per axis k the edge's box [lo_k, hi_k] maps to global slabs [a_k, b_k]
// (slab_axis: monotone, so an AABB overlap in doubles implies a slab overlap); x and y
// slabs group into T x T tiles of S slabs.  In each tile the box reaches,
//   cand = AND_k  LE_k[b_k] & GE_k[a_k]        (local slabs, clamped into the tile)
// are the tile's OBBs whose slab-rounded AABB overlaps the edge's — together a superset of
// the rtree query of World::checkRayValid (src/World.cpp:130-162).  An OBB in several of
// those tiles is kept only in the first one along each axis (FX / FY rows), with
// can_pass_gate the filling OBBs are masked out (:150-153).  The (edge, OBB) pairs go to
// the wave's queue at offsets from a wave scan of the lanes' popcounts and are tested 64
// at a time behind an exact AABB prefilter in doubles (the rtree's closed overlap; for
// MODE 0 in the queued test, for MODE 1 before queueing):
//   MODE 0  OBB::checkCollisionWithRay (src/OBB.cpp:10-61);
//   MODE 1  the points s + (e - s) k/32, k = 1..32 (d32_pair_hit: only the k an interval
//           bound admits are evaluated exactly).  The slab range and the prefilter box are
//           widened by a hair, so points rounded past the edge's box stay covered.
// An edge is invalid iff some pair hits — the reference's answer.
constexpr int kQueueV5 = 256;

// IDX: the edges are given as a k-NN table instead of endpoint arrays — edge e runs from
// node e / kk to node nbr[e] (s1 = the nodes; a missing neighbour, -1, is the degenerate
// edge from the node to itself), as epp_knn_edges would lay them out.
//
// MotionMask (IDX, count != nullptr): the planner's edge mask folded in -- a failed motion's
// table entry becomes -1, out16 (if given) receives the masked table as u16 (0xFFFF: no
// edge), and count[0] / count[1] gain the kept edges / those into node `target` (one atomic
// per workgroup), as k_mask_edges_count (planner.hip) would after the launch.
template <int W, int MODE, bool IDX>
__global__ __launch_bounds__(1024) void k_motions_v5(const WorldView* __restrict__ wv, const double* __restrict__ s1,
                                                     const double* __restrict__ s2, const int32_t* __restrict__ nbr,
                                                     int kk, int64_t n, int can_pass, uint8_t* __restrict__ valid,
                                                     uint32_t rec_bytes, uint32_t tile_bytes, MotionMask mm) {
    constexpr int BLOCK = 1024;
    constexpr int STRIDE = slab_row_stride(W);
    // PF: the exact AABB prefilter in the queued test instead of the candidate rounds --
    // the analytic mode (a candidate round then costs a bit-pick and an append; the queued
    // ray test pays the 6 compares with every lane busy): 29.2-29.9 -> 28.7-29.2 us at C3.
    // Discrete32 keeps it in the rounds: there the 12 % more queued pairs reach the heavier
    // d32 test (35.9 -> 38.7 us with it in the queue).
#if defined(EPP_MOTIONS_PF_FLUSH)
    constexpr bool PF = true;  // (A/B: both modes)
#else
    constexpr bool PF = MODE == 0;
#endif
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    EPP_MTL_DECL;
    {
        // records and tile rows: up to 8 16-byte loads per thread in flight before the
        // first store (a load -> store loop would wait out one L2 round trip per chunk)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* src0 = reinterpret_cast<const u32x4*>(wv->blob + wv->off_aos);
        const u32x4* src1 = reinterpret_cast<const u32x4*>(wv->blob + wv->off_slab);
        u32x4* dst = reinterpret_cast<u32x4*>(lds);
        const uint32_t n0 = rec_bytes / 16, n1 = tile_bytes / 16, nt = n0 + n1;
        constexpr int U = 8;
        for (uint32_t b = threadIdx.x; b < nt; b += U * BLOCK) {
            u32x4 r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {  // (unconditional loads: clamped in range)
                const uint32_t o = min(b + u * BLOCK, nt - 1);
                r[u] = *(o < n0 ? src0 + o : src1 + (o - n0));
            }
#pragma unroll
            for (int u = 0; u < U; ++u)  // (past the end: the last chunk again, same bytes)
                dst[min(b + u * BLOCK, nt - 1)] = r[u];
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double* recs = reinterpret_cast<const double*>(lds);
    const uint32_t* tiles = reinterpret_cast<const uint32_t*>(lds + rec_bytes);
    constexpr uint32_t kWaveBytes = kQueueV5 * 4 + 64;
    unsigned char* wbase = lds + rec_bytes + tile_bytes + wave * kWaveBytes;
    uint32_t* queue = reinterpret_cast<uint32_t*>(wbase);
    uint8_t* flags = wbase + kQueueV5 * 4;
    const int S = wv->slab_n, SL = wv->slab_log, T = wv->tile_n;
    const uint32_t TW = wv->tile_words;
    const int G[3] = {T * S, T * S, S};
    const float sof[3] = {wv->sofx, wv->sofy, wv->sofz}, sinv[3] = {wv->six, wv->siy, wv->siz};
    const double rg = wv->r_gate, ro = wv->r_obst;
    const bool cp = can_pass != 0;
    // (the planner batch's per-problem counts: kept edges, those into the goal)
    [[maybe_unused]] uint32_t* s_pk = nullptr;
    [[maybe_unused]] uint32_t* s_pg = nullptr;
    if constexpr (IDX) {
        __shared__ uint32_t s_pcnt[2][64];
        s_pk = s_pcnt[0];
        s_pg = s_pcnt[1];
        if (mm.mark && threadIdx.x < 64) s_pk[threadIdx.x] = s_pg[threadIdx.x] = 0u;
    }
    __syncthreads();
#ifdef EPP_MOTIONS_TL
    tl_c = __builtin_readcyclecounter() - tl_t0;  // staging
#endif
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    uint32_t mk_keep = 0, mk_tgt = 0;  // (MotionMask counts)
    // (packed rows: only the first *rows_n rows hold a table row)
    const int64_t ne = (IDX && mm.rows_n) ? min(n, (int64_t)min(*mm.rows_n, (unsigned long long)(n / kk)) * kk) : n;
    for (int64_t i0 = (int64_t)blockIdx.x * BLOCK + wave * 64; i0 < ne; i0 += stride) {
        const int64_t i = i0 + lane;
        const bool act = i < ne;
        double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
        int32_t jraw = -1;  // (IDX: the table entry)
        if (act) {
            if (IDX) {
                const int64_t u = mm.rowmap ? (int64_t)mm.rowmap[i / kk] : i / kk;
                const int32_t j = nbr[i];
                jraw = j;
                const int64_t v = j < 0 ? u : (int64_t)j;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    s[k] = s1[3 * u + k];
                    e[k] = s1[3 * v + k];
                }
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    s[k] = s1[3 * i + k];
                    e[k] = s2[3 * i + k];
                }
            }
        }
        flags[lane] = 1;
        EPP_MTL_NOW(tl_b);
        int ga[3], gb[3];
        double blo[3], bhi[3];  // the edge's box (rtree query box, World.cpp:137-141)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double lo = (e[k] < s[k]) ? e[k] : s[k];
            const double hi = (s[k] < e[k]) ? e[k] : s[k];
            blo[k] = MODE == 1 ? lo - (1e-9 + 1e-12 * fabs(lo)) : lo;
            bhi[k] = MODE == 1 ? hi + (1e-9 + 1e-12 * fabs(hi)) : hi;
            ga[k] = slab_axis(lo, sof[k], sinv[k], G[k]);
            gb[k] = slab_axis(hi, sof[k], sinv[k], G[k]);
            if (MODE == 1) {
                ga[k] = ga[k] > 0 ? ga[k] - 1 : 0;
                gb[k] = gb[k] < G[k] - 1 ? gb[k] + 1 : G[k] - 1;
            }
        }
        const int tx0 = ga[0] >> SL, ty0 = ga[1] >> SL;
        const int ntx = (gb[0] >> SL) - tx0 + 1;
        const int ntiles = act ? ntx * ((gb[1] >> SL) - ty0 + 1) : 0;
        uint32_t qn = 0;  // queued pairs (wave-uniform)
        auto flush = [&]() {
            EPP_MTL_NOW(tl_f);
            wave_lds_sync();  // the appends are visible
            for (uint32_t base = 0; base < qn; base += 64) {
                const uint32_t jq = base + lane;
                const bool has = jq < qn;
                const uint32_t q = has ? queue[jq] : 0u;
                const int owner = (int)(q & 63u);
                double ps[3], pe[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    ps[k] = __shfl(s[k], owner);
                    pe[k] = __shfl(e[k], owner);
                }
                if (has) {
                    const double* rec = recs + (size_t)(q >> 6) * kRecDoubles;
                    bool hit;
                    bool keep = true;  // (PF false: tested before queueing)
                    if constexpr (PF) {
                        // the exact AABB prefilter here, on the owner's box (closed, as the
                        // rtree query; MODE 1 widened by a hair), instead of in the rounds
#pragma unroll
                        for (int k = 0; k < 3; ++k) {
                            const double l = (pe[k] < ps[k]) ? pe[k] : ps[k], h = (ps[k] < pe[k]) ? pe[k] : ps[k];
                            const double bl = MODE == 1 ? l - (1e-9 + 1e-12 * fabs(l)) : l;
                            const double bh = MODE == 1 ? h + (1e-9 + 1e-12 * fabs(h)) : h;
                            keep = keep & !((rec[F_HIX + k] < bl) | (bh < rec[F_LOX + k]));
                        }
                    }
                    if (MODE == 0) {  // (the AABB overlap: `keep`, tested above)
                        const uint32_t m = (uint32_t)__double_as_longlong(rec[R_META]);
                        hit = keep && rec_ray_hit(rec, ps, pe, (m & META_GATE) ? rg : ro);
                    } else {
                        hit = keep && d32_pair_hit(rec, ps, pe, rg, ro, cp);
                    }
                    if (hit) flags[owner] = 0;
                }
            }
            wave_lds_sync();
            qn = 0;
            EPP_MTL_ADD(tl_flush, tl_f);
        };
        // Candidate words of tile j (0 <= j < ntiles) of this lane's edge; returns the
        // tile's OBB ids.  An OBB in several of the box's tiles is kept in its first tile
        // along x and y only (FX / FY rows), filling OBBs are dropped with can_pass_gate.
        auto tile_cand = [&](int j, uint32_t (&cand)[W]) __attribute__((always_inline)) -> const uint16_t* {
            int tx = tx0, ty = ty0;
            if (j == 1) {
                tx = ntx > 1 ? tx0 + 1 : tx0;
                ty = ntx > 1 ? ty0 : ty0 + 1;
            } else if (j > 1) {
                tx = tx0 + j % ntx;
                ty = ty0 + j / ntx;
            }
            const uint32_t* tile = tiles + (size_t)(ty * T + tx) * TW;
            const int la[3] = {min(max(ga[0] - (tx << SL), 0), S - 1), min(max(ga[1] - (ty << SL), 0), S - 1), ga[2]};
            const int lb[3] = {min(max(gb[0] - (tx << SL), 0), S - 1), min(max(gb[1] - (ty << SL), 0), S - 1), gb[2]};
#pragma unroll
            for (int w = 0; w < W; ++w) cand[w] = ~0u;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t* le = tile + ((2 * k) * S + lb[k]) * STRIDE;
                const uint32_t* ge = tile + ((2 * k + 1) * S + la[k]) * STRIDE;
#pragma unroll
                for (int w = 0; w < W; ++w) cand[w] &= le[w] & ge[w];
            }
            const uint32_t* tail = tile + 6 * S * STRIDE;
            const uint32_t fx = tx > tx0 ? ~0u : 0u, fy = ty > ty0 ? ~0u : 0u, fl = cp ? ~0u : 0u;
#pragma unroll
            for (int w = 0; w < W; ++w) cand[w] &= (tail[w] | ~fx) & (tail[W + w] | ~fy) & ~(tail[2 * W + w] & fl);
            return reinterpret_cast<const uint16_t*>(tail + 3 * W);
        };
        // Tiles are taken two at a time (the second is where an edge crossing one tile
        // boundary continues; more is rare).  One wave-uniform loop then walks every
        // lane's candidates, one per lane and round: the exact prefilter in doubles drops
        // the OBBs whose AABB misses the edge's box (closed, as the rtree query; MODE 1:
        // the box widened by a hair, since a rounded point may sit an ulp past it), and the
        // survivors are appended to the wave's queue at ballot ranks.
        for (int jp = 0;; jp += 2) {
            if (!__builtin_amdgcn_ballot_w64(jp < ntiles)) break;
            uint32_t ca[W], cb[W];
            const uint16_t* ida = nullptr;
            const uint16_t* idb = nullptr;
#pragma unroll
            for (int w = 0; w < W; ++w) ca[w] = cb[w] = 0u;
            if (jp < ntiles) ida = tile_cand(jp, ca);
            if (jp + 1 < ntiles) idb = tile_cand(jp + 1, cb);
            EPP_MTL_NOW(tl_p);
#ifndef EPP_MOTIONS_ROUNDS  // (A/B: the one-candidate-per-lane rounds for the analytic mode too)
            if constexpr (PF && W <= 2) {  // (wider rows: the rounds, whose registers fit)
                // Every candidate queued at once: a wave scan of the lanes' candidate counts
                // gives each lane its queue slots, and each lane writes its own (a loop as
                // long as the busiest lane's count, a few instructions per entry) instead of
                // one candidate per lane and round through the wave (~27 instructions per
                // round).  The order of the queue does not change the answer (any hit).
                uint32_t c = 0;
#pragma unroll
                for (int w = 0; w < W; ++w) c += (uint32_t)(__popc(ca[w]) + __popc(cb[w]));
                uint32_t tot;
                const uint32_t off = wave_excl_scan(c, lane, tot);
                if (tot > 0u && tot <= (uint32_t)kQueueV5) {  // wave-uniform
                    if (qn + tot > (uint32_t)kQueueV5) flush();
                    uint32_t at = qn + off;
#pragma unroll
                    for (int w = 0; w < 2 * W; ++w) {
                        uint32_t cw = w < W ? ca[w] : cb[w - W];
                        const uint16_t* tid = w < W ? ida : idb;  // (non-null whenever cw != 0)
                        while (cw) {
                            const uint32_t bit = (uint32_t)__builtin_ctz(cw);
                            cw &= cw - 1u;
                            queue[at++] = (uint32_t)tid[32 * (w % W) + bit] << 6 | (uint32_t)lane;
                        }
                    }
                    qn += tot;
                    if (qn > (uint32_t)(kQueueV5 - 64)) flush();
                    EPP_MTL_ADD(tl_e, tl_p);
                    continue;
                }
                if (tot == 0u) {
                    EPP_MTL_ADD(tl_e, tl_p);
                    continue;
                }
                // (more candidates than the queue holds: the rounds below)
            }
#endif
#ifdef EPP_MOTIONS_W1MASK  // (A/B) one-word tiles: both tiles' candidates as one 64-bit mask
            uint64_t cm = W == 1 ? ((uint64_t)ca[0] | ((uint64_t)cb[0] << 32)) : 0ull;
#endif
            for (;;) {
                bool has = false;
                uint32_t wsel = 0, bit = 0;
#ifdef EPP_MOTIONS_W1MASK
                if (W == 1) {
                    has = cm != 0ull;
                    const uint32_t b64 = (uint32_t)__builtin_ctzll(cm | (1ull << 63));
                    cm &= cm - 1ull;
                    wsel = b64 >> 5;
                    bit = b64 & 31u;
                } else
#endif
#pragma unroll
                for (int w = 0; w < 2 * W; ++w) {
                    uint32_t& cw = w < W ? ca[w] : cb[w - W];
                    const bool take = !has && cw != 0u;
                    if (take) {
                        wsel = (uint32_t)w;
                        bit = (uint32_t)__builtin_ctz(cw);
                        cw &= cw - 1u;
                    }
                    has = has || take;
                }
                if constexpr (PF) {  // every candidate queued; the prefilter runs in the flush
                    const unsigned long long hb = __builtin_amdgcn_ballot_w64(has);
                    if (!hb) break;
                    if (has) {
                        const uint16_t* tid = wsel < (uint32_t)W ? ida : idb;
                        queue[qn + lanes_below(hb)] = (uint32_t)tid[32 * (wsel % (uint32_t)W) + bit] << 6 | (uint32_t)lane;
                    }
                    qn += (uint32_t)__popcll(hb);
                    if (qn > (uint32_t)(kQueueV5 - 64)) flush();
                    continue;
                }
                if (!__builtin_amdgcn_ballot_w64(has)) break;
                uint32_t id = 0;
                bool keep = false;
                if (has) {
                    const uint16_t* tid = wsel < (uint32_t)W ? ida : idb;
                    id = tid[32 * (wsel % (uint32_t)W) + bit];
                    const double* rec = recs + (size_t)id * kRecDoubles;
                    keep = !((rec[F_HIX] < blo[0]) | (bhi[0] < rec[F_LOX]) | (rec[F_HIY] < blo[1]) |
                             (bhi[1] < rec[F_LOY]) | (rec[F_HIZ] < blo[2]) | (bhi[2] < rec[F_LOZ]));
                }
                const unsigned long long kb = __builtin_amdgcn_ballot_w64(keep);
                if (keep) queue[qn + lanes_below(kb)] = id << 6 | (uint32_t)lane;
                qn += (uint32_t)__popcll(kb);
                EPP_MTL_CNT(tl_q, (uint32_t)__popcll(kb));
                if (qn > (uint32_t)(kQueueV5 - 64)) flush();
            }
            EPP_MTL_ADD(tl_e, tl_p);
        }
        EPP_MTL_ADD(tl_walk, tl_b);
        flush();
        if (act) valid[i] = flags[lane];
        if (IDX && (mm.count || mm.out16)) {  // (launch-uniform)
            const bool keep = act && flags[lane] != 0 && jraw >= 0;
            if (act && flags[lane] == 0) mm.nbr_w[i] = -1;
            if (act && mm.out16) mm.out16[i] = keep ? (uint16_t)jraw : (uint16_t)0xFFFF;
            mk_keep += keep ? 1u : 0u;
            mk_tgt += (keep && jraw == mm.target) ? 1u : 0u;
            if (mm.mark && act) {  // (launch-uniform) the planner batch's marks and counts
                const int32_t u = mm.rowmap[i / kk];
                if (i % kk == 0) mm.mark[u] = 1;
                if (keep) {
                    mm.mark[jraw] = 1;
                    const int pb = u >> mm.ns_log;
                    atomicAdd(&s_pk[pb], 1u);
                    if ((jraw & ((1 << mm.ns_log) - 1)) == 1) atomicAdd(&s_pg[pb], 1u);
                }
            }
        }
        wave_lds_sync();
    }
    if constexpr (IDX) {
        if (mm.mark) {  // (launch-uniform) one atomic per workgroup, problem and counter
            __syncthreads();
            if ((int)threadIdx.x < mm.nprob) {
                if (s_pk[threadIdx.x]) atomicAdd(mm.pkept + threadIdx.x, (unsigned long long)s_pk[threadIdx.x]);
                if (s_pg[threadIdx.x]) atomicAdd(mm.pgoal + threadIdx.x, (unsigned long long)s_pg[threadIdx.x]);
            }
        }
    }
    if (IDX && mm.count) {  // one atomic per workgroup and counter
        __shared__ uint32_t mk_part[2][BLOCK / 64];
        for (int o = 32; o > 0; o >>= 1) {
            mk_keep += (uint32_t)__shfl_xor((int)mk_keep, o, 64);
            mk_tgt += (uint32_t)__shfl_xor((int)mk_tgt, o, 64);
        }
        if (lane == 0) {
            mk_part[0][wave] = mk_keep;
            mk_part[1][wave] = mk_tgt;
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            uint32_t t = 0;
            for (int w = 0; w < BLOCK / 64; ++w) t += mk_part[threadIdx.x][w];
            if (t) atomicAdd(mm.count + threadIdx.x, (unsigned long long)t);
        }
    }
    EPP_MTL_END;
}

}  // namespace
}  // namespace epp

using namespace epp;

namespace {
// LDS bytes of k_motions_v5 for this world (records, tile rows, wave queues), 0 when the
// world has no tile tables or they do not fit the budget.
uint32_t motions_v5_lds(const WorldView& w) {
    if (w.slab_n <= 0) return 0;
    const uint32_t recb5 = (uint32_t)(((size_t)w.n_obb * kRecDoubles * 8 + 15) & ~size_t(15));
    const uint32_t tileb = (uint32_t)((size_t)w.tile_n * w.tile_n * w.tile_words * 4);
    const uint32_t shm5 = recb5 + tileb + 16u * (kQueueV5 * 4 + 64);
    return shm5 > kLdsBudget ? 0 : shm5;
}

// k_motions_v5 when the world has tile tables and they, the records and the wave queues
// fit the LDS budget; returns false (nothing launched) otherwise.
bool launch_motions_v5(const WorldView* dw, const WorldView& w, const double* s1, const double* s2,
                       const int32_t* nbr, int kk, int64_t n, int32_t can_pass_gate, int32_t mode, uint8_t* valid,
                       hipStream_t st, const MotionMask& mm = MotionMask{}) {
    const uint32_t shm5 = motions_v5_lds(w);
    if (shm5 == 0) return false;
    const uint32_t recb5 = (uint32_t)(((size_t)w.n_obb * kRecDoubles * 8 + 15) & ~size_t(15));
    const uint32_t tileb = (uint32_t)((size_t)w.tile_n * w.tile_n * w.tile_words * 4);
    const int per_cu = std::max(1, std::min(2, (int)((160u * 1024u) / shm5)));
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 1023) / 1024, (int64_t)cu_count() * per_cu));
#define EPP_LAUNCH_M5(WW, MM, II)                                                                                 \
    do {                                                                                                          \
        allow_lds(k_motions_v5<WW, MM, II>);                                                                      \
        hipLaunchKernelGGL((k_motions_v5<WW, MM, II>), dim3(grid), dim3(1024), shm5, st, dw, s1, s2, nbr, kk, n, \
                           can_pass_gate, valid, recb5, tileb, mm);                                               \
    } while (0)
#define EPP_LAUNCH_M5W(MM, II)                       \
    switch (w.slab_w) {                              \
        case 1: EPP_LAUNCH_M5(1, MM, II); break;     \
        case 2: EPP_LAUNCH_M5(2, MM, II); break;     \
        case 4: EPP_LAUNCH_M5(4, MM, II); break;     \
        case 8: EPP_LAUNCH_M5(8, MM, II); break;     \
        case 16: EPP_LAUNCH_M5(16, MM, II); break;   \
        default: EPP_LAUNCH_M5(32, MM, II); break;   \
    }
    if (nbr) {
        if (mode == 0) {
            EPP_LAUNCH_M5W(0, true)
        } else {
            EPP_LAUNCH_M5W(1, true)
        }
    } else {
        if (mode == 0) {
            EPP_LAUNCH_M5W(0, false)
        } else {
            EPP_LAUNCH_M5W(1, false)
        }
    }
#undef EPP_LAUNCH_M5W
#undef EPP_LAUNCH_M5
    return true;
}
}  // namespace

extern "C" {

// Kernel choice: small batches (<= kSmallMotions edges, <= kSmallMaxObbs OBBs) take the
// brute-force k_motions_small (small.hip; no index needed); else k_motions_v5 (slab filter) for worlds of <= 1024 OBBs whose records and
// slab rows fit a CU's LDS; else the cell-list LDS kernels (k_motions_v4 analytic,
// k_motions_d32b discrete32) when the coarse grid, the records and the wave queues fit;
// else k_motions.  Test hooks (not for production use): EPP_MOTIONS_KERNEL=generic forces
// k_motions, =v4 skips k_motions_v5; EPP_MOTIONS_BLOCK = 512 | 1024 forces the cell-list
// kernels' workgroup size.
epp_status epp_check_motions(const epp_world* world, const double* s1, const double* s2, int64_t n,
                             int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!s1 || !s2 || !valid)) || (mode != 0 && mode != 1)) {
        set_error("epp_check_motions: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    SmallWorld sw = small_world(world);
    if (small_motions(sw, n)) {
        if (const epp_status st =
                launch_motions_small(sw, mode, s1, s2, n, can_pass_gate != 0 ? 1 : 0, valid, (hipStream_t)stream))
            return st;
        return note_record_reader(world, sw, (hipStream_t)stream);
    }
    sw.lease = {};  // (a stale index is rebuilt below)
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    const WorldView& w = ix.view;
    hipStream_t st = (hipStream_t)stream;
    const char* forced = std::getenv("EPP_MOTIONS_KERNEL");
    const bool generic = forced && std::string(forced) == "generic";
    // LDS: coarse grid + lists (blob up to `meta`), the records, per-wave queue/flags/heads,
    // and a 32-byte float filter record per OBB
    const uint32_t front = w.off_meta;
    const uint32_t recb = (uint32_t)(((size_t)w.n_obb * kRecDoubles * 8 + 15) & ~size_t(15));
    auto extra_for = [&](int blk) -> uint32_t {
        const uint32_t q = mode == 0 ? (uint32_t)kQueueM : (uint32_t)kQueueD32;
        return (uint32_t)((blk / 64) * ((q + 1) * 4 + 64 + 256) + (uint32_t)w.n_obb * 32u);
    };
    // Block size: 512 threads when two such blocks fit a CU's LDS (small worlds: C4's 64
    // OBBs, v4 28 vs 32 us per 1M edges), else 1024 (C3's 512 OBBs stage ~95 KB, one block
    // per CU, and 1024 threads double the waves behind the LDS walk: v4 52 vs 69 us)
    // k_motions_v5 when the world has tile tables and they, the records and the queues fit
    const bool force_v4 = forced && std::string(forced) == "v4";
    if (!generic && !force_v4 &&
        launch_motions_v5(ix.dview, w, s1, s2, nullptr, 1, n, can_pass_gate, mode, valid, st))
        return launch_error("epp_check_motions");
    const int eb = env_int("EPP_MOTIONS_BLOCK", 0);
    const int block = eb == 512 ? 512 : eb == 1024 ? 1024 : (2u * (front + recb + extra_for(512)) <= 160u * 1024u ? 512 : 1024);
    const uint32_t shm = front + recb + extra_for(block);
    if (!generic && front % 16 == 0 && shm <= 160u * 1024u) {
        const int grid = (int)std::max<int64_t>(
            1, std::min<int64_t>((n + block - 1) / block, (int64_t)cu_count() * std::max(1, (int)((160u * 1024u) / shm))));
        const WorldView* dw = ix.dview;
#define EPP_LAUNCH_M(KERNEL)                                                                                           \
    do {                                                                                                               \
        allow_lds(KERNEL);                                                                                             \
        hipLaunchKernelGGL(KERNEL, dim3(grid), dim3(block), shm, st, dw, s1, s2, n, can_pass_gate, valid, front, recb); \
    } while (0)
        if (mode == 0) {
            if (block == 1024) EPP_LAUNCH_M((k_motions_v4<1024>));
            else EPP_LAUNCH_M((k_motions_v4<512>));
        } else {
            if (block == 1024) EPP_LAUNCH_M((k_motions_d32b<1024>));
            else EPP_LAUNCH_M((k_motions_d32b<512>));
        }
#undef EPP_LAUNCH_M
        return launch_error("epp_check_motions");
    }
    const int aligned = ((reinterpret_cast<uintptr_t>(s1) | reinterpret_cast<uintptr_t>(s2)) & 15) == 0;
    const int grid = grid_for((n + 3) / 4, 0);
    if (mode == 0)
        hipLaunchKernelGGL((k_motions<0>), dim3(grid), dim3(kBlock), 0, st, w, s1, s2, n, can_pass_gate, valid, aligned);
    else
        hipLaunchKernelGGL((k_motions<1>), dim3(grid), dim3(kBlock), 0, st, w, s1, s2, n, can_pass_gate, valid, aligned);
    return launch_error("epp_check_motions");
}

epp_status epp_check_knn_motions(const epp_world* world, const double* nodes, const int32_t* nbr, int32_t n,
                                 int32_t k, int32_t can_pass_gate, int32_t mode, uint8_t* valid, void* stream) {
    if (!world || n < 0 || k <= 0 || (n > 0 && (!nodes || !nbr || !valid)) || (mode != 0 && mode != 1)) {
        set_error("epp_check_knn_motions: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int64_t m = (int64_t)n * k;
    if (m == 0) return EPP_OK;
    SmallWorld sw = small_world(world);
    if (small_motions(sw, m) || std::getenv("EPP_MOTIONS_KERNEL")) {
        set_error("epp_check_knn_motions: not for this batch / world (use epp_knn_edges + epp_check_motions)");
        return EPP_ERR_UNSUPPORTED;
    }
    sw.lease = {};
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    if (!launch_motions_v5(ix.dview, ix.view, nodes, nullptr, nbr, k, m, can_pass_gate, mode, valid,
                           (hipStream_t)stream)) {
        set_error("epp_check_knn_motions: not for this batch / world (use epp_knn_edges + epp_check_motions)");
        return EPP_ERR_UNSUPPORTED;
    }
    return launch_error("epp_check_knn_motions");
}

}  // extern "C"

epp_status epp::check_knn_motions_masked(const epp_world* world, const double* nodes, int32_t* nbr, int32_t n,
                                         int32_t k, int32_t can_pass_gate, uint8_t* valid, uint16_t* out16,
                                         int32_t target, int64_t* count, void* stream) {
    if (!world || n < 0 || k <= 0 || (n > 0 && (!nodes || !nbr || !valid || !count))) {
        set_error("check_knn_motions_masked: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int64_t m = (int64_t)n * k;
    if (m == 0) return EPP_OK;
    SmallWorld sw = small_world(world);
    if (small_motions(sw, m) || std::getenv("EPP_MOTIONS_KERNEL")) {
        set_error("check_knn_motions_masked: not for this batch / world");
        return EPP_ERR_UNSUPPORTED;
    }
    sw.lease = {};
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    MotionMask mm;
    mm.nbr_w = nbr;
    mm.out16 = out16;
    mm.target = target;
    mm.count = reinterpret_cast<unsigned long long*>(count);
    if (!launch_motions_v5(ix.dview, ix.view, nodes, nullptr, nbr, k, m, can_pass_gate, 0, valid, (hipStream_t)stream,
                           mm)) {
        set_error("check_knn_motions_masked: not for this batch / world");
        return EPP_ERR_UNSUPPORTED;
    }
    return launch_error("check_knn_motions_masked");
}

bool epp::knn_motions_rows_supported(const epp_world* world) {
    if (!world) return false;
    IndexLease ix;
    if (ensure_index(world, &ix) != EPP_OK) return false;
    return motions_v5_lds(ix.view) != 0;
}

epp_status epp::check_knn_motions_rows(const epp_world* world, const double* nodes, int32_t* rows32,
                                       const int32_t* ids32, const int64_t* rows_n, int32_t cap, int32_t k,
                                       int32_t can_pass_gate, uint8_t* valid, uint16_t* out16, int32_t target,
                                       int64_t* count, void* stream, const MotionMask* marks) {
    if (!world || cap < 0 || k <= 0 || (cap > 0 && (!nodes || !rows32 || !ids32 || !rows_n || !valid || (!count && !out16))) ||
        (marks && marks->mark && (!out16 || !marks->pkept || !marks->pgoal || marks->nprob < 1 || marks->nprob > 64))) {
        set_error("check_knn_motions_rows: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int64_t m = (int64_t)cap * k;
    if (m == 0) return EPP_OK;
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    MotionMask mm;
    mm.nbr_w = rows32;
    mm.out16 = out16;
    mm.target = target;
    mm.count = reinterpret_cast<unsigned long long*>(count);
    mm.rowmap = ids32;
    mm.rows_n = reinterpret_cast<const unsigned long long*>(rows_n);
    if (marks) {
        mm.mark = marks->mark;
        mm.pkept = marks->pkept;
        mm.pgoal = marks->pgoal;
        mm.ns_log = marks->ns_log;
        mm.nprob = marks->nprob;
    }
    if (!launch_motions_v5(ix.dview, ix.view, nodes, nullptr, rows32, k, m, can_pass_gate, 0, valid,
                           (hipStream_t)stream, mm)) {
        set_error("check_knn_motions_rows: not for this world");
        return EPP_ERR_UNSUPPORTED;
    }
    return launch_error("check_knn_motions_rows");
}

extern "C" {

#ifdef EPP_MOTIONS_TL
// diagnostics builds only: the per-wave time split of the last k_motions_v4 launch
epp_status epp_dbg_motions_tl(unsigned long long* out, int64_t waves) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_motions_tl), (size_t)std::min<int64_t>(waves, kMtlWaves) * 48) ==
                   hipSuccess
               ? EPP_OK
               : EPP_ERR_HIP;
}
#endif

}  // extern "C"

// states.hip — batched state validity checks for gfx950 (MI355X).
//
//   World::checkPointValidity(p, canPassGate)  src/World.cpp:80-104
//   World::checkPointValidity(p, minDistance)  src/World.cpp:106-128  (MINDIST)
//   + optional wave-ballot compaction of the valid states (no reference counterpart)
//
// Three kernels, chosen by what fits (launch_states):
//   k_states_v5  default: records + lists + fine-cell class table staged in LDS, one
//                class lookup per state, exact fp64 tests only for the ~10% of states
//                whose class cell some inflated AABB reaches;
//   k_states_v4  worlds whose staged part exceeds kStageBudget (e.g. C3's 512 OBBs):
//                class table read through L2, records + lists in LDS;
//   k_states     generic: any world size, unaligned buffers (coarse grid walk).
// Layout: a lane owns consecutive states (96 B = six 16-B loads for four) and writes their
// flag bytes with one store.
#include "collision_common.h"

namespace epp {
namespace {

// STAGE: 0 = world read from HBM/L2, 1 = front (masks, cell starts) in LDS, 2 = all in LDS
template <int STAGE, bool MINDIST, bool ALIGNED>
__global__ __launch_bounds__(kBlock) void k_states(WorldView w, const double* __restrict__ xyz,
                                                   int64_t n, int can_pass, double md,
                                                   uint8_t* __restrict__ valid,
                                                   int32_t* __restrict__ compact_idx,
                                                   unsigned long long* __restrict__ n_valid,
                                                   uint32_t stage_bytes) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63;
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
    WaveScratch* ws = reinterpret_cast<WaveScratch*>(lds + (threadIdx.x >> 6) * ((sizeof(WaveScratch) + 15) & ~15u));
    const unsigned char* staged = STAGE ? stage_world(w, lds + kScratchBytes, stage_bytes) : w.blob;
    const Acc a = make_acc(staged, STAGE == 2 ? staged : w.blob, w);

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
    // tail: the last n % 4 states, one lane each
    if (blockIdx.x == 0 && threadIdx.x < (int)(n - 4 * groups)) {
        const int64_t i = 4 * groups + threadIdx.x;
        const bool ok = state_valid_scalar<MINDIST>(a, w, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2],
                                                    can_pass != 0, md);
        valid[i] = ok ? 1 : 0;
        if (compact_idx && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

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
    uint32_t hdr[64];  // the queued states' list headers (start << 12 | count)
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

// Per-wave timeline of k_states_v5 (diagnostics builds only: -DEPP_STATES_TL, see
// scripts/states_timeline.py): lane 0 stamps s_memrealtime (100 MHz) at entry, after the
// staging barrier, after the first group's classification (its data arrived), after its
// exact path, at the end; plus HW_ID.
#ifdef EPP_STATES_TL
constexpr int kTlWaves = 1 << 16;
__device__ unsigned long long g_states_tl[kTlWaves][6];
#define EPP_STL(k)                                                                                  \
    do {                                                                                            \
        const int w_ = (int)((blockIdx.x * BLOCK + threadIdx.x) >> 6);                             \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                             \
        if ((threadIdx.x & 63) == 0 && w_ < kTlWaves) g_states_tl[w_][k] = t_;                      \
    } while (0)
#else
#define EPP_STL(k) \
    do {           \
    } while (0)
#endif

// PREFETCH: groups per lane > 1 (the next group's loads overlap this one's work);
// single-pass launches (e.g. 1M states on 256 CUs) drop the second buffer's registers.
// SPL: states per lane and group (4: 96 B = six 16-B loads, 8: 192 B = twelve); one
// flag store of SPL bytes.  More states per lane = fewer waves, i.e. fewer executions
// of the per-wave fixed costs (setup, staging, the exact path).
// SC: staging chunks (16 B) per lane: enough for the staged bytes (launcher's choice).
template <bool MINDIST, bool COMPACT, int BLOCK, bool PREFETCH, int SPL, bool C8, int SC>
__global__ __launch_bounds__(BLOCK) void k_states_v5(const WorldView* __restrict__ wv,
                                                     const double* xyz, int64_t groups, int64_t n,
                                                     int can_pass, double md, uint8_t* __restrict__ valid,
                                                     int32_t* __restrict__ compact_idx,
                                                     unsigned long long* __restrict__ n_valid, uint32_t stage_bytes) {
    __shared__ WaveQueue5 queues[BLOCK / 64];
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_blob[];
    const int lane = threadIdx.x & 63;
    EPP_STL(0);
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
    constexpr int kStageChunks = SC;
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
    // the class table: bytes (C8, staged right after the lists) or u16
    const unsigned char* cls_base = lds_blob + ((C8 ? wv->off_cls8 : wv->off_bitmap) - wv->off_aos);
    [[maybe_unused]] const unsigned char* cls_nz = cls_base + ((wv->bm_words + 1u + 31u) >> 5) * 8u;  // (sparse classes)
    const uint32_t* hdrs = reinterpret_cast<const uint32_t*>(lds_blob + lists_off);
    const uint16_t* ids_all = reinterpret_cast<const uint16_t*>(lds_blob + ids_off);
    const double* recs = reinterpret_cast<const double*>(lds_blob);
    const float ox = wv->bofx, oy = wv->bofy, oz = wv->bofz, ix = wv->bix, iy = wv->biy, iz = wv->biz;
    const uint32_t nx = (uint32_t)wv->bnx, ny = (uint32_t)wv->bny, nz = (uint32_t)wv->bnz;
    const double rg = wv->r_gate, ro = wv->r_obst;
    __syncthreads();
    EPP_STL(1);
    auto cls_of = [&](double px, double py, double pz) -> uint32_t {
        const uint32_t cx = cell_axis5(px, ox, ix, nx - 1), cy = cell_axis5(py, oy, iy, ny - 1),
                       cz = cell_axis5(pz, oz, iz, nz - 1);
        const uint32_t idx = __umul24(__umul24(cz, ny) + cy, nx) + cx;
#ifndef EPP_V5_DENSE_CLS
        if (C8) {  // sparse byte classes: the occupancy word, then (occupied cells) the class byte
            const uint64_t wd = reinterpret_cast<const uint64_t*>(cls_base)[idx >> 5];
            const uint32_t m = (uint32_t)wd, sh = idx & 31u;
            const uint32_t rank = (uint32_t)(wd >> 32) + (uint32_t)__popc(m & ((1u << sh) - 1u));
            return ((m >> sh) & 1u) ? (uint32_t)cls_nz[rank] : 0u;
        }
#endif
        return C8 ? (uint32_t)cls_base[idx] : (uint32_t)reinterpret_cast<const uint16_t*>(cls_base)[idx];
    };
#ifdef EPP_STATES_TL
    uint32_t tl_needy = 0, tl_pairs = 0;  // (diagnostics) queued states and pairs
#endif
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
        EPP_STL(2);
        // the needy states' list headers, read now (one LDS round trip for all four,
        // overlapping the ballot arithmetic) and queued with the state
        uint32_t hd[SPL];
#pragma unroll
        for (int k = 0; k < SPL; ++k) hd[k] = hdrs[needy[k] ? c[k] : 0u];  // list 0 is empty
        uint32_t hits = 0;
#ifdef EPP_STATES_NOEXACT  // diagnostics builds only (wrong answers): the cost of the exact path
#pragma unroll
        for (int k = 0; k < SPL; ++k) hits |= needy[k] ? 1u << k : 0u;
        if (false) {
#else
        if (total > 0) {  // wave-uniform
#endif
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
                        qu->hdr[slot] = hd[k];
                    }
                }
                wave_lds_sync();
                const uint32_t tq = min(total - r0, 64u);
                // lane e < tq owns queued state e: its candidate list
                const bool act = (uint32_t)lane < tq;
                const uint32_t hq = act ? qu->hdr[lane] : 0u;
                const uint32_t cnt = hq & 4095u, first = hq >> 12;
                uint32_t ptot;
                const uint32_t poff = wave_excl_scan(cnt, lane, ptot);
#ifdef EPP_STATES_TL
                tl_needy += tq;
                tl_pairs += ptot;
#endif
                bool hit_e = false;
                if (ptot <= 128u) {
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
                    const double* rc = reinterpret_cast<const double*>(lds_blob);
                    const uint16_t* idl = reinterpret_cast<const uint16_t*>(lds_blob + ids_off) + first;
                    const double px = qu->x[lane], py = qu->y[lane], pz = qu->z[lane];
                    for (uint32_t j = 0; j < cnt; ++j)
                        hit_e |= rec_hit<MINDIST>(rc + (size_t)idl[j] * kRecDoubles, rg, ro, px, py, pz, can_pass != 0,
                                                  md);
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
        }
        EPP_STL(3);
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
#ifdef EPP_STATES_TL
    EPP_STL(4);
    if (lane == 0) {
        unsigned hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const int w_ = (int)((blockIdx.x * BLOCK + threadIdx.x) >> 6);
        if (w_ < kTlWaves)
            g_states_tl[w_][5] = hw | ((unsigned long long)min(tl_needy, 65535u) << 32) |
                                 ((unsigned long long)min(tl_pairs, 65535u) << 48);
    }
#endif
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

// ---- launch ---------------------------------------------------------------------------
// Kernel choice: small batches (<= kSmallStates states, <= kSmallMaxObbs OBBs) take the
// brute-force k_states_small (small.hip; no index needed); else k_states_v5 when its staged part fits and the buffers are aligned, else
// k_states_v4 (aligned buffers), else k_states.  Test hooks (not for production use):
// EPP_STATES_KERNEL = v4 | generic skips the faster kernels, EPP_V5_BLOCK = 512 | 1024
// forces the k_states_v5 workgroup size, so every path and shape can be checked against
// the oracle.
enum class StatesKernel { V5, V4, Generic };
StatesKernel forced_kernel() {
    const char* v = std::getenv("EPP_STATES_KERNEL");
    if (!v || !*v) return StatesKernel::V5;
    const std::string k(v);
    return k == "generic" ? StatesKernel::Generic : k == "v4" ? StatesKernel::V4 : StatesKernel::V5;
}

// k_states_v5 stages records, lists and the class table (bytes when there are, else u16):
// [off_aos, end of the byte table) or [off_aos, blob_bytes)
uint32_t v5_staged(const WorldView& w) {
    return (w.off_cls8 ? ((w.off_cls8 + w.cls8_bytes + 15u) & ~15u) : w.blob_bytes) - w.off_aos;
}
bool v5_fits(const WorldView& w) {
    const uint32_t sb = v5_staged(w);
    return sb <= kStageBudget && sb + 16u + queue5_bytes<1024>() <= 160u * 1024u;
}

// Launch shape of k_states_v5.  Single pass (every lane one group, e.g. 1M states on 256
// CUs): two 512-thread workgroups per CU when two staged copies fit in LDS (1M states:
// 8.3-8.4 us vs 8.7-8.8 us for one 1024-thread workgroup — each half of the CU syncs and
// stages on its own), else one 1024-thread workgroup.  More than one pass: one 512-thread
// workgroup per CU, the next group prefetched.
struct V5Shape {
    int64_t gN;
    int bs, grid;
    bool pf;
};
V5Shape v5_shape(int64_t n, uint32_t sb) {
    V5Shape r{};
    const int64_t cus = cu_count();
    r.gN = n / 4;
    const int forced = env_int("EPP_V5_BLOCK", 0);
    if (forced == 256 && 4u * (sb + 16u + queue5_bytes<256>()) <= 160u * 1024u && r.gN <= 4 * cus * 256) {
        // (test hook / A/B) single pass on four 256-thread workgroups per CU
        r.bs = 256;
        r.grid = (int)std::max<int64_t>(1, (r.gN + 255) / 256);
        r.pf = false;
        return r;
    }
    const bool two = forced == 0 && 2u * (sb + 16u + queue5_bytes<512>()) <= 160u * 1024u && r.gN <= 2 * cus * 512;
    if (two) {
        r.bs = 512;
        r.grid = (int)std::max<int64_t>(1, (r.gN + 511) / 512);
        r.pf = false;
        return r;
    }
    const bool single = r.gN <= cus * 1024;
    r.bs = forced == 512 ? 512 : forced == 1024 ? 1024 : (single ? 1024 : 512);
    r.grid = (int)std::max<int64_t>(1, std::min<int64_t>((r.gN + r.bs - 1) / r.bs, cus));
    r.pf = r.gN > (int64_t)r.grid * r.bs;  // more than one group per lane
    return r;
}

bool v4_stage(const WorldView& w) { return (w.off_bitmap - w.off_aos) + sizeof(StateQueue4) <= 160u * 1024u; }
// resident workgroups only (every block loops): LDS-limited, at most 3 per CU
int v4_grid(const WorldView& w, int64_t n) {
    const int64_t items = std::max<int64_t>(1, n / 2);
    const int64_t need = (items + kBlock4 - 1) / kBlock4;
    const uint32_t lds = sizeof(StateQueue4) + (v4_stage(w) ? w.off_bitmap - w.off_aos : 0u);
    const int per_cu = std::max(1, std::min<int>(3, (int)((160u * 1024u) / lds)));
    const int64_t cap = (int64_t)cu_count() * per_cu;
    return (int)std::max<int64_t>(1, std::min(need, cap));
}

template <bool MINDIST>
epp_status launch_states(const WorldView& w, const WorldView* dw, const double* xyz, int64_t n, int32_t can_pass,
                         double md, uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    auto nv = reinterpret_cast<unsigned long long*>(n_valid);
    const char* what = MINDIST ? "epp_check_states_mindist" : "epp_check_states";
    const StatesKernel want = forced_kernel();
    const bool x16 = (reinterpret_cast<uintptr_t>(xyz) & 15) == 0;
    if (want == StatesKernel::V5 && v5_fits(w) && x16 && (reinterpret_cast<uintptr_t>(valid) & 3) == 0) {
#ifdef EPP_V5_STAGECAP  // (diagnostics timing probes only: WRONG answers) stage at most this many bytes
        const uint32_t sb = std::min<uint32_t>(v5_staged(w), EPP_V5_STAGECAP);
#else
        const uint32_t sb = v5_staged(w);
#endif
        V5Shape sh = v5_shape(n, sb);
        if (sh.bs == 256 && compact_idx) {  // (the 256-thread shape is instantiated without compaction)
            sh.bs = 512;
            sh.grid = (int)std::max<int64_t>(1, (sh.gN + 511) / 512);
        }
        const uint32_t dyn = sb + 16u;  // the staged world + the dummy slot of the copy
#define EPP_LAUNCH_V5S(C, B, P, C8, SC)                                                                              \
    do {                                                                                                             \
        allow_lds(k_states_v5<MINDIST, C, B, P, 4, C8, SC>, queue5_bytes<B>());                                      \
        hipLaunchKernelGGL((k_states_v5<MINDIST, C, B, P, 4, C8, SC>), dim3(sh.grid), dim3(B), dyn, st, dw, xyz, sh.gN, \
                           n, can_pass, md, valid, compact_idx, nv, sb);                                             \
    } while (0)
        // staging chunks per lane: as many as the staged bytes need (1, 2 or 3), else half
        // the budget's or the whole budget's
        const bool half_stage = sb <= (uint32_t)kStageBudget / 2;
#define EPP_LAUNCH_V5C(C, B, P, C8)                                                              \
    do {                                                                                         \
        if (sb <= (uint32_t)B * 16u) EPP_LAUNCH_V5S(C, B, P, C8, 1);                              \
        else if (sb <= (uint32_t)B * 32u) EPP_LAUNCH_V5S(C, B, P, C8, 2);                         \
        else if (sb <= (uint32_t)B * 48u) EPP_LAUNCH_V5S(C, B, P, C8, 3);                         \
        else if (half_stage) EPP_LAUNCH_V5S(C, B, P, C8, (int)(kStageBudget / 2 / (B * 16)));    \
        else EPP_LAUNCH_V5S(C, B, P, C8, (int)(kStageBudget / (B * 16)));                        \
    } while (0)
#define EPP_LAUNCH_V5(C, B, P)                                 \
    do {                                                       \
        if (w.off_cls8) EPP_LAUNCH_V5C(C, B, P, true);          \
        else EPP_LAUNCH_V5C(C, B, P, false);                    \
    } while (0)
#define EPP_LAUNCH_V5B(B)                                \
    do {                                                 \
        if (sh.pf) {                                     \
            if (compact_idx) EPP_LAUNCH_V5(true, B, true);  \
            else EPP_LAUNCH_V5(false, B, true);          \
        } else {                                         \
            if (compact_idx) EPP_LAUNCH_V5(true, B, false); \
            else EPP_LAUNCH_V5(false, B, false);         \
        }                                                \
    } while (0)
        if (sh.bs == 256) EPP_LAUNCH_V5(false, 256, false);  // (EPP_V5_BLOCK=256, single pass)
        else if (sh.bs == 512) EPP_LAUNCH_V5B(512);
        else EPP_LAUNCH_V5B(1024);
#undef EPP_LAUNCH_V5B
#undef EPP_LAUNCH_V5
#undef EPP_LAUNCH_V5C
#undef EPP_LAUNCH_V5S
        return launch_error(what);
    }
    if (want != StatesKernel::Generic && x16 && (reinterpret_cast<uintptr_t>(valid) & 1) == 0 &&
        n / 2 < 0xFFFFFFFFll) {
        const uint32_t sb = w.off_bitmap - w.off_aos;
        const bool stg = v4_stage(w);
        const int g4 = v4_grid(w, n);
        const uint32_t items = (uint32_t)(n / 2);
#define EPP_LAUNCH_V4(S, C)                                                                                      \
    do {                                                                                                         \
        allow_lds(k_states_v4<MINDIST, S, C>, sizeof(StateQueue4));                                              \
        hipLaunchKernelGGL((k_states_v4<MINDIST, S, C>), dim3(g4), dim3(kBlock4), S ? sb : 0, st, dw, xyz, items, n, \
                           can_pass, md, valid, compact_idx, nv, sb);                                            \
    } while (0)
        if (compact_idx) {
            if (stg) EPP_LAUNCH_V4(true, true);
            else EPP_LAUNCH_V4(false, true);
        } else {
            if (stg) EPP_LAUNCH_V4(true, false);
            else EPP_LAUNCH_V4(false, false);
        }
#undef EPP_LAUNCH_V4
        return launch_error(what);
    }
    // generic: stage the whole world when it is small (several blocks per CU), else only
    // the front (occupancy masks + cell starts) and read the OBB table through L1/L2
    const bool aligned = (x16 & ((reinterpret_cast<uintptr_t>(valid) & 3) == 0));
    const bool lds = w.front_bytes + kScratchBytes <= kLdsBudget;
    const uint32_t stage = !lds ? 0u : (w.blob_bytes <= 40u * 1024u ? w.blob_bytes : w.front_bytes);
    const uint32_t shm = kScratchBytes + stage;
    const int grid = grid_for(std::max<int64_t>(1, n / 4), shm);
#define EPP_LAUNCH_STATES(L, A)                                                                              \
    do {                                                                                                     \
        allow_lds(k_states<L, MINDIST, A>);                                                                  \
        hipLaunchKernelGGL((k_states<L, MINDIST, A>), dim3(grid), dim3(kBlock), shm, st, w, xyz, n, can_pass, md, \
                           valid, compact_idx, nv, stage);                                                   \
    } while (0)
    const int mode = stage == 0 ? 0 : (stage == w.blob_bytes ? 2 : 1);
    if (mode == 2 && aligned) EPP_LAUNCH_STATES(2, true);
    else if (mode == 2) EPP_LAUNCH_STATES(2, false);
    else if (mode == 1 && aligned) EPP_LAUNCH_STATES(1, true);
    else if (mode == 1) EPP_LAUNCH_STATES(1, false);
    else if (aligned) EPP_LAUNCH_STATES(0, true);
    else EPP_LAUNCH_STATES(0, false);
#undef EPP_LAUNCH_STATES
    return launch_error(what);
}

}  // namespace
}  // namespace epp

using namespace epp;

extern "C" {

epp_status epp_check_states(const epp_world* world, const double* xyz, int64_t n, int32_t can_pass_gate,
                            uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid)) || (compact_idx && !n_valid)) {
        set_error("epp_check_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    SmallWorld sw = small_world(world);
    if (small_states(sw, n)) {
        if (const epp_status st = launch_states_small(sw, false, xyz, n, can_pass_gate, 0.0, valid, compact_idx,
                                                      n_valid, (hipStream_t)stream))
            return st;
        return note_record_reader(world, sw, (hipStream_t)stream);
    }
    sw.lease = {};  // (a stale index is rebuilt below)
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    return launch_states<false>(ix.view, ix.dview, xyz, n, can_pass_gate, 0.0, valid,
                                compact_idx, n_valid, stream);
}

#ifdef EPP_STATES_TL
// diagnostics builds only: the per-wave timeline of the last k_states_v5 launch
epp_status epp_dbg_states_tl(unsigned long long* out, int64_t waves) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_states_tl), (size_t)std::min<int64_t>(waves, kTlWaves) * 48) == hipSuccess
               ? EPP_OK
               : EPP_ERR_HIP;
}
#endif

epp_status epp_check_states_mindist(const epp_world* world, const double* xyz, int64_t n, double min_distance,
                                    uint8_t* valid, void* stream) {
    if (!world || n < 0 || (n > 0 && (!xyz || !valid))) {
        set_error("epp_check_states_mindist: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    SmallWorld sw = small_world(world);
    if (small_states(sw, n)) {
        if (const epp_status st =
                launch_states_small(sw, true, xyz, n, 0, min_distance, valid, nullptr, nullptr, (hipStream_t)stream))
            return st;
        return note_record_reader(world, sw, (hipStream_t)stream);
    }
    sw.lease = {};  // (a stale index is rebuilt below)
    IndexLease ix;
    if (const epp_status st = ensure_index(world, &ix)) return st;
    return launch_states<true>(ix.view, ix.dview, xyz, n, 0, min_distance, valid, nullptr,
                               nullptr, stream);
}

}  // extern "C"

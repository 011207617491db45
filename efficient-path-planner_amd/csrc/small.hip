// small.hip — brute-force kernels for small queries (the latency path).
//
// A few hundred states or edges (PathPlanner::checkTrajectoryValidity's lookahead rows,
// the one-at-a-time StateValidator / MotionValidator calls) do not pay for the device
// index: after epp_world_update the index is stale (rebuilt lazily), and these kernels
// test every query against every OBB record instead — read from the device blob when the
// index is current, else straight from the pinned host copy of the new version.  Same
// tests, in the same order of OBBs, as the index kernels:
//   states   World::checkPointValidity(p, canPassGate / minDistance)  src/World.cpp:80-128
//   motions  World::checkRayValid (mode 0)                            src/World.cpp:130-162
//            the 32-step discretised check (mode 1)                   BASELINE config 3
// Each workgroup stages the records in LDS; every lane then walks all OBBs in step (the
// same record for the whole wave: LDS broadcast), and the exact test runs only when some
// lane's query passes the AABB test (a wave-uniform branch).
#include <immintrin.h>

#include "collision_common.h"
#include "small_body.h"
#include "small_sync.h"

namespace epp {
namespace {

template <bool MINDIST, bool COMPACT>
__global__ __launch_bounds__(kSmallBlock) void k_states_small(const double* __restrict__ recs, int n_obb, double rg,
                                                              double ro, const double* __restrict__ xyz, int64_t n,
                                                              int per, int can_pass, double md,
                                                              uint8_t* __restrict__ valid,
                                                              int32_t* __restrict__ compact_idx,
                                                              unsigned long long* __restrict__ n_valid,
                                                              uint32_t* done, uint32_t seq) {
    extern __shared__ double srec[];
    states_small_body<MINDIST, COMPACT>(srec, blockIdx.x, recs, n_obb, rg, ro, xyz, n, per, can_pass, md, valid,
                                        compact_idx, n_valid);
    publish_done(done, seq);
}

template <int MODE>
__global__ __launch_bounds__(kSmallBlock) void k_motions_small(const double* __restrict__ recs, int n_obb, double rg,
                                                               double ro, const double* __restrict__ s1,
                                                               const double* __restrict__ s2, int64_t n, int per,
                                                               int can_pass, uint8_t* __restrict__ valid,
                                                               uint32_t* done, uint32_t seq) {
    extern __shared__ double srec[];
    uint32_t* s_hit = reinterpret_cast<uint32_t*>(srec + (((size_t)n_obb * kRecDoubles + 1) & ~size_t(1)));
    const int t = threadIdx.x, slices = kSmallBlock / per, slice = t / per, j = t - slice * per;
    const int64_t i = (int64_t)blockIdx.x * per + j;
    const bool act = i < n;
    double s[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0}, lo[3], hi[3];
    stage_records(srec, recs, n_obb * kRecDoubles, [&] {
        if (act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                s[k] = s1[3 * i + k];
                e[k] = s2[3 * i + k];
            }
        }
    });
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        // the rtree query box (src/World.cpp:137-141); mode 1: widened by a hair, since a
        // rounded point may sit an ulp past it
        const double l = (e[k] < s[k]) ? e[k] : s[k], h = (s[k] < e[k]) ? e[k] : s[k];
        lo[k] = MODE == 1 ? l - (1e-9 + 1e-12 * fabs(l)) : l;
        hi[k] = MODE == 1 ? h + (1e-9 + 1e-12 * fabs(h)) : h;
    }
    if (t < per) s_hit[t] = 0u;
    __syncthreads();
    const int o0 = (int)((int64_t)slice * n_obb / slices), o1 = (int)((int64_t)(slice + 1) * n_obb / slices);
    if (MODE == 0 && can_pass == kCanPassBoth) {
        // both answers of each ray in one pass: bit 0 valid with canPassGate = false (every
        // record), bit 1 with true (the filling records skipped, src/World.cpp:150-153).  A
        // hit on a record other than a filling one decides both; a filling hit only bit 0.
        bool any = false, solid = false;
        for (int o = o0; o < o1; ++o) {
            const double* r = srec + (size_t)o * kRecDoubles;
            const uint32_t m = (uint32_t)__double_as_longlong(r[R_META]);
            const bool filling = (m & META_FILLING) != 0u;
            const bool overlap = !((r[F_HIX] < lo[0]) | (hi[0] < r[F_LOX]) | (r[F_HIY] < lo[1]) | (hi[1] < r[F_LOY]) |
                                   (r[F_HIZ] < lo[2]) | (hi[2] < r[F_LOZ]));
            const bool c = act & overlap & !solid & !(filling & any);
            if (__builtin_amdgcn_ballot_w64(c) && c && rec_ray_hit(r, s, e, (m & META_GATE) ? rg : ro)) {
                any = true;
                solid = solid | !filling;
            }
        }
        const uint32_t bits = (any ? 1u : 0u) | (solid ? 2u : 0u);
        if (bits) atomicOr(&s_hit[j], bits);  // (LDS)
        __syncthreads();
        if (slice == 0 && act) valid[i] = (uint8_t)(s_hit[j] ^ 3u);
        publish_done(done, seq);
        return;
    }
    const bool cp = can_pass != 0;
    auto cand_of = [&](const double* r, bool hit) {
        const uint32_t m = (uint32_t)__double_as_longlong(r[R_META]);
        const bool overlap = !((r[F_HIX] < lo[0]) | (hi[0] < r[F_LOX]) | (r[F_HIY] < lo[1]) | (hi[1] < r[F_LOY]) |
                               (r[F_HIZ] < lo[2]) | (hi[2] < r[F_LOZ]));
        return act & !hit & overlap & !(cp & ((m & META_FILLING) != 0u));  // :150-153
    };
    auto test = [&](const double* r) {
        const uint32_t m = (uint32_t)__double_as_longlong(r[R_META]);
        return MODE == 0 ? rec_ray_hit(r, s, e, (m & META_GATE) ? rg : ro) : d32_pair_hit(r, s, e, rg, ro, cp);
    };
    bool hit = false;
    int o = o0;
    for (; o + 2 <= o1; o += 2) {  // two records' AABB tests before any branch
        const double* r = srec + (size_t)o * kRecDoubles;
        const bool c0 = cand_of(r, hit), c1 = cand_of(r + kRecDoubles, hit);
        if (__builtin_amdgcn_ballot_w64(c0) && c0) hit = test(r);
        if (__builtin_amdgcn_ballot_w64(c1 & !hit) && c1 && !hit) hit = test(r + kRecDoubles);
    }
    for (; o < o1; ++o) {
        const double* r = srec + (size_t)o * kRecDoubles;
        const bool c = cand_of(r, hit);
        if (__builtin_amdgcn_ballot_w64(c) && c) hit = test(r);
    }
    if (hit) s_hit[j] = 1u;
    __syncthreads();
    if (slice == 0 && act) valid[i] = s_hit[j] ? 0 : 1;
    publish_done(done, seq);
}

// test hook (not for production use): EPP_STATES_KERNEL / EPP_MOTIONS_KERNEL set to
// anything but "small" forces the index kernels
bool small_allowed(const char* var) {
    const char* v = std::getenv(var);
    return !v || !*v || std::string(v) == "small";
}

}  // namespace

bool small_states(const SmallWorld& sw, int64_t n) {
    return n <= kSmallStates && sw.n_obb <= kSmallMaxObbs && small_allowed("EPP_STATES_KERNEL");
}
bool small_motions(const SmallWorld& sw, int64_t n) {
    return n <= kSmallMotions && sw.n_obb <= kSmallMaxObbs && small_allowed("EPP_MOTIONS_KERNEL");
}

epp_status launch_states_small(const SmallWorld& sw, bool mindist, const double* xyz, int64_t n, int32_t can_pass,
                               double md, uint8_t* valid, int32_t* compact_idx, int64_t* n_valid, hipStream_t st,
                               uint32_t* done, uint32_t seq) {
    const int per = small_per(n), grid = (int)((n + per - 1) / per);
    const size_t shm = small_shm(sw.n_obb);
    auto nv = reinterpret_cast<unsigned long long*>(n_valid);
#define EPP_LAUNCH_SS(M, C)                                                                                          \
    hipLaunchKernelGGL((k_states_small<M, C>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate, \
                       sw.r_obst, xyz, n, per, can_pass, md, valid, compact_idx, nv, done, seq)
    if (mindist) EPP_LAUNCH_SS(true, false);
    else if (compact_idx) EPP_LAUNCH_SS(false, true);
    else EPP_LAUNCH_SS(false, false);
#undef EPP_LAUNCH_SS
    return launch_error(mindist ? "epp_check_states_mindist" : "epp_check_states");
}

epp_status launch_motions_small(const SmallWorld& sw, int32_t mode, const double* s1, const double* s2, int64_t n,
                                int32_t can_pass, uint8_t* valid, hipStream_t st, uint32_t* done, uint32_t seq) {
    const int per = small_per_motions(n), grid = (int)((n + per - 1) / per);
    const size_t shm = small_shm(sw.n_obb);
    if (mode == 0)
        hipLaunchKernelGGL((k_motions_small<0>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate,
                           sw.r_obst, s1, s2, n, per, can_pass, valid, done, seq);
    else
        hipLaunchKernelGGL((k_motions_small<1>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate,
                           sw.r_obst, s1, s2, n, per, can_pass, valid, done, seq);
    return launch_error("epp_check_motions");
}

// ---- synchronous host path ----------------------------------------------------------
namespace {
// per host thread: pinned completion slots (one per workgroup) and the call counter
struct DoneSlots {
    uint32_t* p = nullptr;
    uint32_t seq = 0;
    ~DoneSlots() {
        if (p) (void)hipHostFree(p);
    }
};
constexpr int kMaxSmallGroups = (int)std::max<int64_t>(kSmallStates / kSmallBlock, kSmallMotions / 16);
static_assert(kSmallStates / kSmallBlock <= kMaxSmallGroups && kSmallMotions / 16 <= kMaxSmallGroups,
              "completion slots for the small workgroups");

// Polls the slots until every workgroup has published `seq`; a stream that completes or
// fails without them ends the wait through hipStreamQuery (checked every ~1k polls).
epp_status wait_done(const uint32_t* done, int groups, uint32_t seq, hipStream_t st, const char* what) {
    for (uint64_t spin = 0;; ++spin) {
        int b = 0;
        while (b < groups && __atomic_load_n(done + b, __ATOMIC_ACQUIRE) == seq) ++b;
        if (b == groups) return EPP_OK;
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) {
                set_error(std::string(what) + ": " + hipGetErrorString(q));
                return EPP_ERR_HIP;
            }
            b = 0;
            while (b < groups && __atomic_load_n(done + b, __ATOMIC_ACQUIRE) == seq) ++b;
            if (b == groups) return EPP_OK;
            set_error(std::string(what) + ": kernel completed without its completion flags");
            return EPP_ERR_RUNTIME;
        }
        _mm_pause();
    }
}

template <typename Launch>
epp_status run_sync(int64_t n, int per, hipStream_t st, const char* what, Launch&& launch) {
    thread_local DoneSlots ds;
    if (!ds.p && hipHostMalloc(reinterpret_cast<void**>(&ds.p), kMaxSmallGroups * sizeof(uint32_t),
                               hipHostMallocDefault) != hipSuccess) {
        ds.p = nullptr;
        set_error(std::string(what) + ": pinned completion slots: hipHostMalloc failed");
        return EPP_ERR_HIP;
    }
    const uint32_t seq = ++ds.seq;
    const int groups = (int)((n + per - 1) / per);
    if (const epp_status rc = launch(ds.p, seq)) return rc;
    return wait_done(ds.p, groups, seq, st, what);
}
}  // namespace

epp_status states_small_sync(const epp_world* world, bool mindist, const double* xyz, int64_t n, int32_t can_pass,
                             double md, uint8_t* valid, hipStream_t st, bool* handled) {
    const SmallWorld sw = small_world(world);
    *handled = n > 0 && small_states(sw, n);
    if (!*handled) return EPP_OK;
    return run_sync(n, small_per(n), st, mindist ? "checkPointsMinDistance" : "checkPoints", [&](uint32_t* done, uint32_t seq) {
        return launch_states_small(sw, mindist, xyz, n, can_pass, md, valid, nullptr, nullptr, st, done, seq);
    });
}

epp_status motions_small_sync(const epp_world* world, int32_t mode, const double* s1, const double* s2, int64_t n,
                              int32_t can_pass, uint8_t* valid, hipStream_t st, bool* handled) {
    const SmallWorld sw = small_world(world);
    *handled = n > 0 && small_motions(sw, n);
    if (!*handled) return EPP_OK;
    return run_sync(n, small_per_motions(n), st, "checkRays", [&](uint32_t* done, uint32_t seq) {
        return launch_motions_small(sw, mode, s1, s2, n, can_pass, valid, st, done, seq);
    });
}

}  // namespace epp


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
#include "small_sync.h"

namespace epp {
namespace {

constexpr int kSmallBlock = 256;

// Completion flag of a workgroup for the synchronous host path (done != NULL): every
// thread's stores (the flags, in host memory) are made visible system-wide, then one
// lane publishes `seq` in the workgroup's slot; the host polls the slots instead of
// synchronising the stream.
__device__ __forceinline__ void publish_done(uint32_t* done, uint32_t seq) {
    if (!done) return;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void stage_records(double* srec, const double* recs, int nd) {
    // four loads in flight per lane (the records may be in host memory: PCIe latency)
    for (int e = threadIdx.x; e < nd; e += 4 * kSmallBlock) {
        double v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = e + q * kSmallBlock < nd ? recs[e + q * kSmallBlock] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (e + q * kSmallBlock < nd) srec[e + q * kSmallBlock] = v[q];
    }
}

template <bool MINDIST, bool COMPACT>
__global__ __launch_bounds__(kSmallBlock) void k_states_small(const double* __restrict__ recs, int n_obb, double rg,
                                                              double ro, const double* __restrict__ xyz, int64_t n,
                                                              int can_pass, double md, uint8_t* __restrict__ valid,
                                                              int32_t* __restrict__ compact_idx,
                                                              unsigned long long* __restrict__ n_valid,
                                                              uint32_t* done, uint32_t seq) {
    extern __shared__ double srec[];
    stage_records(srec, recs, n_obb * kRecDoubles);
    const int64_t i = (int64_t)blockIdx.x * kSmallBlock + threadIdx.x;
    const bool act = i < n;
    const double px = act ? xyz[3 * i] : 0.0, py = act ? xyz[3 * i + 1] : 0.0, pz = act ? xyz[3 * i + 2] : 0.0;
    __syncthreads();
    bool hit = false;
    for (int o = 0; o < n_obb; ++o) {
        const double* r = srec + (size_t)o * kRecDoubles;
        // rtree contains(point): strict  src/World.cpp:83
        const bool in = act & (r[F_LOX] < px) & (px < r[F_HIX]) & (r[F_LOY] < py) & (py < r[F_HIY]) &
                        (r[F_LOZ] < pz) & (pz < r[F_HIZ]);
        if (__builtin_amdgcn_ballot_w64(in)) hit |= in && rec_hit<MINDIST>(r, rg, ro, px, py, pz, can_pass != 0, md);
    }
    if (act) {
        valid[i] = hit ? 0 : 1;
        if (COMPACT && !hit) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
    publish_done(done, seq);
}

template <int MODE>
__global__ __launch_bounds__(kSmallBlock) void k_motions_small(const double* __restrict__ recs, int n_obb, double rg,
                                                               double ro, const double* __restrict__ s1,
                                                               const double* __restrict__ s2, int64_t n, int can_pass,
                                                               uint8_t* __restrict__ valid, uint32_t* done,
                                                               uint32_t seq) {
    extern __shared__ double srec[];
    stage_records(srec, recs, n_obb * kRecDoubles);
    const int64_t i = (int64_t)blockIdx.x * kSmallBlock + threadIdx.x;
    const bool act = i < n;
    double s[3], e[3], lo[3], hi[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s[k] = act ? s1[3 * i + k] : 0.0;
        e[k] = act ? s2[3 * i + k] : 0.0;
        // the rtree query box (src/World.cpp:137-141); mode 1: widened by a hair, since a
        // rounded point may sit an ulp past it
        const double l = (e[k] < s[k]) ? e[k] : s[k], h = (s[k] < e[k]) ? e[k] : s[k];
        lo[k] = MODE == 1 ? l - (1e-9 + 1e-12 * fabs(l)) : l;
        hi[k] = MODE == 1 ? h + (1e-9 + 1e-12 * fabs(h)) : h;
    }
    __syncthreads();
    const bool cp = can_pass != 0;
    bool hit = false;
    for (int o = 0; o < n_obb; ++o) {
        const double* r = srec + (size_t)o * kRecDoubles;
        const uint32_t m = (uint32_t)__double_as_longlong(r[R_META]);
        const bool overlap = !((r[F_HIX] < lo[0]) | (hi[0] < r[F_LOX]) | (r[F_HIY] < lo[1]) | (hi[1] < r[F_LOY]) |
                               (r[F_HIZ] < lo[2]) | (hi[2] < r[F_LOZ]));
        const bool cand = act & !hit & overlap & !(cp & ((m & META_FILLING) != 0u));  // :150-153
        if (__builtin_amdgcn_ballot_w64(cand) && cand)
            hit = MODE == 0 ? rec_ray_hit(r, s, e, (m & META_GATE) ? rg : ro) : d32_pair_hit(r, s, e, rg, ro, cp);
    }
    if (act) valid[i] = hit ? 0 : 1;
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
    const int grid = (int)((n + kSmallBlock - 1) / kSmallBlock);
    const size_t shm = (size_t)sw.n_obb * kRecDoubles * sizeof(double);
    auto nv = reinterpret_cast<unsigned long long*>(n_valid);
#define EPP_LAUNCH_SS(M, C)                                                                                          \
    hipLaunchKernelGGL((k_states_small<M, C>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate, \
                       sw.r_obst, xyz, n, can_pass, md, valid, compact_idx, nv, done, seq)
    if (mindist) EPP_LAUNCH_SS(true, false);
    else if (compact_idx) EPP_LAUNCH_SS(false, true);
    else EPP_LAUNCH_SS(false, false);
#undef EPP_LAUNCH_SS
    return launch_error(mindist ? "epp_check_states_mindist" : "epp_check_states");
}

epp_status launch_motions_small(const SmallWorld& sw, int32_t mode, const double* s1, const double* s2, int64_t n,
                                int32_t can_pass, uint8_t* valid, hipStream_t st, uint32_t* done, uint32_t seq) {
    const int grid = (int)((n + kSmallBlock - 1) / kSmallBlock);
    const size_t shm = (size_t)sw.n_obb * kRecDoubles * sizeof(double);
    if (mode == 0)
        hipLaunchKernelGGL((k_motions_small<0>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate,
                           sw.r_obst, s1, s2, n, can_pass, valid, done, seq);
    else
        hipLaunchKernelGGL((k_motions_small<1>), dim3(grid), dim3(kSmallBlock), shm, st, sw.recs, sw.n_obb, sw.r_gate,
                           sw.r_obst, s1, s2, n, can_pass, valid, done, seq);
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
constexpr int kMaxSmallGroups = (int)(kSmallStates / kSmallBlock);

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
epp_status run_sync(int64_t n, hipStream_t st, const char* what, Launch&& launch) {
    thread_local DoneSlots ds;
    if (!ds.p && hipHostMalloc(reinterpret_cast<void**>(&ds.p), kMaxSmallGroups * sizeof(uint32_t),
                               hipHostMallocDefault) != hipSuccess) {
        ds.p = nullptr;
        set_error(std::string(what) + ": pinned completion slots: hipHostMalloc failed");
        return EPP_ERR_HIP;
    }
    const uint32_t seq = ++ds.seq;
    const int groups = (int)((n + kSmallBlock - 1) / kSmallBlock);
    if (const epp_status rc = launch(ds.p, seq)) return rc;
    return wait_done(ds.p, groups, seq, st, what);
}
}  // namespace

epp_status states_small_sync(const epp_world* world, bool mindist, const double* xyz, int64_t n, int32_t can_pass,
                             double md, uint8_t* valid, hipStream_t st, bool* handled) {
    const SmallWorld sw = small_world(world);
    *handled = n > 0 && small_states(sw, n);
    if (!*handled) return EPP_OK;
    return run_sync(n, st, mindist ? "checkPointsMinDistance" : "checkPoints", [&](uint32_t* done, uint32_t seq) {
        return launch_states_small(sw, mindist, xyz, n, can_pass, md, valid, nullptr, nullptr, st, done, seq);
    });
}

epp_status motions_small_sync(const epp_world* world, int32_t mode, const double* s1, const double* s2, int64_t n,
                              int32_t can_pass, uint8_t* valid, hipStream_t st, bool* handled) {
    const SmallWorld sw = small_world(world);
    *handled = n > 0 && small_motions(sw, n);
    if (!*handled) return EPP_OK;
    return run_sync(n, st, "checkRays", [&](uint32_t* done, uint32_t seq) {
        return launch_motions_small(sw, mode, s1, s2, n, can_pass, valid, st, done, seq);
    });
}

}  // namespace epp

// small_body.h — device bodies of the brute-force small-query kernels (small.hip), shared
// with the fused check + refit kernel of the online step (minsnap.hip).  See small.hip.
#pragma once
#include "collision_common.h"
#include "completion.h"

namespace epp {
namespace {

constexpr int kSmallBlock = 256;

// Completion flag of a workgroup for the synchronous host path (done != NULL): every
// thread's stores (the flags, in host memory) are made visible system-wide, then one
// lane publishes `seq` in the workgroup's slot; the host polls the slots instead of
// synchronising the stream.
__device__ __forceinline__ void publish_done(uint32_t* done, uint32_t seq) {
    if (!done) return;
    wg_stores_settled();
    if (threadIdx.x == 0) __hip_atomic_store(done + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The records (n_obb x kRecDoubles doubles, 16-byte aligned start) into LDS: every 16-byte load
// of up to 128 OBBs in flight at once (the records may be in host memory: one PCIe round
// trip instead of one per few loads); `before` runs between the loads and the stores
// (the caller issues its own loads there, so they overlap too).
template <typename F>
__device__ __forceinline__ void stage_records(double* srec, const double* recs, int nd, F&& before) {
    constexpr int kQ = (128 * kRecDoubles / 2 + kSmallBlock - 1) / kSmallBlock;  // 16-byte loads per lane
    const int n2 = nd / 2;
    const double2* s2 = reinterpret_cast<const double2*>(recs);
    double2* d2 = reinterpret_cast<double2*>(srec);
    double2 v[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        const int e = threadIdx.x + q * kSmallBlock;
        v[q] = e < n2 ? s2[e] : make_double2(0.0, 0.0);
    }
    before();
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        const int e = threadIdx.x + q * kSmallBlock;
        if (e < n2) d2[e] = v[q];
    }
    for (int e = threadIdx.x + kQ * kSmallBlock; e < n2; e += kSmallBlock) d2[e] = s2[e];  // (> 128 OBBs)
    if ((nd & 1) && threadIdx.x == 0) srec[nd - 1] = recs[nd - 1];  // (odd OBB count: 136-byte records)
}

// A workgroup takes `per` queries (64, 128 or 256) and splits the OBB list into
// kSmallBlock / per slices, one per group of `per` threads: the few hundred queries of a
// latency-path call keep every wave of the workgroup busy, and each wave walks a shorter
// list.  A slice's hit marks the query's LDS flag; slice 0 writes the answers.
__host__ __device__ inline int small_per(int64_t n) { return n <= 64 ? 64 : (n <= 128 ? 128 : kSmallBlock); }
// Motions: a motion test costs ~10x a point test and the planner's shortcut batch (every
// vertex pair of a path, long edges) overlaps many OBBs, so the OBB loop is split finer:
// 16 edges per workgroup, 16 slices of the OBBs (<= 64 workgroups for kSmallMotions edges).
__host__ __device__ inline int small_per_motions(int64_t) { return 16; }
__host__ __device__ inline size_t small_shm(int n_obb) { return (((size_t)n_obb * kRecDoubles + 1) & ~size_t(1)) * 8 + kSmallBlock * 4; }

// The body of k_states_small for logical workgroup `blk` (its queries [blk per, (blk+1)
// per)), with `srec` the workgroup's dynamic LDS (small_shm bytes).  Also run by the fused
// check + refit kernel (minsnap.hip, k_check_refit) on the workgroups after the refit's.
template <bool MINDIST, bool COMPACT>
__device__ __forceinline__ void states_small_body(double* srec, int blk, const double* __restrict__ recs, int n_obb,
                                                  double rg, double ro, const double* __restrict__ xyz, int64_t n,
                                                  int per, int can_pass, double md, uint8_t* __restrict__ valid,
                                                  int32_t* __restrict__ compact_idx,
                                                  unsigned long long* __restrict__ n_valid) {
    uint32_t* s_hit = reinterpret_cast<uint32_t*>(srec + (((size_t)n_obb * kRecDoubles + 1) & ~size_t(1)));
    const int t = threadIdx.x, slices = kSmallBlock / per, slice = t / per, j = t - slice * per;
    const int64_t i = (int64_t)blk * per + j;
    const bool act = i < n;
    double px = 0.0, py = 0.0, pz = 0.0;
    stage_records(srec, recs, n_obb * kRecDoubles, [&] {
        if (act) {
            px = xyz[3 * i];
            py = xyz[3 * i + 1];
            pz = xyz[3 * i + 2];
        }
    });
    if (t < per) s_hit[t] = 0u;
    __syncthreads();
    const int o0 = (int)((int64_t)slice * n_obb / slices), o1 = (int)((int64_t)(slice + 1) * n_obb / slices);
    const bool cp = can_pass != 0;
    // rtree contains(point): strict  src/World.cpp:83
    auto inside = [&](const double* r) {
        return act & (r[F_LOX] < px) & (px < r[F_HIX]) & (r[F_LOY] < py) & (py < r[F_HIY]) & (r[F_LOZ] < pz) &
               (pz < r[F_HIZ]);
    };
    bool hit = false;
    int o = o0;
    for (; o + 4 <= o1; o += 4) {  // four records' AABB tests before any branch (their LDS reads overlap)
        const double* r = srec + (size_t)o * kRecDoubles;
        const bool in0 = inside(r), in1 = inside(r + kRecDoubles), in2 = inside(r + 2 * kRecDoubles),
                   in3 = inside(r + 3 * kRecDoubles);
        if (__builtin_amdgcn_ballot_w64(in0 | in1 | in2 | in3)) {
            hit |= in0 && rec_hit<MINDIST>(r, rg, ro, px, py, pz, cp, md);
            hit |= in1 && rec_hit<MINDIST>(r + kRecDoubles, rg, ro, px, py, pz, cp, md);
            hit |= in2 && rec_hit<MINDIST>(r + 2 * kRecDoubles, rg, ro, px, py, pz, cp, md);
            hit |= in3 && rec_hit<MINDIST>(r + 3 * kRecDoubles, rg, ro, px, py, pz, cp, md);
        }
    }
    for (; o < o1; ++o) {
        const double* r = srec + (size_t)o * kRecDoubles;
        const bool in = inside(r);
        if (__builtin_amdgcn_ballot_w64(in)) hit |= in && rec_hit<MINDIST>(r, rg, ro, px, py, pz, cp, md);
    }
    if (hit) s_hit[j] = 1u;
    __syncthreads();
    if (slice == 0 && act) {
        const bool ok = s_hit[j] == 0u;
        valid[i] = ok ? 1 : 0;
        if (COMPACT && ok) compact_idx[atomicAdd(n_valid, 1ull)] = (int32_t)i;
    }
}

}  // namespace
}  // namespace epp

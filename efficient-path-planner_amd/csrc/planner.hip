// planner.hip — device building blocks of the batch planner that replaces OMPL's
// RRT*/FMT* driver behind PathPlanner::planPath (src/PathPlanner.cpp:80-158):
//
//   k_sample_uniform : counter-based uniform state sampler (splitmix64) —
//                      the state sampler OMPL's RealVectorStateSpace would provide
//   k_knn            : k nearest neighbours of every node (brute force, LDS-tiled)
//   k_knn_edges      : gathers the candidate edges (node, neighbour) for the motion check
//
// Validity of the sampled states and of the edges is checked by the collision kernels
// (collision.hip); the host runs the shortest-path search over the valid edges.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cstdio>
#include <mutex>
#include <string>

#include "cached_ws.h"
#include "completion.h"
#include "epp_internal.h"

namespace epp {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// (clr, nclr: words a later kernel on the stream needs zeroed -- the planner's compaction
// status words -- cleared here instead of by a separate fill launch)
__global__ void k_sample_uniform(uint64_t seed, double lox, double loy, double loz, double hix,
                                 double hiy, double hiz, int64_t n, int64_t start,
                                 double* __restrict__ xyz, unsigned long long* __restrict__ clr, int64_t nclr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nclr) clr[i] = 0ull;
    if (i >= n) return;
    const uint64_t c = (uint64_t)(start + i) * 3ull;
    const double u0 = (double)(splitmix64(seed ^ c) >> 11) * 0x1.0p-53;
    const double u1 = (double)(splitmix64(seed ^ (c + 1)) >> 11) * 0x1.0p-53;
    const double u2 = (double)(splitmix64(seed ^ (c + 2)) >> 11) * 0x1.0p-53;
    xyz[3 * i] = lox + (hix - lox) * u0;
    xyz[3 * i + 1] = loy + (hiy - loy) * u1;
    xyz[3 * i + 2] = loz + (hiz - loz) * u2;
}

constexpr int kKnnBlock = 256;

template <int K>
__global__ __launch_bounds__(kKnnBlock) void k_knn(const double* __restrict__ nodes, int n, double r2max,
                                                   int32_t* __restrict__ nbr) {
    __shared__ double tile[kKnnBlock * 3];
    const int i = blockIdx.x * kKnnBlock + threadIdx.x;
    double px = 0, py = 0, pz = 0;
    if (i < n) {
        px = nodes[3 * i];
        py = nodes[3 * i + 1];
        pz = nodes[3 * i + 2];
    }
    double bd[K];
    int bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bd[k] = r2max;
        bi[k] = -1;
    }
    for (int t0 = 0; t0 < n; t0 += kKnnBlock) {
        const int j = t0 + threadIdx.x;
        __syncthreads();
        if (j < n) {
            tile[3 * threadIdx.x] = nodes[3 * j];
            tile[3 * threadIdx.x + 1] = nodes[3 * j + 1];
            tile[3 * threadIdx.x + 2] = nodes[3 * j + 2];
        }
        __syncthreads();
        const int m = min(kKnnBlock, n - t0);
        for (int c = 0; c < m; ++c) {
            const double dx = tile[3 * c] - px, dy = tile[3 * c + 1] - py, dz = tile[3 * c + 2] - pz;
            const double d = (dx * dx + dy * dy) + dz * dz;
            if (d < bd[K - 1] && t0 + c != i) {  // strict: earlier index wins ties
                double vd = d;
                int vi = t0 + c;
                bool shift = false;  // once placed, the tail shifts down by one (keeps tie order)
#pragma unroll
                for (int k = 0; k < K; ++k) {  // insertion after any equal distances
                    shift = shift || vd < bd[k];
                    if (shift) {
                        const double td = bd[k];
                        const int ti = bi[k];
                        bd[k] = vd;
                        bi[k] = vi;
                        vd = td;
                        vi = ti;
                    }
                }
            }
        }
    }
    if (i < n)
#pragma unroll
        for (int k = 0; k < K; ++k) nbr[(int64_t)i * K + k] = bi[k];
}

// ---- k-NN over a uniform grid (exact; same answer as k_knn) ------------------------
// Cells of edge h hold ~3 nodes; every query walks shells of cells around its own cell
// until the k-th best squared distance is below the squared distance to the nearest
// face of the searched block (minus a rounding margin) — then no unvisited node can
// enter the list.  Candidates are ranked by (distance, index), so the visiting order
// (atomics in the scatter) never changes the result.
struct KnnGrid {
    double lo[3];
    double h, inv_h;
    int dims[3];
    int ncell;
    int next;    // k_knn_tile's block queue
    int nretry;  // k_knn_tile's retry list length
    int why[4];  // retry causes (diagnostics): list overflow, K-th beyond Dcut, shell rule, crowded (or spilled)
    // the planner's row-restricted k-NN (k_knn_list_ellipse): the ellipsoid
    // |x - qs| + |x - qg| <= qbound (1e300: unused)
    double qs[3], qg[3], qbound;
};

constexpr int kBoundsThreads = 1024;
constexpr int kBoundsBlocks = 64;
constexpr int kKnnDefaultTile = 1;     // grid k-NN kernel without EPP_KNN_TILE: 1 k_knn_tile, 2 k_knn_wave
constexpr double kNodesPerCell = 1.5;  // mean nodes per grid cell (EPP_KNN_NPC overrides in -DEPP_KNN_DIAG builds; tuned for k_knn_tile: ~90 queries per 4^3 block -> 2 lanes each)

// The grid over the box [mn, mx] for n nodes: cells of edge h with ~npc nodes each (flat
// point sets: thin slabs), at most cap cells.  Host (caller-given box) and device (the
// nodes' bounding box) compute it the same way.
__host__ __device__ inline void knn_grid_shape(const double (&mn)[3], const double (&mx)[3], int n, int cap,
                                               double npc, KnnGrid* g) {
    double ext[3], vol = 1.0, emax = 0.0;
    for (int d = 0; d < 3; ++d) {
        ext[d] = mx[d] - mn[d];
        emax = fmax(emax, ext[d]);
    }
    const double floor_ext = fmax(emax, 1e-9) * 1e-3;
    for (int d = 0; d < 3; ++d) vol *= fmax(ext[d], floor_ext);
    double h = cbrt(npc * vol / (double)(n > 1 ? n : 1));
    h = fmax(h, 1e-12);
    int dims[3];
    long long cells;
    for (;;) {
        cells = 1;
        for (int d = 0; d < 3; ++d) {
            dims[d] = (int)fmin(ext[d] / h, 1023.0) + 1;
            cells *= dims[d];
        }
        if (cells <= cap) break;
        h *= 1.25;
    }
    for (int d = 0; d < 3; ++d) {
        g->lo[d] = mn[d];
        g->dims[d] = dims[d];
    }
    g->h = h;
    g->inv_h = 1.0 / h;
    g->ncell = (int)cells;
    g->next = 0;
    g->nretry = 0;
    for (int i = 0; i < 4; ++i) g->why[i] = 0;
    for (int d = 0; d < 3; ++d) g->qs[d] = g->qg[d] = 0.0;
    g->qbound = 1e300;
}

// Per-block min/max of the node coordinates: part[6 * block] = (min xyz, max xyz).  Also
// clears the cell counters (cnt and fill, nclr ints) for k_knn_count / k_knn_scatter.
__global__ __launch_bounds__(kBoundsThreads) void k_knn_bounds_part(const double* __restrict__ nodes, int n,
                                                                    double* __restrict__ part, int* __restrict__ clr,
                                                                    int nclr) {
    for (int i = blockIdx.x * kBoundsThreads + threadIdx.x; i < nclr; i += gridDim.x * kBoundsThreads) clr[i] = 0;
    __shared__ double smin[3][kBoundsThreads / 64], smax[3][kBoundsThreads / 64];
    double mn[3] = {1e308, 1e308, 1e308}, mx[3] = {-1e308, -1e308, -1e308};
    for (int i = blockIdx.x * kBoundsThreads + threadIdx.x; i < n; i += gridDim.x * kBoundsThreads)
        for (int d = 0; d < 3; ++d) {
            const double v = nodes[3 * i + d];
            mn[d] = fmin(mn[d], v);
            mx[d] = fmax(mx[d], v);
        }
    for (int d = 0; d < 3; ++d)
        for (int o = 32; o > 0; o >>= 1) {
            mn[d] = fmin(mn[d], __shfl_xor(mn[d], o, 64));
            mx[d] = fmax(mx[d], __shfl_xor(mx[d], o, 64));
        }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < 3; ++d) {
            smin[d][wv] = mn[d];
            smax[d][wv] = mx[d];
        }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBoundsThreads / 64; ++w)
            for (int d = 0; d < 3; ++d) {
                mn[d] = fmin(mn[d], smin[d][w]);
                mx[d] = fmax(mx[d], smax[d][w]);
            }
        for (int d = 0; d < 3; ++d) {
            part[6 * blockIdx.x + d] = mn[d];
            part[6 * blockIdx.x + 3 + d] = mx[d];
        }
    }
}

// Grid shape from the block partials (one thread).
__global__ void k_knn_setup(const double* __restrict__ part, int nparts, int n, int cell_cap, double npc,
                            KnnGrid* __restrict__ g) {
    if (threadIdx.x >= 64 || blockIdx.x != 0) return;
    // one wave folds the partials (all loads in flight at once), lane 0 does the rest
    double mn[3] = {1e308, 1e308, 1e308}, mx[3] = {-1e308, -1e308, -1e308};
    for (int b = threadIdx.x; b < nparts; b += 64)
        for (int d = 0; d < 3; ++d) {
            mn[d] = fmin(mn[d], part[6 * b + d]);
            mx[d] = fmax(mx[d], part[6 * b + 3 + d]);
        }
    for (int d = 0; d < 3; ++d)
        for (int o = 32; o > 0; o >>= 1) {
            mn[d] = fmin(mn[d], __shfl_xor(mn[d], o, 64));
            mx[d] = fmax(mx[d], __shfl_xor(mx[d], o, 64));
        }
    if (threadIdx.x != 0) return;
    knn_grid_shape(mn, mx, n, cell_cap, npc, g);
}

// The caller-box path: the grid computed on the host, written here; clears the counters.
__global__ __launch_bounds__(kBoundsThreads) void k_knn_prep(KnnGrid gv, KnnGrid* __restrict__ g,
                                                             int* __restrict__ clr, int nclr) {
    for (int i = blockIdx.x * kBoundsThreads + threadIdx.x; i < nclr; i += gridDim.x * kBoundsThreads) clr[i] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *g = gv;
}

__device__ __forceinline__ int knn_cell_axis(double v, const KnnGrid& g, int d) {
    const int c = (int)((v - g.lo[d]) * g.inv_h);
    return c < 0 ? 0 : (c >= g.dims[d] ? g.dims[d] - 1 : c);
}

__global__ void k_knn_count(const double* __restrict__ nodes, int n, const KnnGrid* __restrict__ gp,
                            int* __restrict__ cell_of, int* __restrict__ cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const KnnGrid g = *gp;
    const int cx = knn_cell_axis(nodes[3 * i], g, 0), cy = knn_cell_axis(nodes[3 * i + 1], g, 1),
              cz = knn_cell_axis(nodes[3 * i + 2], g, 2);
    const int c = (cz * g.dims[1] + cy) * g.dims[0] + cx;
    cell_of[i] = c;
    atomicAdd(&cnt[c], 1);
}

// ---- decoupled look-back (single-pass ordered scans) ---------------------------------
// A block publishes its chunk's total as soon as it has counted it ("aggregate"), then
// its inclusive prefix once it knows its exclusive one.  Its look-back reads the status
// words of the 64 blocks before it at once (one lane each), waits for every one of them to
// be published in this launch, and sums back to the nearest inclusive prefix -- no
// block waits on a chain of predecessors (they publish their aggregates without waiting).
// Status word: [63..40] launch tag (24 bits, never 0), [39] inclusive flag, [38..0] value.
// The status words are zeroed on the stream before every launch (a zero word carries no
// tag, so it reads as unpublished); the tag is a second guard, against a word published by
// an earlier launch on another stream.  Blocks only wait on lower-numbered blocks, which are
// dispatched first, so the wait always ends.
constexpr int kTagShift = 40;
constexpr unsigned long long kIncl = 1ull << 39, kValMask = kIncl - 1ull;
std::atomic<uint32_t> g_scan_tag{0};
uint32_t next_scan_tag() {
    uint32_t t;
    do t = (g_scan_tag.fetch_add(1, std::memory_order_relaxed) + 1u) & 0xffffffu;
    while (t == 0u);
    return t;
}
__device__ __forceinline__ void lb_publish(unsigned long long* st, int b, uint32_t tag, bool incl, long long v) {
    const unsigned long long w = ((unsigned long long)tag << kTagShift) | (incl ? kIncl : 0ull) | ((unsigned long long)v & kValMask);
    __hip_atomic_store(st + b, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Exclusive prefix of block b (called by one whole wavefront; every lane gets it).
__device__ __forceinline__ long long lb_exclusive(unsigned long long* st, int b, uint32_t tag) {
    const int lane = threadIdx.x & 63;
    long long acc = 0;
    for (int hi = b - 1; hi >= 0; hi -= 64) {  // window [hi - 63, hi], lane l reads block hi - l
        const int j = hi - lane;
        unsigned long long w = 0ull;
        if (j >= 0) {
            do w = __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while ((uint32_t)(w >> kTagShift) != tag);
        }
        const unsigned long long pm = __ballot(j >= 0 && (w & kIncl));
        // the nearest inclusive prefix (lowest lane with one) ends the walk
        const int stop = pm ? __builtin_ctzll(pm) : 64;
        long long v = (lane <= stop && j >= 0) ? (long long)(w & kValMask) : 0ll;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc += v;
        if (pm) break;
    }
    return acc;
}

// exclusive scan of cnt[0..ncell) into start[0..ncell]: block b scans cells
// [b kScanTile, (b+1) kScanTile), 16 consecutive counts per thread (16-byte loads and
// stores), its offset by look-back (lb_exclusive).  The grid is
// sized for the largest possible cell count (the count itself is on the device); blocks
// past it exit (no block waits on a later one).
constexpr int kScanThreads = 256, kScanPer = 16, kScanTile = kScanThreads * kScanPer;
__device__ __forceinline__ void knn_scan_block(const KnnGrid* __restrict__ gp, const int* __restrict__ cnt,
                                               int* __restrict__ start, unsigned long long* __restrict__ st,
                                               uint32_t tag, const int b) {
    static_assert(kScanPer % 4 == 0, "16-byte runs");
    __shared__ int wsum[kScanThreads / 64];
    __shared__ int s_excl;
    const int nc = gp->ncell;
    if (b * kScanTile > nc) return;  // (block-uniform; the block holding nc itself writes start[nc])
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b0 = b * kScanTile + kScanPer * threadIdx.x;
    int v[kScanPer];
    if (b0 + kScanPer <= nc) {  // (cnt and start are 256-byte aligned, b0 a multiple of 16)
#pragma unroll
        for (int u = 0; u < kScanPer / 4; ++u) {
            const int4 q = reinterpret_cast<const int4*>(cnt + b0)[u];
            v[4 * u] = q.x;
            v[4 * u + 1] = q.y;
            v[4 * u + 2] = q.z;
            v[4 * u + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < kScanPer; ++u) v[u] = b0 + u < nc ? cnt[b0 + u] : 0;
    }
    int sum = 0;
#pragma unroll
    for (int u = 0; u < kScanPer; ++u) sum += v[u];
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int wbase = 0, tile = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
        wbase += w < wv ? wsum[w] : 0;
        tile += wsum[w];
    }
    if (wv == 0) {
        if (lane == 0) lb_publish(st, b, tag, b == 0, tile);
        const long long ex = b == 0 ? 0ll : lb_exclusive(st, b, tag);
        if (lane == 0) {
            if (b > 0) lb_publish(st, b, tag, true, ex + tile);
            s_excl = (int)ex;
        }
    }
    __syncthreads();
    int acc = s_excl + wbase + incl - sum;
    if (b0 + kScanPer <= nc) {
#pragma unroll
        for (int u = 0; u < kScanPer / 4; ++u) {
            int4 q;
            q.x = acc;
            q.y = q.x + v[4 * u];
            q.z = q.y + v[4 * u + 1];
            q.w = q.z + v[4 * u + 2];
            acc = q.w + v[4 * u + 3];
            reinterpret_cast<int4*>(start + b0)[u] = q;
        }
    } else {
#pragma unroll
        for (int u = 0; u < kScanPer; ++u) {
            if (b0 + u <= nc) start[b0 + u] = acc;  // (b0 + u == nc: the total)
            acc += v[u];
        }
    }
}
__global__ __launch_bounds__(kScanThreads) void k_knn_scan(const KnnGrid* __restrict__ gp,
                                                           const int* __restrict__ cnt,
                                                           int* __restrict__ start,
                                                           unsigned long long* __restrict__ st, uint32_t tag) {
    knn_scan_block(gp, cnt, start, st, tag, blockIdx.x);
}

__global__ void k_knn_scatter(const double* __restrict__ nodes, int n, const int* __restrict__ cell_of,
                              const int* __restrict__ start, int* __restrict__ fill,
                              double* __restrict__ sxyz, int* __restrict__ sidx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int c = cell_of[i];
    const int pos = start[c] + atomicAdd(&fill[c], 1);
    if (pos >= start[c + 1]) return;  // cannot happen with cleared counters; never write out of range
    sidx[pos] = i;
    sxyz[3 * pos] = nodes[3 * i];
    sxyz[3 * pos + 1] = nodes[3 * i + 1];
    sxyz[3 * pos + 2] = nodes[3 * i + 2];
}

// Insert candidate (d, j) into the sorted top-K (distance, then index): ties keep the
// lower index first, so the visiting order never changes the result.  Branch-free: the
// entries ahead of (d, j) form a prefix of the list; each slot keeps its entry, takes
// (d, j), or takes its predecessor -- independent selects instead of a shifting chain of
// per-slot branches (which compiled to ~12 instructions, an exec-mask branch and four
// 64-bit moves per slot).
template <int K>
__device__ __forceinline__ void knn_insert(double (&bd)[K], int (&bi)[K], double d, int j) {
    if (!((d < bd[K - 1]) | ((d == bd[K - 1]) & (j < bi[K - 1])))) return;
    bool ahead[K];  // (bitwise, not short-circuit: no branches)
#pragma unroll
    for (int k = 0; k < K; ++k) ahead[k] = (bd[k] < d) | ((bd[k] == d) & (bi[k] < j));
#pragma unroll
    for (int k = K - 1; k >= 1; --k) {  // (reads slot k-1 before it is rewritten)
        bd[k] = ahead[k] ? bd[k] : (ahead[k - 1] ? d : bd[k - 1]);
        bi[k] = ahead[k] ? bi[k] : (ahead[k - 1] ? j : bi[k - 1]);
    }
    bd[0] = ahead[0] ? bd[0] : d;
    bi[0] = ahead[0] ? bi[0] : j;
}

// Exact stopping rule after shell r: the K-th best squared distance is below the squared
// distance from p to the nearest face of the searched (2r+1)^3 block that has cells
// beyond it (minus a rounding margin).  Also true when no cells are left.
// knn_bound returns that squared distance (+inf: no cells left; 0: never).
__device__ __forceinline__ double knn_bound(const KnnGrid& g, const int (&c)[3], const double (&p)[3], int r) {
    double dmin = 1e300;
    bool all = true;
    for (int d = 0; d < 3; ++d) {
        if (c[d] - r > 0) {
            dmin = fmin(dmin, p[d] - (g.lo[d] + (double)(c[d] - r) * g.h));
            all = false;
        }
        if (c[d] + r < g.dims[d] - 1) {
            dmin = fmin(dmin, (g.lo[d] + (double)(c[d] + r + 1) * g.h) - p[d]);
            all = false;
        }
    }
    if (all) return INFINITY;
    dmin -= g.h * 1e-6;  // cell assignment rounds; stay conservative
    return dmin > 0 ? dmin * dmin : 0.0;
}

template <int K>
__device__ __forceinline__ bool knn_done(const KnnGrid& g, const int (&c)[3], const double (&p)[3], int r,
                                         const double (&bd)[K]) {
    const double b = knn_bound(g, c, p, r);
    return b == INFINITY || bd[K - 1] < b;
}

// Shells r_from, r_from + 1, ... from global memory until knn_done (candidates BATCH
// at a time: their loads are in flight together).
template <int K, int BATCH = 4>
__device__ void knn_walk(const KnnGrid& g, const int (&c)[3], const double (&p)[3], int self, double (&bd)[K],
                         int (&bi)[K], const double* __restrict__ sxyz, const int* __restrict__ sidx,
                         const int* __restrict__ start, int r_from) {
    const int rmax = max(g.dims[0], max(g.dims[1], g.dims[2]));
    for (int r = r_from; r <= rmax; ++r) {
        for (int dz = -r; dz <= r; ++dz) {
            const int z = c[2] + dz;
            if (z < 0 || z >= g.dims[2]) continue;
            for (int dy = -r; dy <= r; ++dy) {
                const int y = c[1] + dy;
                if (y < 0 || y >= g.dims[1]) continue;
                const bool face = (dz == -r || dz == r || dy == -r || dy == r);
                const int step = (face || r == 0) ? 1 : 2 * r;
                for (int dx = -r; dx <= r; dx += step) {
                    const int x = c[0] + dx;
                    if (x < 0 || x >= g.dims[0]) continue;
                    const int cell = (z * g.dims[1] + y) * g.dims[0] + x;
                    const int e = start[cell + 1];
                    for (int q0 = start[cell]; q0 < e; q0 += BATCH) {
                        double dd[BATCH];
                        int jj[BATCH];
#pragma unroll
                        for (int u = 0; u < BATCH; ++u) {
                            const int q = min(q0 + u, e - 1);
                            jj[u] = q0 + u < e ? sidx[q] : self;  // past the cell: skipped below
                            const double ddx = sxyz[3 * q] - p[0], ddy = sxyz[3 * q + 1] - p[1], ddz = sxyz[3 * q + 2] - p[2];
                            dd[u] = (ddx * ddx + ddy * ddy) + ddz * ddz;
                        }
#pragma unroll
                        for (int u = 0; u < BATCH; ++u)
                            if (jj[u] != self) knn_insert<K>(bd, bi, dd[u], jj[u]);
                    }
                }
            }
        }
        if (knn_done<K>(g, c, p, r, bd)) break;
    }
}

template <int K>
__global__ __launch_bounds__(256) void k_knn_grid(const KnnGrid* __restrict__ gp, int n, double r2max,
                                                  const double* __restrict__ sxyz,
                                                  const int* __restrict__ sidx,
                                                  const int* __restrict__ start,
                                                  int32_t* __restrict__ nbr) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;  // queries in cell order: coherent walks
    if (t >= n) return;
    const KnnGrid g = *gp;
    const int self = sidx[t];
    const double p[3] = {sxyz[3 * t], sxyz[3 * t + 1], sxyz[3 * t + 2]};
    const int c[3] = {knn_cell_axis(p[0], g, 0), knn_cell_axis(p[1], g, 1), knn_cell_axis(p[2], g, 2)};
    double bd[K];
    int bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bd[k] = r2max;
        bi[k] = 0x7fffffff;
    }
    knn_walk<K>(g, c, p, self, bd, bi, sxyz, sidx, start, 0);
#pragma unroll
    for (int k = 0; k < K; ++k) nbr[(int64_t)self * K + k] = bi[k] == 0x7fffffff ? -1 : bi[k];
}

// ---- tiled grid k-NN ----------------------------------------------------------------
// A workgroup takes a block of kTileB^3 cells: the block plus a kTileH-cell halo is
// copied into LDS and every query of the block looks at the kTileW^3 cube of cells
// around its own (shells 0..kTileH) out of LDS.  The per-query walk of k_knn_grid is
// bound by dependent global round trips; here they are LDS reads.
//
// Selection.  The sorted top-K insert costs ~K*12 VALU per candidate, and a wave pays
// it whenever any of its lanes inserts -- nearly always.  So the cube is scanned twice
// on float coordinates (relative to the block centre, one 16-byte LDS record per
// candidate): pass 1 histograms the squared distances into kTileNB quarter-octave bins;
// the bin where the running count reaches K gives a bound Dcut; pass 2 lists the
// candidates with float distance below Dcut + 2*delta (<= kTileL per query).  Only the
// listed candidates get an exact (double, from global memory) distance and the insert.
// delta bounds the float error of a squared distance within a halo (<= ~1e-4 h^2; 1e-3
// h^2 is used), so every candidate with exact d <= Dcut is listed; if the exact K-th
// distance is <= Dcut the result is therefore exact.  Queries where that check, the
// list size or the exact stopping rule after shell kTileH fails -- and all queries of a
// halo over capacity -- go to a retry list that k_knn_retry walks from global memory.
//
// Lanes per query: a block holds ~64..160 queries at ~2 nodes per cell; with fewer
// queries than threads, 2 or 4 adjacent lanes share one query (cube rows split between
// them; the histogram and the list are shared through LDS atomics), so blocks take about
// the same time whatever their query count.  Blocks come from a queue (costs differ).
// (Splitting blocks of more than 128 queries into two z-layer work units was tried in
// round 4: at ~1.5 nodes per cell the C4 tables have as many blocks as resident
// workgroups, so a second half only starts once a workgroup is free -- it lengthened the
// launch, 99 -> 110 us in the isolated trace.  A per-lane register histogram in pass 1
// instead of the LDS atomics was tried too; its build faulted in the crowded-cluster test
// and was withdrawn.  So was a first pass-1 stage over the 3^3 cells around the query: its
// cut alone is a valid but looser bound (exact phase 22 -> 29 us p50), and completing the
// bins below it from the rest of the cube takes two walks where one did (pass 1 19.8 ->
// 24.2 us p50; blocks at the grid's edges, where the 3^3 cells hold fewer than K, 42-50).)
#ifdef EPP_KNN_DIAG
constexpr int kKnnTlBlocks = 65536;  // timeline records
constexpr int kKnnRetryTl = 4096;    // retried queries recorded (k_knn_retry)
__device__ unsigned long long g_knn_retry_tl[kKnnRetryTl][4];
#endif
// Device asserts of k_knn_tile's invariants in the diagnostics build (-DEPP_KNN_DIAG); the
// product guards them instead (the query then takes the retry path)
#ifdef EPP_KNN_DIAG
#define EPP_KNN_ASSERT(c) assert(c)
#else
#define EPP_KNN_ASSERT(c) \
    do {                 \
    } while (0)
#endif
constexpr int kTileB = 4, kTileH = 2, kTileE = kTileB + 2 * kTileH, kTileCells = kTileE * kTileE * kTileE;
constexpr int kTileW = 2 * kTileH + 1;  // cube edge around the query's cell
constexpr int kTileRows = kTileW * kTileW;
constexpr int kTileCap = 1344;          // candidates a halo may hold (else its queries retry)
constexpr int kTileThreads = 256;
constexpr int kTileL = 32;              // per-query list length
constexpr int kTileNB = 16;             // histogram bins (16-bit counters, two per word)
constexpr int kTileSpill = 32;          // queries past 128 a block sends to the retry list (see below)
constexpr double kTileDelta = 1e-3;     // float error allowance, in h^2
#ifndef EPP_KNN_PASS1R2  // (diagnostics A/B builds may override; exact either way)
#define EPP_KNN_PASS1R2 4.5
#endif
constexpr double kPass1R2 = EPP_KNN_PASS1R2;  // pass 1 first visits the cells within sqrt(4.5) h

// A halo candidate in LDS.  Default: float x, y, z relative to the block centre + the
// node's sorted position (16 B).  EPP_KNN_PACK8 (A/B): x, y, z as 21-bit fixed point over
// [-4h, 4h) (quantum q = 4h / 2^20 ~ 3.8e-6 h) in 8 bytes, the sorted positions in a
// separate array read only by the exact phase -- half the LDS bytes per candidate in
// passes 1 and 2.  The squared distance from the integer differences (exact in float) times
// q^2 is within ~7e-5 h^2 of the exact one (|difference| <= 3h per axis, each coordinate
// rounded by <= q / 2), inside kTileDelta.
#ifdef EPP_KNN_PACK8
typedef uint2 TileCand;
struct TileQ {
    int x, y, z;
};
__device__ __forceinline__ TileQ tile_q(const uint2 c) {
    return {(int)(c.x & 0x1FFFFFu), (int)((c.x >> 21) | ((c.y & 0x3FFu) << 11)), (int)(c.y >> 10)};
}
__device__ __forceinline__ float tile_d(const uint2 c, const TileQ& p, float kq2) {
    const TileQ t = tile_q(c);
    const float dx = (float)(t.x - p.x), dy = (float)(t.y - p.y), dz = (float)(t.z - p.z);
    return ((dx * dx + dy * dy) + dz * dz) * kq2;
}
__device__ __forceinline__ int tile_key(const uint2, int q) { return q; }  // (self test: the LDS position)
#else
typedef float4 TileCand;
typedef float4 TileQ;
__device__ __forceinline__ TileQ tile_q(const float4 c) { return c; }
__device__ __forceinline__ float tile_d(const float4 c, const float4& pf, float) {
    const float dx = c.x - pf.x, dy = c.y - pf.y, dz = c.z - pf.z;
    return (dx * dx + dy * dy) + dz * dz;
}
__device__ __forceinline__ int tile_key(const float4 c, int) { return __float_as_int(c.w); }  // (sorted position)
#endif

// Visits the candidates of cube rows row0, row0 + rstep, ... around a query (a row =
// kTileW consecutive halo cells along x, one contiguous LDS range), four candidates at a
// time so their LDS reads are in flight together.  f(q, d_float, key, valid), key = what
// the self test compares (tile_key).
template <class F>
__device__ __forceinline__ void tile_rows(const int* cst, const TileCand* cand, int h0, int row0, int rstep,
                                          const TileQ& pf, float kq2, F&& f) {
    for (int row = row0; row < kTileRows; row += rstep) {
        const int a = h0 + ((row / kTileW) * kTileE + row % kTileW) * kTileE;
        const int q1 = cst[a + kTileW];
        for (int q = cst[a]; q < q1; q += 4) {
            TileCand c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = cand[min(q + u, q1 - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int qq = min(q + u, q1 - 1);
                f(qq, tile_d(c[u], pf, kq2), tile_key(c[u], qq), q + u < q1);
            }
        }
    }
}

// tile_rows restricted to the cells that can hold a candidate with squared distance
// <= thr: a row is skipped when its (y, z) gap alone exceeds thr, else trimmed to the x
// cells within reach (still one contiguous LDS range).  fr = the query's offset inside its
// own cell per axis; gaps are shrunk by a hair, so the culling only ever keeps too much.
__device__ __forceinline__ double tile_gap(int off, double fr, double h) {
    const double g = off < 0 ? fr + (double)(-off - 1) * h : (off > 0 ? (h - fr) + (double)(off - 1) * h : 0.0);
    return fmax(g - 1e-6 * h, 0.0);
}

template <class F>
__device__ __forceinline__ void tile_rows_near(const int* cst, const TileCand* cand, int h0, int row0, int rstep,
                                               const TileQ& pf, float kq2, const double (&fr)[3], double h, double thr,
                                               F&& f) {
    const double gx1 = tile_gap(1, fr[0], h), gx2 = tile_gap(2, fr[0], h);
    const double gxm1 = tile_gap(-1, fr[0], h), gxm2 = tile_gap(-2, fr[0], h);
    for (int row = row0; row < kTileRows; row += rstep) {
        const int rz = row / kTileW, ry = row % kTileW;
        const double gy = tile_gap(ry - kTileH, fr[1], h), gz = tile_gap(rz - kTileH, fr[2], h);
        const double gyz = gy * gy + gz * gz;
        if (gyz > thr) continue;
        const double rem = thr - gyz;
        const int xa = gxm2 * gxm2 <= rem ? 0 : (gxm1 * gxm1 <= rem ? 1 : 2);
        const int xb = gx2 * gx2 <= rem ? 4 : (gx1 * gx1 <= rem ? 3 : 2);
        const int a = h0 + (rz * kTileE + ry) * kTileE;
        const int q1 = cst[a + xb + 1];
        for (int q = cst[a + xa]; q < q1; q += 4) {
            TileCand c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) c[u] = cand[min(q + u, q1 - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int qq = min(q + u, q1 - 1);
                f(qq, tile_d(c[u], pf, kq2), tile_key(c[u], qq), q + u < q1);
            }
        }
    }
}
static_assert(kTileW == 5 && kTileH == 2, "tile_rows_near trims rows of 5 cells");

template <int K>
__device__ __forceinline__ void knn_store(int32_t* __restrict__ nbr, int self, const int (&bi)[K]) {
#pragma unroll
    for (int k = 0; k < K; ++k) nbr[(int64_t)self * K + k] = bi[k] == 0x7fffffff ? -1 : bi[k];
}

// Queries the tile pass could not settle (rare: sparse corners, crowded halos), one
// wave per query so a single far walk does not serialise on dependent global loads:
// lanes take x-rows of cells (each one contiguous range of the cell-sorted nodes) and
// keep their own top-K.  First the cube of radius kTileH + 1, then one shell at a time
// until the stopping rule holds -- tested cheaply as ">= K listed candidates below the
// bound" over all lanes -- then K rounds of a wave-wide (distance, index) arg-min merge
// the lane lists; lane 0 writes the result.  Called by whole waves.
template <int K>
__device__ __forceinline__ void knn_retry_wave(const KnnGrid& g, double r2max, const double* __restrict__ nodes,
                               const double* __restrict__ sxyz, const int* __restrict__ sidx,
                               const int* __restrict__ start, int self, double bound2, int32_t* __restrict__ nbr) {
    const int lane = threadIdx.x & 63;
    const int rmax = max(g.dims[0], max(g.dims[1], g.dims[2]));
    const double p[3] = {nodes[3 * (int64_t)self], nodes[3 * (int64_t)self + 1], nodes[3 * (int64_t)self + 2]};
    const int c[3] = {knn_cell_axis(p[0], g, 0), knn_cell_axis(p[1], g, 1), knn_cell_axis(p[2], g, 2)};
    // Without a bound (a crowded or spilled tile query) a trial bound of (1.6h)^2 is tried
    // first: it holds ~26 nodes at the grid's density (~35 in the dense blocks that spill),
    // and the list is exact whenever it holds at least K (every node outside is farther
    // than every listed one); else the per-lane shell walk below.  ((2h)^2 held ~70 nodes
    // in a spilling block: those retries took 7-16 us against 4.7 for the bounded ones.)
    const bool trial = !(bound2 < 1e299);
    const double b2 = trial ? 2.56 * g.h * g.h : bound2;
    if (b2 < 1e299) {  // wave-uniform
        // K actual candidates lie within sqrt(bound2) (the tile pass found them, with the
        // same exact distances), so the true top K is among the candidates with
        // d <= bound2 in the box p +- sqrt(bound2) (cell mapping monotone; the radius is
        // padded against the rounding of p +- r).  Rows of the box are spread over the
        // lanes; every candidate within the bound goes to an LDS list (a few dozen), and
        // each listed entry's rank in (distance, index) order is counted against the whole
        // list: the K lowest ranks are the answer.  No per-lane sorted lists, no merge
        // rounds.  (A list over capacity falls through to the per-lane walk below.)
        constexpr int kCap = 512;
        __shared__ double s_d[kCap];
        __shared__ int s_j[kCap];
        __shared__ int s_n;
        if (lane == 0) s_n = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the clear before any append
        const double r = sqrt(b2) * (1.0 + 1e-9) + 1e-12 * (1.0 + fabs(p[0]) + fabs(p[1]) + fabs(p[2]));
        int lo[3], hi[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = knn_cell_axis(p[d] - r, g, d);
            hi[d] = knn_cell_axis(p[d] + r, g, d);
        }
        const int ny = hi[1] - lo[1] + 1, nz = hi[2] - lo[2] + 1;
        for (int row = lane; row < ny * nz; row += 64) {
            const int a = ((lo[2] + row / ny) * g.dims[1] + lo[1] + row % ny) * g.dims[0];
            const int e = start[a + hi[0] + 1];
            for (int q0 = start[a + lo[0]]; q0 < e; q0 += 4) {
                double dd[4];
                int jj[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = min(q0 + u, e - 1);
                    jj[u] = q0 + u < e ? sidx[q] : self;  // past the row: skipped below
                    const double ddx = sxyz[3 * q] - p[0], ddy = sxyz[3 * q + 1] - p[1], ddz = sxyz[3 * q + 2] - p[2];
                    dd[u] = (ddx * ddx + ddy * ddy) + ddz * ddz;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (jj[u] != self && dd[u] <= b2 && dd[u] < r2max) {
                        const int at = atomicAdd(&s_n, 1);
                        if (at < kCap) {
                            s_d[at] = dd[u];
                            s_j[at] = jj[u];
                        }
                    }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's appends are complete
        const int cnt = s_n;
        if (cnt <= 64 && (!trial || cnt >= K)) {  // wave-uniform: entry i on lane i
            // ranks against the other entries read by v_readlane (no LDS round trip per
            // entry, which the loop below waits out)
            const bool mine = lane < cnt;
            const double di = mine ? s_d[lane] : 0.0;
            const int ji = mine ? s_j[lane] : 0;
            const int dlo = __double2loint(di), dhi = __double2hiint(di);
            int rank = 0;
            for (int f = 0; f < cnt; ++f) {
                const double df = __hiloint2double(__builtin_amdgcn_readlane(dhi, f), __builtin_amdgcn_readlane(dlo, f));
                rank += ((df < di) | ((df == di) & (__builtin_amdgcn_readlane(ji, f) < ji))) ? 1 : 0;
            }
            if (mine && rank < K) nbr[(int64_t)self * K + rank] = ji;
            if (lane >= cnt && lane < K) nbr[(int64_t)self * K + lane] = -1;  // (fewer than K)
            return;
        }
        if (cnt <= kCap && (!trial || cnt >= K)) {  // wave-uniform
            for (int i = lane; i < cnt; i += 64) {
                const double di = s_d[i];
                const int ji = s_j[i];
                int rank = 0;
                for (int f = 0; f < cnt; ++f) {  // (every lane reads entry f: LDS broadcast)
                    const double df = s_d[f];
                    rank += ((df < di) | ((df == di) & (s_j[f] < ji))) ? 1 : 0;
                }
                if (rank < K) nbr[(int64_t)self * K + rank] = ji;
            }
            for (int k = cnt + lane; k < K; k += 64) nbr[(int64_t)self * K + k] = -1;  // (fewer than K)
            return;
        }
    }
    double bd[K];
    int bi[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        bd[k] = r2max;
        bi[k] = 0x7fffffff;
    }
    // candidates of cells [xa, xb] of row (y, z) into the lane's list
    auto scan = [&](int y, int z, int xa, int xb) {
        const int a = (z * g.dims[1] + y) * g.dims[0];
        const int e = start[a + xb + 1];
        for (int q0 = start[a + xa]; q0 < e; q0 += 4) {
            double dd[4];
            int jj[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = min(q0 + u, e - 1);
                jj[u] = q0 + u < e ? sidx[q] : self;  // past the row: skipped below
                const double ddx = sxyz[3 * q] - p[0], ddy = sxyz[3 * q + 1] - p[1], ddz = sxyz[3 * q + 2] - p[2];
                dd[u] = (ddx * ddx + ddy * ddy) + ddz * ddz;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (jj[u] != self) knn_insert<K>(bd, bi, dd[u], jj[u]);
        }
    };
    if (bound2 < 1e299) {  // wave-uniform
        // K actual candidates lie within sqrt(bound2) (the tile pass found them), so every
        // candidate of the true top K does too: one pass over the cells of the box
        // p +- sqrt(bound2) (the cell mapping is monotone; the radius is padded against
        // the rounding of p +- r), rows spread over the lanes, no stopping rule
        const double r = sqrt(bound2) * (1.0 + 1e-9) + 1e-12 * (1.0 + fabs(p[0]) + fabs(p[1]) + fabs(p[2]));
        int lo[3], hi[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = knn_cell_axis(p[d] - r, g, d);
            hi[d] = knn_cell_axis(p[d] + r, g, d);
        }
        const int ny = hi[1] - lo[1] + 1, nz = hi[2] - lo[2] + 1;
        for (int row = lane; row < ny * nz; row += 64) scan(lo[1] + row % ny, lo[2] + row / ny, lo[0], hi[0]);
    } else {
    for (int R = kTileH + 1;; ++R) {  // wave-uniform
        // rows of shell R (the whole cube the first time)
        const bool cube = R == kTileH + 1;
        const int w = 2 * R + 1;
        for (int row = lane; row < w * w; row += 64) {
            const int dz = row / w - R, dy = row % w - R;
            const int z = c[2] + dz, y = c[1] + dy;
            if (z < 0 || z >= g.dims[2] || y < 0 || y >= g.dims[1]) continue;
            const int xa = max(c[0] - R, 0), xb = min(c[0] + R, g.dims[0] - 1);
            if (cube || dz == -R || dz == R || dy == -R || dy == R) {
                scan(y, z, xa, xb);
            } else {  // inner rows: only the shell's two end cells
                if (c[0] - R >= 0) scan(y, z, c[0] - R, c[0] - R);
                if (c[0] + R < g.dims[0]) scan(y, z, c[0] + R, c[0] + R);
            }
        }
        const double bound = knn_bound(g, c, p, R);
        if (bound != INFINITY && R < rmax && !(r2max < bound)) {  // (radius below it: done)
            int below = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) below += (bi[k] != 0x7fffffff && bd[k] < bound) ? 1 : 0;
            for (int o = 32; o > 0; o >>= 1) below += __shfl_xor(below, o, 64);
            if (below < K) continue;
        }
        break;
    }
    }
    // merge: K rounds of arg-min over the lane list heads
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double md = bd[0];
        int mi = bi[0];
        for (int o = 32; o > 0; o >>= 1) {
            const double od = __shfl_xor(md, o, 64);
            const int oi = __shfl_xor(mi, o, 64);
            if (od < md || (od == md && oi < mi)) {
                md = od;
                mi = oi;
            }
        }
        if (lane == 0) nbr[(int64_t)self * K + k] = mi == 0x7fffffff ? -1 : mi;
        if (mi != 0x7fffffff && bi[0] == mi) {  // the winning lane drops its head
#pragma unroll
            for (int t = 0; t + 1 < K; ++t) {
                bd[t] = bd[t + 1];
                bi[t] = bi[t + 1];
            }
            bd[K - 1] = r2max;
            bi[K - 1] = 0x7fffffff;
        }
    }
}

// (An LDS copy of the halo's exact coordinates for the exact phase was tried: with it two
// workgroups fit per CU instead of three, and the kernel was slower.  So was an exact phase
// with one wavefront per query -- its candidates one per lane, ranks counted by v_readlane,
// 145 -> 114 VGPRs: each query then waits out its own gathers one after another, ~3 us per
// query and wave against ~22 us for all of a block's queries at once on one thread each;
// 126 -> 185 us per table.  And four workgroups per CU (halo cap 992, 24-entry lane lists,
// 128 VGPRs with 5 spilled): 126 -> 142 us per table.)
template <int K>
__global__ __launch_bounds__(kTileThreads, 3) void k_knn_tile(KnnGrid* __restrict__ gp, double r2max,
                                                           const double* __restrict__ nodes,
                                                           const double* __restrict__ sxyz,
                                                           const int* __restrict__ sidx,
                                                           const int* __restrict__ start,
                                                           int* __restrict__ retry, double* __restrict__ retry_b,
                                                           int32_t* __restrict__ nbr, int mode,
                                                           unsigned long long* __restrict__ dbg) {
    __shared__ TileCand cand[kTileCap];                    // x, y, z (block-centre relative) [, sorted position]
#ifdef EPP_KNN_PACK8
    __shared__ int spos[kTileCap];                         // sorted positions (exact phase)
#define EPP_SPOS(q) spos[q]
#else
#define EPP_SPOS(q) __float_as_int(cand[q].w)
#endif
    __shared__ uint16_t qh[kTileCap];                      // the block's queries (LDS positions)
    __shared__ int cst[kTileCells + 1];                    // halo cell -> LDS offset
    __shared__ uint32_t hist[kTileNB / 2][kTileThreads];  // [bin pair][query slot]
    __shared__ uint16_t lst[kTileL][kTileThreads];         // [entry][lane]: each lane's own list
    __shared__ int wsum[kTileThreads / 64];
    __shared__ uint8_t s_nown[kTileThreads];  // list entries per lane (saturated)
    __shared__ int8_t s_cut[kTileThreads];    // histogram cut per query slot
    __shared__ int s_nq, s_b;
    const KnnGrid g = *gp;
    const int nbx = (g.dims[0] + kTileB - 1) / kTileB, nby = (g.dims[1] + kTileB - 1) / kTileB,
              nbz = (g.dims[2] + kTileB - 1) / kTileB;
    const int nblocks = nbx * nby * nbz;
    const int n_nodes = start[g.ncell];  // (the guards below: retry appends, sorted positions)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kPer = kTileCells / kTileThreads;  // halo cells per thread
    static_assert(kTileCells % kTileThreads == 0, "");
    // histogram origin: bins span d in [t0, 16 t0), t0 ~ a quarter of the expected K-th
    // squared distance at ~2 nodes per cell (~(K/16)^(2/3) * 1.5 h^2)
    const float kscale = K <= 4 ? 0.40f : K <= 8 ? 0.63f : 1.0f;
    const double t0 = g.h * g.h * 0.35 * kscale;
    const float inv_t0 = (float)(1.0 / t0);
    const double delta = kTileDelta * g.h * g.h;
#ifdef EPP_KNN_PACK8
    const double qs = 1048576.0 / (4.0 * g.h);              // quanta per unit length
    const float kq2 = (float)(1.0 / (qs * qs));             // squared quantum
#else
    const float kq2 = 1.0f;
#endif
    for (;;) {
        if (threadIdx.x == 0) s_b = atomicAdd(&gp->next, 1);
        __syncthreads();
        const int b = s_b;  // block-uniform
        if (b >= nblocks) break;
        const int bx = b % nbx, by = (b / nbx) % nby, bz = b / (nbx * nby);
        const int ox = bx * kTileB - kTileH, oy = by * kTileB - kTileH, oz = bz * kTileB - kTileH;
        const double cen[3] = {g.lo[0] + (ox + 0.5 * kTileE) * g.h, g.lo[1] + (oy + 0.5 * kTileE) * g.h,
                               g.lo[2] + (oz + 0.5 * kTileE) * g.h};
#ifdef EPP_KNN_DIAG
        // phase timeline (diagnostics builds): begin, halo sizes scanned, halo copied, first
        // query round's pass 1 / pass 2 / exact phase done, all queries done, end; counts
        unsigned long long tl[8] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0};
#define EPP_KTL(k) \
    do {           \
        if (tl[k] == 0ull) tl[k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define EPP_KTL(k) \
    do {           \
    } while (0)
#endif
        // 1. halo cell sizes -> exclusive scan (thread t owns halo cells kPer*t ..)
        int cnt[kPer], cell0[kPer], tot = 0;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int t = kPer * threadIdx.x + u;
            const int x = ox + t % kTileE, y = oy + (t / kTileE) % kTileE, z = oz + t / (kTileE * kTileE);
            const bool in = x >= 0 && x < g.dims[0] && y >= 0 && y < g.dims[1] && z >= 0 && z < g.dims[2];
            const int cell = in ? (z * g.dims[1] + y) * g.dims[0] + x : 0;
            const int s0 = start[cell], s1 = start[cell + 1];
            cnt[u] = in ? s1 - s0 : 0;
            cell0[u] = s0;
            tot += cnt[u];
        }
        int incl = tot;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int base = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kTileThreads / 64; ++w) {
            base += w < wv ? wsum[w] : 0;
            total += wsum[w];
        }
        base += incl - tot;
        {
            int acc = base;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                cst[kPer * threadIdx.x + u] = acc;
                acc += cnt[u];
            }
        }
        if (threadIdx.x == 0) {
            cst[kTileCells] = total;
            s_nq = 0;
        }
        __syncthreads();
        EPP_KTL(1);
        if (total <= kTileCap) {  // block-uniform
            // 2. copy the halo's candidates; list the block's own nodes as queries
            int acc = base;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int t = kPer * threadIdx.x + u;
                const int hx = t % kTileE, hy = (t / kTileE) % kTileE, hz = t / (kTileE * kTileE);
                const bool inner = hx >= kTileH && hx < kTileH + kTileB && hy >= kTileH && hy < kTileH + kTileB &&
                                   hz >= kTileH && hz < kTileH + kTileB;
                const int q0 = (inner && cnt[u]) ? atomicAdd(&s_nq, cnt[u]) : 0;
                for (int q = 0; q < cnt[u]; ++q) {
                    const int sg = cell0[u] + q;
                    const double x = sxyz[3 * sg], y = sxyz[3 * sg + 1], z = sxyz[3 * sg + 2];
#ifdef EPP_KNN_PACK8
                    auto qz = [&](double v) {
                        const int i = (int)rint(v * qs) + (1 << 20);
                        return (uint32_t)min(max(i, 0), (1 << 21) - 1);
                    };
                    const uint32_t ux = qz(x - cen[0]), uy = qz(y - cen[1]), uz = qz(z - cen[2]);
                    cand[acc + q] = make_uint2(ux | (uy << 21), (uy >> 11) | (uz << 10));
                    spos[acc + q] = sg;
#else
                    cand[acc + q] = make_float4((float)(x - cen[0]), (float)(y - cen[1]), (float)(z - cen[2]),
                                                __int_as_float(sg));  // (sorted position: see the exact phase)
#endif
                    if (inner) qh[q0 + q] = (uint16_t)(acc + q);
                }
                acc += cnt[u];
            }
            __syncthreads();
            EPP_KTL(2);
            // 3. queries, lpq adjacent lanes per query
#ifdef EPP_KNN_DIAG
            const int nq_all = mode == 4 ? 0 : s_nq;  // mode 4: timing ablation (inexact; diagnostics builds only)
#else
            const int nq_all = s_nq;
#endif
            // block-uniform; one lane per query only above 128 + kTileSpill queries (a second
            // round of queries would cost the block ~45 us).  A block just past 128 queries
            // keeps two lanes per query for its first 128 and sends the rest to the retry list
            // (one wave each in k_knn_retry, in parallel): with one lane per query such a
            // block was the launch's slowest (~104 us against ~85 for the next).
            const bool spill = nq_all > kTileThreads / 2 && nq_all <= kTileThreads / 2 + kTileSpill;
            const int nq = spill ? kTileThreads / 2 : nq_all;
            if (spill)
                for (int q = nq + (int)threadIdx.x; q < nq_all; q += kTileThreads) {
                    const int at = atomicAdd(&gp->nretry, 1);
                    EPP_KNN_ASSERT(at < n_nodes);
                    if (at >= n_nodes) continue;
                    retry[at] = sidx[EPP_SPOS(qh[q])];
                    retry_b[at] = INFINITY;
                    atomicAdd(&gp->why[3], 1);
                }
            const int lpq = nq <= kTileThreads / 4 ? 4 : nq <= kTileThreads / 2 ? 2 : 1;
            const int slot = threadIdx.x / lpq, sub = threadIdx.x % lpq;
            // (a query's lpq lanes are adjacent lanes of one wave: its histogram needs no
            // workgroup barrier; the exact phase reads the lists on other threads, after one)
            for (int qb = 0; qb < nq; qb += kTileThreads / lpq) {  // block-uniform
                const int qi = qb + slot;
                const bool live = qi < nq;
                const int me = live ? qh[qi] : 0;
                const TileQ pf = tile_q(cand[me]);
                const int sself = EPP_SPOS(me);  // the query's sorted position
                const int skey = tile_key(cand[me], me);  // what its self test compares
                // exact coordinates and cell (the row offsets; the final distances)
                const double p[3] = {sxyz[3 * (int64_t)sself], sxyz[3 * (int64_t)sself + 1], sxyz[3 * (int64_t)sself + 2]};
                const int c[3] = {knn_cell_axis(p[0], g, 0), knn_cell_axis(p[1], g, 1), knn_cell_axis(p[2], g, 2)};
                const int h0 = ((c[2] - oz - kTileH) * kTileE + (c[1] - oy - kTileH)) * kTileE + (c[0] - ox - kTileH);
                const double fr[3] = {p[0] - (g.lo[0] + (double)c[0] * g.h), p[1] - (g.lo[1] + (double)c[1] * g.h),
                                      p[2] - (g.lo[2] + (double)c[2] * g.h)};
                // pass 1: histogram of bin keys (exponent + two mantissa bits of d / t0): the
                // query's slot of `hist`, LDS atomics from its lanes (one wave: in-order LDS
                // operations order the clear before them and the read after).  First over
                // the cells within sqrt(kPass1R2) h only (about half the cube); its counts
                // are complete for every bin ending below kPass1R2 h^2 - delta (a candidate
                // of a skipped cell has exact d > kPass1R2 h^2, float d > that - delta), so
                // its cut stands when it ends there -- nearly always; else the whole cube.
                int cut = -1;
                for (int full = 0; full < 2; ++full) {  // query-uniform (the slot's lanes read one histogram)
                    if (sub == 0) {
#pragma unroll
                        for (int w = 0; w < kTileNB / 2; ++w) hist[w][slot] = 0u;
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    auto bin = [&](int, float d, int j, bool valid) {
                        const int kb = max((int)(__float_as_uint(d * inv_t0) >> 21) - (127 << 2), 0);
                        if (valid && j != skey && kb < kTileNB) atomicAdd(&hist[kb >> 1][slot], 1u << ((kb & 1) << 4));
                    };
                    if (live) {
                        if (full) tile_rows(cst, cand, h0, sub, lpq, pf, kq2, bin);
                        else tile_rows_near(cst, cand, h0, sub, lpq, pf, kq2, fr, g.h, kPass1R2 * g.h * g.h, bin);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    int run = 0;
                    cut = -1;
#pragma unroll
                    for (int w = 0; w < kTileNB / 2; ++w) {
                        const uint32_t hv = hist[w][slot];
                        run += hv & 0xffff;
                        if (run >= K && cut < 0) cut = 2 * w;
                        run += hv >> 16;
                        if (run >= K && cut < 0) cut = 2 * w + 1;
                    }
                    const double edge = cut < 0 ? INFINITY : (double)__uint_as_float((uint32_t)(cut + 1 + (127 << 2)) << 21) * t0;
                    if (full || edge <= kPass1R2 * g.h * g.h - delta) break;
                }
                EPP_KTL(3);
                // Dcut: upper edge of bin `cut` (none reached K: no bound)
                const double dcut = cut < 0 ? INFINITY : (double)__uint_as_float((uint32_t)(cut + 1 + (127 << 2)) << 21) * t0;
                const float dlist = (float)(dcut + 2.0 * delta);
                // pass 2: list the candidates below Dcut + 2 delta, visiting only the cells
                // within Dcut + 3 delta (a candidate's float distance is within delta of
                // its exact one, which is at least its cell's distance); every lane keeps
                // its own list (its column of lst: no atomics)
                int nown = 0;
                if (live) {
                    const double thr2 = cut < 0 ? INFINITY : dcut + 3.0 * delta;
                    tile_rows_near(cst, cand, h0, sub, lpq, pf, kq2, fr, g.h, thr2, [&](int q, float d, int j, bool valid) {
                        if (valid && j != skey && d < dlist) {
                            if (nown < kTileL) lst[nown][threadIdx.x] = (uint16_t)q;
                            ++nown;
                        }
                    });
                }
                // The exact phase runs compacted: query slot t on thread t, i.e. the first
                // 256 / lpq threads as full waves (with lpq lanes per query only one lane of
                // each would work, and the idle lanes would still take the SIMD's issue
                // cycles).  The list counts and cuts go through LDS, ordered by a barrier.
                s_nown[threadIdx.x] = (uint8_t)min(nown, 255);
                if (sub == 0) s_cut[slot] = (int8_t)cut;
                __syncthreads();
                EPP_KTL(4);
                const int qx = qb + (int)threadIdx.x;
                if ((int)threadIdx.x < kTileThreads / lpq && qx < nq) {
                const int tcol = (int)threadIdx.x * lpq;  // the query's first list column
                const int sx = EPP_SPOS(qh[qx]);
                const int self = sidx[sx];
                const double p[3] = {sxyz[3 * (int64_t)sx], sxyz[3 * (int64_t)sx + 1], sxyz[3 * (int64_t)sx + 2]};
                const int c[3] = {knn_cell_axis(p[0], g, 0), knn_cell_axis(p[1], g, 1), knn_cell_axis(p[2], g, 2)};
                const int cutx = s_cut[threadIdx.x];
                const double dcut = cutx < 0 ? INFINITY : (double)__uint_as_float((uint32_t)(cutx + 1 + (127 << 2)) << 21) * t0;
                int ncol[4];
#pragma unroll
                for (int o = 0; o < 4; ++o) ncol[o] = o < lpq ? (int)s_nown[tcol + o] : 0;
                int nl = 0;
                bool ok = true;
                double rbound = INFINITY;  // (none: the retry walks shells)
#pragma unroll
                for (int o = 0; o < 4; ++o)
                    if (o < lpq) {
                        nl += ncol[o];
                        ok = ok && ncol[o] <= kTileL;
                    }
                if (ok) {
                    double bd[K];
                    int bi[K];
                    bool guard_ok = true;
                    const int tot_halo = cst[kTileCells];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        bd[k] = r2max;
                        bi[k] = 0x7fffffff;
                    }
                    // exact distances of the listed candidates (the query's lanes' columns in
                    // turn), kLoads at a time in flight
                    constexpr int kLoads = 4;
                    for (int i0 = 0; i0 < nl; i0 += kLoads) {
                        double dd[kLoads];
                        int jj[kLoads];
#pragma unroll
                        for (int u = 0; u < kLoads; ++u) {
                            int e = min(i0 + u, nl - 1), col = 0;  // entry e -> (lane column, row)
                            bool go = true;
#pragma unroll
                            for (int o = 0; o < 3; ++o) {
                                const bool past = (go & (o + 1 < lpq)) & (e >= ncol[o]);
                                e -= past ? ncol[o] : 0;
                                col += past ? 1 : 0;
                                go = past;
                            }
                            // (the halo's entries are its cells' contiguous runs of the cell-sorted
                            // copy: these gathers hit the few KB the block's queries share in L1,
                            // where the nodes' original order scattered them over the table)
                            // (guards: a listed LDS position inside the halo, its sorted position
                            // inside the table -- what a wrong pass-1 cut or list could break; a
                            // failed guard sends the query to the retry instead of reading out of
                            // range; the diagnostics build asserts them)
                            const int q0 = lst[e][tcol + col];
                            const bool qok = q0 >= 0 && q0 < tot_halo;
                            const int q = qok ? q0 : 0;
                            const int sg0 = EPP_SPOS(q);
                            const bool sok = sg0 >= 0 && sg0 < n_nodes;
                            EPP_KNN_ASSERT(qok && sok);
                            guard_ok = guard_ok && qok && sok;
                            const int sg = sok ? sg0 : 0;
                            jj[u] = sidx[sg];
                            const double ddx = sxyz[3 * (int64_t)sg] - p[0], ddy = sxyz[3 * (int64_t)sg + 1] - p[1],
                                         ddz = sxyz[3 * (int64_t)sg + 2] - p[2];
                            dd[u] = (ddx * ddx + ddy * ddy) + ddz * ddz;
                        }
#ifdef EPP_KNN_DIAG
                        if (mode == 5 || mode == 6) {  // timing ablation (inexact): no inserts
                            bd[0] = fmin(bd[0], fmin(fmin(dd[0], dd[1]), fmin(dd[2], dd[3])));
                            continue;
                        }
#endif
#pragma unroll
                        for (int u = 0; u < kLoads; ++u)
                            if (i0 + u < nl) knn_insert<K>(bd, bi, dd[u], jj[u]);
                    }
                    // exact when the K-th distance is within the listed range and the cube
                    // suffices (stopping rule after shell kTileH)
                    const bool in_range = bd[K - 1] <= dcut;
                    ok = guard_ok && in_range && knn_done<K>(g, c, p, kTileH, bd);
#ifdef EPP_KNN_DIAG
                    if (mode == 5 || mode == 6) ok = true;  // (ablation: no retries, no answer)
                    else
#endif
                    if (ok) knn_store<K>(nbr, self, bi);
                    else atomicAdd(&gp->why[in_range ? 2 : 1], 1);
                    // a retry's search bound: K actual candidates within bd[K-1] (<= r2max)
                    rbound = bd[K - 1];
                } else {
                    atomicAdd(&gp->why[0], 1);
                }
                if (!ok) {
                    const int at = atomicAdd(&gp->nretry, 1);
                    EPP_KNN_ASSERT(at < n_nodes);
                    if (at < n_nodes) {  // (each node retries at most once: at < n)
                        retry[at] = self;
                        retry_b[at] = rbound;
                    }
                }
#ifdef EPP_KNN_DIAG
                if (tl[5] == 0ull) tl[5] = __builtin_amdgcn_s_memrealtime();
#endif
                }
                __syncthreads();  // the next round rewrites the lists, histograms and counts
            }
            EPP_KTL(6);
        } else {
            // crowded halo: the block's queries retry from global memory
            for (int t2 = threadIdx.x; t2 < kTileB * kTileB * kTileB; t2 += kTileThreads) {
                const int x = bx * kTileB + t2 % kTileB, y = by * kTileB + (t2 / kTileB) % kTileB,
                          z = bz * kTileB + t2 / (kTileB * kTileB);
                if (x >= g.dims[0] || y >= g.dims[1] || z >= g.dims[2]) continue;
                const int cell = (z * g.dims[1] + y) * g.dims[0] + x;
                const int e = start[cell + 1];
                for (int t = start[cell]; t < e; ++t) {
                    const int at = atomicAdd(&gp->nretry, 1);
                    EPP_KNN_ASSERT(at < n_nodes);
                    if (at >= n_nodes) continue;
                    retry[at] = sidx[t];
                    retry_b[at] = INFINITY;
                }
                if (e > start[cell]) atomicAdd(&gp->why[3], e - start[cell]);
            }
        }
        __syncthreads();  // the LDS tile is rewritten by the next block
#ifdef EPP_KNN_DIAG
        if (dbg && threadIdx.x == 0 && b < kKnnTlBlocks) {  // (thread 0 is a query lane of slot 0)
            tl[7] = __builtin_amdgcn_s_memrealtime();
            for (int k = 0; k < 8; ++k) dbg[16 * b + k] = tl[k];
            dbg[16 * b + 8] = (unsigned long long)s_nq;
            dbg[16 * b + 9] = (unsigned long long)total;
            dbg[16 * b + 10] = blockIdx.x;
        }
#endif
    }
}

// The planner's row-restricted k-NN: the nodes x with |x - qs| + |x - qg| <= qbound (widened
// by 1e-8 relative + 1e-6 m, looser than k_pack_ellipse_rows' test) listed as unbounded
// retry queries, so k_knn_retry answers exactly them, one wave each: a few thousand
// queries spread over the whole chip instead of k_knn_tile's blocks, each of which takes
// the whole kernel's ~80 us latency however few of them run.  After the scatter (the retry
// list reuses cell_of).
__global__ __launch_bounds__(256) void k_knn_list_ellipse(KnnGrid* __restrict__ gp, const double* __restrict__ nodes,
                                                          int n, int* __restrict__ retry,
                                                          double* __restrict__ retry_b) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < n) {
        const double* q = gp->qs;
        const double* r = gp->qg;
        const double x = nodes[3 * i], y = nodes[3 * i + 1], z = nodes[3 * i + 2];
        const double ds = sqrt((x - q[0]) * (x - q[0]) + (y - q[1]) * (y - q[1]) + (z - q[2]) * (z - q[2]));
        const double dg = sqrt((x - r[0]) * (x - r[0]) + (y - r[1]) * (y - r[1]) + (z - r[2]) * (z - r[2]));
        in = ds + dg <= gp->qbound * (1.0 + 1e-8) + 1e-6;
    }
    const unsigned long long bal = __ballot(in);
    if (!bal) return;  // (uniform per wave)
    const int lane = threadIdx.x & 63;
    const int first = __ffsll(bal) - 1;
    int base = 0;
    if (lane == first) base = atomicAdd(&gp->nretry, __popcll(bal));
    base = __shfl(base, first, 64);
    if (!in) return;
    const int at = base + __popcll(bal & ((1ull << lane) - 1ull));
    retry[at] = i;
    retry_b[at] = INFINITY;
}

// Retry list of k_knn_tile: one wave per query (knn_retry_wave).
// One wavefront per workgroup.  (knn_retry_wave is inlined: as a call it took the grid
// parameters by reference to the caller's local copy, which then lived in scratch --
// global-memory round trips on every cell index.)
template <int K>
__global__ __launch_bounds__(64) void k_knn_retry(const KnnGrid* __restrict__ gp, double r2max,
                                                   const double* __restrict__ nodes,
                                                   const double* __restrict__ sxyz,
                                                   const int* __restrict__ sidx,
                                                   const int* __restrict__ start,
                                                   const int* __restrict__ retry,
                                                   const double* __restrict__ retry_b,
                                                   int32_t* __restrict__ nbr) {
    const KnnGrid g = *gp;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
    const int nq = min(g.nretry, start[g.ncell]);  // (the list holds at most one entry per node)
    for (int i = wave; i < nq; i += nwaves) {  // wave-uniform
#ifdef EPP_KNN_DIAG
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
        knn_retry_wave<K>(g, r2max, nodes, sxyz, sidx, start, retry[i], retry_b[i], nbr);
#ifdef EPP_KNN_DIAG
        // (diagnostics builds) per retried query: start, end (10 ns ticks), bound, node
        if ((threadIdx.x & 63) == 0 && i < kKnnRetryTl) {
            g_knn_retry_tl[i][0] = t0;
            g_knn_retry_tl[i][1] = __builtin_amdgcn_s_memrealtime();
            g_knn_retry_tl[i][2] = (unsigned long long)__double_as_longlong(retry_b[i]);
            g_knn_retry_tl[i][3] = (unsigned long long)retry[i];
        }
#endif
    }
}

// ---- wave-per-query grid k-NN (k_knn_wave) ---------------------------------------------
// The same 4^3-cell blocks, 2-cell halos and block queue as k_knn_tile, but the halo's
// exact coordinates sit in LDS (SoA doubles) and one wavefront takes one query at a time:
//   1. the query's 5^3-cell cube is five z-slabs; each slab's five y-rows are one
//      contiguous LDS range (rows ly-2..ly+2 of the halo, x cells outside lx-2..lx+2
//      filtered by the halo x index kept with the node id).  The ranges are concatenated
//      and spread over the lanes, up to kWaveSlots candidates per lane, every lane doing
//      the same work (no per-query loop lengths, no divergence);
//   2. exact squared distance per candidate (the oracle's (dx dx + dy dy) + dz dz), and a
//      key: one of 128 linear bins of d over [0, 8 h^2) (monotone in d: every candidate at or below
//      the K-th distance has a key at or below the K-th one's);
//   3. the smallest cut with >= K keys at or below it, by bisection over the bins on
//      wave ballots (no histogram, no atomics);
//   4. the candidates at or below the cut (K plus a fraction of a bin, on average) go to a
//      per-wave LDS list; each listed entry's rank in (distance, index) order is counted
//      against the list: ranks < K are the answer, the rank K-1 entry the K-th distance for
//      the stopping rule after shell kTileH (knn_done).
// A query whose cube holds more than 64 kWaveSlots positions or whose list exceeds
// kWaveList, or that fails the stopping rule, goes to the retry list (k_knn_retry), as in
// k_knn_tile.  k_knn_tile's lanes-per-query scheme runs ~375 wave-instructions per query
// and waits on long dependent LDS chains of its busiest lane (SQ_WAIT_ANY ~66 % of its
// wave cycles); here a query is ~10 short LDS round trips and a fixed instruction count.
constexpr int kWaveThreads = 512;                // = kTileCells: one halo cell per thread
constexpr int kWaveCap = 1344;                   // halo candidates (else the block's queries retry)
constexpr int kWaveSlots = 6;                    // candidate slots per lane: 384 cube positions (~278 at 1.5 nodes per cell)
constexpr int kWaveList = 64;                    // listed candidates per query (else retry)
constexpr int kWaveBins = 128;                   // distance keys: linear bins over [0, 8 h^2)
static_assert(kTileCells == kWaveThreads, "one halo cell per thread");

template <int K>
__global__ __launch_bounds__(kWaveThreads, 6) void k_knn_wave(KnnGrid* __restrict__ gp, double r2max,
                                                              const double* __restrict__ sxyz,
                                                              const int* __restrict__ sidx,
                                                              const int* __restrict__ start,
                                                              int* __restrict__ retry, double* __restrict__ retry_b,
                                                              int32_t* __restrict__ nbr,
                                                              unsigned long long* __restrict__ dbg) {
    static_assert(K <= kWaveList && K <= 64, "");
    constexpr int kWaves = kWaveThreads / 64;
    __shared__ double hxv[kWaveCap], hyv[kWaveCap], hzv[kWaveCap];  // exact coordinates
    __shared__ int hid[kWaveCap];                                   // node id | halo x index << 29
    __shared__ uint32_t qh[kWaveCap];  // the block's queries: LDS position | halo x, y, z << 11, 14, 17
    __shared__ int cst[kTileCells + 1];                              // halo cell -> LDS offset
    __shared__ double ld[kWaves][kWaveList];                         // per-wave list: distances
    __shared__ int lj[kWaves][kWaveList];                            //                node ids
    __shared__ int wsum[kWaves];
    __shared__ int s_nq, s_b;
    __shared__ KnnGrid s_g;
    if (threadIdx.x == 0) s_g = *gp;  // (visible after the loop's first barrier)
    // (the grid parameters are read where they are used -- from gp or the LDS copy -- not
    // held in registers through the query loop: the scalar register file is this kernel's
    // tight resource)
    const int dims0 = gp->dims[0], dims1 = gp->dims[1], dims2 = gp->dims[2];
    const int nbx = (dims0 + kTileB - 1) / kTileB, nby = (dims1 + kTileB - 1) / kTileB,
              nbz = (dims2 + kTileB - 1) / kTileB;
    const int nblocks = nbx * nby * nbz;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const double inv_w = (double)kWaveBins / (8.0 * gp->h * gp->h);  // bins per unit of squared distance
    const int t = threadIdx.x;
    const int hx = t % kTileE, hy = (t / kTileE) % kTileE, hz = t / (kTileE * kTileE);  // this thread's halo cell
    for (;;) {
        if (t == 0) s_b = atomicAdd(&gp->next, 1);
        __syncthreads();
        const int b = s_b;  // block-uniform
        if (b >= nblocks) break;
        const int bx = b % nbx, by = (b / nbx) % nby, bz = b / (nbx * nby);
        const int ox = bx * kTileB - kTileH, oy = by * kTileB - kTileH, oz = bz * kTileB - kTileH;
#ifdef EPP_KNN_DIAG
        // phase timeline (diagnostics builds; scripts/knn_timeline.py): begin, halo scanned,
        // halo copied, wave 0's first query done, wave 0's queries done, (same), all waves
        // done, end; wave 0's query count and s_memtime cycles in its query loop
        unsigned long long tl[8] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0, 0, 0};
        unsigned long long cyc0 = 0, nq0 = 0;
#endif
        // 1. halo cell sizes -> exclusive scan
        const int x = ox + hx, y = oy + hy, z = oz + hz;
        const bool in = x >= 0 && x < dims0 && y >= 0 && y < dims1 && z >= 0 && z < dims2;
        const int cell = in ? (z * dims1 + y) * dims0 + x : 0;
        const int s0 = start[cell];
        const int cnt = in ? start[cell + 1] - s0 : 0;
        int incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        if (t == 0) s_nq = 0;
        __syncthreads();
        int base = incl - cnt, total = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            base += w < wv ? wsum[w] : 0;
            total += wsum[w];
        }
        cst[t] = base;
        if (t == 0) cst[kTileCells] = total;
#ifdef EPP_KNN_DIAG
        tl[1] = __builtin_amdgcn_s_memrealtime();
#endif
        if (total <= kWaveCap) {  // block-uniform
            // 2. copy the halo's nodes; list the block's own as queries
            const bool inner = hx >= kTileH && hx < kTileH + kTileB && hy >= kTileH && hy < kTileH + kTileB &&
                               hz >= kTileH && hz < kTileH + kTileB;
            const int q0 = (inner && cnt) ? atomicAdd(&s_nq, cnt) : 0;
            for (int q = 0; q < cnt; ++q) {
                const int sg = s0 + q, pos = base + q;
                hxv[pos] = sxyz[3 * (int64_t)sg];
                hyv[pos] = sxyz[3 * (int64_t)sg + 1];
                hzv[pos] = sxyz[3 * (int64_t)sg + 2];
                hid[pos] = sidx[sg] | (hx << 29);
                if (inner) qh[q0 + q] = (uint32_t)pos | ((uint32_t)hx << 11) | ((uint32_t)hy << 14) | ((uint32_t)hz << 17);
            }
            __syncthreads();
            const int nq = s_nq;
#ifdef EPP_KNN_DIAG
            tl[2] = __builtin_amdgcn_s_memrealtime();
            cyc0 = __builtin_amdgcn_s_memtime();
#endif
            // 3. one query per wave at a time
            for (int qi = wv; qi < nq; qi += kWaves) {  // wave-uniform
                // (the query's values are wave-uniform: moved to scalar registers, which
                // keeps the vector file for the candidate slots)
                const uint32_t qv = (uint32_t)__builtin_amdgcn_readfirstlane((int)qh[qi]);
                const int me = (int)(qv & 2047u);
                const int lx = (int)((qv >> 11) & 7u), ly = (int)((qv >> 14) & 7u), lz = (int)((qv >> 17) & 7u);
                auto uni = [](double v) {
                    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
                };
                const double px = uni(hxv[me]), py = uni(hyv[me]), pz = uni(hzv[me]);
                const int self = __builtin_amdgcn_readfirstlane(hid[me]) & 0x1fffffff;
                double bnd;  // the stopping rule's bound after shell kTileH (knn_bound)
                {
                    const KnnGrid g = s_g;  // (LDS: a global load here would wait out an L2 round trip per query)
                    const int c[3] = {ox + lx, oy + ly, oz + lz};
                    const double p[3] = {px, py, pz};
                    bnd = knn_bound(g, c, p, kTileH);
                }
                // the five slab ranges [A_d, B_d): lanes 0-4 read A, lanes 5-9 read B
                int rv = 0;
                if (lane < 10) {
                    const int d = lane < 5 ? lane : lane - 5;
                    const int row = (lz - kTileH + d) * kTileE + (lane < 5 ? ly - kTileH : ly + kTileH);
                    rv = cst[row * kTileE + (lane < 5 ? lx - kTileH : lx + kTileH + 1)];
                }
                int A[5], P[6];
                P[0] = 0;
#pragma unroll
                for (int d = 0; d < 5; ++d) {
                    A[d] = __builtin_amdgcn_readlane(rv, d);
                    P[d + 1] = P[d] + (__builtin_amdgcn_readlane(rv, 5 + d) - A[d]);
                }
                const int T = P[5];  // positions in the five ranges
                int gap[5];          // v -> LDS position: v + A_0 + the gaps between ranges behind v
#pragma unroll
                for (int d = 1; d < 5; ++d) gap[d] = A[d] - (A[d - 1] + (P[d] - P[d - 1]));
                bool done = false;
                double dk = r2max;  // the K-th distance (r2max: fewer than K candidates)
                if (T <= kWaveSlots * 64) {  // wave-uniform
                    // per slot: the exact distance and (key << 11 | LDS position); key
                    // kWaveBins: no candidate
                    double dv[kWaveSlots];
                    uint32_t kp[kWaveSlots];
#pragma unroll
                    for (int s = 0; s < kWaveSlots; ++s) {
                        kp[s] = (uint32_t)kWaveBins << 11;
                        dv[s] = 0.0;
                        if (s * 64 < T) {  // wave-uniform
                            const int v = s * 64 + lane;
                            int pos = A[0] + v;
#pragma unroll
                            for (int d = 1; d < 5; ++d) pos += v >= P[d] ? gap[d] : 0;
                            const bool ok = v < T;
                            const int pc = ok ? pos : me;
                            const double dx = hxv[pc] - px, dy = hyv[pc] - py, dz = hzv[pc] - pz;
                            const double dd = (dx * dx + dy * dy) + dz * dz;
                            const uint32_t cx = ((uint32_t)hid[pc] >> 29) - (uint32_t)(lx - kTileH);  // x cell in the cube?
                            const bool el = ok & (pc != me) & (cx <= 4u) & (dd <= r2max);
                            const double kd = dd * inv_w;
                            const uint32_t key = el ? (kd < (double)(kWaveBins - 1) ? (uint32_t)kd : kWaveBins - 1u) : kWaveBins;
                            kp[s] = (key << 11) | (uint32_t)pc;
                            dv[s] = dd;
                        }
                    }
                    auto count_le = [&](int c) {  // candidates with key <= c
                        const uint32_t lim = (uint32_t)(c + 1) << 11;
                        int n = 0;
#pragma unroll
                        for (int s = 0; s < kWaveSlots; ++s) n += (int)__popcll(__ballot(kp[s] < lim));  // (unused slots: never)
                        return n;
                    };
                    // the smallest cut with >= K keys at or below it (all candidates when
                    // fewer than K)
                    int lo = 0, hi = kWaveBins - 1;
                    if (count_le(hi) >= K) {
                        while (lo < hi) {  // wave-uniform
                            const int mid = (lo + hi) >> 1;
                            if (count_le(mid) >= K) hi = mid;
                            else lo = mid + 1;
                        }
                    }
                    const uint32_t lim = (uint32_t)(hi + 1) << 11;
                    int m = 0;
#pragma unroll
                    for (int s = 0; s < kWaveSlots; ++s) {
                        const bool li = kp[s] < lim;
                        const unsigned long long bl = __ballot(li);
                        const int at = m + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
                        if (li && at < kWaveList) {
                            ld[wv][at] = dv[s];
                            lj[wv][at] = hid[kp[s] & 2047u] & 0x1fffffff;
                        }
                        m += (int)__popcll(bl);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the list is written
                    if (m <= kWaveList) {  // wave-uniform
                        const bool mine = lane < m;
                        const double di = mine ? ld[wv][lane] : 0.0;
                        const int ji = mine ? lj[wv][lane] : 0;
                        // entry f (on lane f) against every lane's own: v_readlane into scalar
                        // registers, no memory round trip per entry
                        const int dlo = __double2loint(di), dhi = __double2hiint(di);
                        int rank = 0;
                        for (int f = 0; f < m; ++f) {  // wave-uniform
                            const double df = __hiloint2double(__builtin_amdgcn_readlane(dhi, f),
                                                               __builtin_amdgcn_readlane(dlo, f));
                            const int jf = __builtin_amdgcn_readlane(ji, f);
                            rank += ((df < di) | ((df == di) & (jf < ji))) ? 1 : 0;
                        }
                        if (m >= K) {
                            const unsigned long long bk = __ballot(mine && rank == K - 1);
                            dk = __shfl(di, bk ? (int)__builtin_ctzll(bk) : 0, 64);  // (one lane: ranks are distinct)
                        }
                        done = bnd == INFINITY || dk < bnd;
                        if (done) {
                            if (mine && rank < K) nbr[(int64_t)self * K + rank] = ji;
                            if (lane >= m && lane < K) nbr[(int64_t)self * K + lane] = -1;  // (fewer than K)
                        } else if (lane == 0) {
                            atomicAdd(&gp->why[2], 1);
                        }
                    } else {
                        dk = INFINITY;  // (list over capacity: the retry walks shells)
                        if (lane == 0) atomicAdd(&gp->why[0], 1);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the list is rewritten next
                } else {
                    dk = INFINITY;
                    if (lane == 0) atomicAdd(&gp->why[0], 1);
                }
                if (!done && lane == 0) {
                    const int at = atomicAdd(&gp->nretry, 1);
                    retry[at] = self;
                    retry_b[at] = dk;
                }
#ifdef EPP_KNN_DIAG
                if (tl[3] == 0ull) tl[3] = __builtin_amdgcn_s_memrealtime();
                ++nq0;
#endif
            }
#ifdef EPP_KNN_DIAG
            tl[4] = tl[5] = __builtin_amdgcn_s_memrealtime();
            cyc0 = __builtin_amdgcn_s_memtime() - cyc0;
#endif
        } else {
            // crowded halo: the block's own nodes retry from global memory
            const bool inner = hx >= kTileH && hx < kTileH + kTileB && hy >= kTileH && hy < kTileH + kTileB &&
                               hz >= kTileH && hz < kTileH + kTileB;
            if (inner && cnt) {
                const int at = atomicAdd(&gp->nretry, cnt);
                for (int q = 0; q < cnt; ++q) {
                    retry[at + q] = sidx[s0 + q];
                    retry_b[at + q] = INFINITY;
                }
                atomicAdd(&gp->why[3], cnt);
            }
        }
        __syncthreads();  // the LDS tile is rewritten by the next block
#ifdef EPP_KNN_DIAG
        if (dbg && threadIdx.x == 0 && b < kKnnTlBlocks) {
            tl[6] = tl[7] = __builtin_amdgcn_s_memrealtime();
            for (int q = 0; q < 8; ++q) dbg[16 * b + q] = tl[q];
            dbg[16 * b + 8] = (unsigned long long)s_nq;
            dbg[16 * b + 9] = (unsigned long long)total;
            dbg[16 * b + 10] = blockIdx.x;
            dbg[16 * b + 11] = nq0;
            dbg[16 * b + 12] = cyc0;
        }
#endif
    }
}

__global__ void k_knn_edges(const double* __restrict__ nodes, const int32_t* __restrict__ nbr, int64_t m,
                            int k, double* __restrict__ s1, double* __restrict__ s2) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const int64_t i = e / k;
    const int32_t j = nbr[e];
    const int64_t jj = j < 0 ? i : j;  // missing neighbour: a degenerate edge
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        s1[3 * e + d] = nodes[3 * i + d];
        s2[3 * e + d] = nodes[3 * jj + d];
    }
}

// Scratch of the grid k-NN, every part 256-byte aligned: grid params | bounds partials | cell_of[n] |
// sidx[n] | sxyz[3n] | cnt[cap+1] | fill[cap+1] | scan status words | start[cap+1] | retry
// bounds[n]  (cap = max(64, n)).  cnt, fill and the status words are one range, cleared by
// the launch's first kernel: the workspace may hold anything when a launch starts (a caller
// workspace carved from a buffer that held other data, a tag of an earlier launch).
struct KnnLayout {
    size_t part, cell, sidx, sxyz, cnt, start, fill, rbnd, stat, bytes;
    int cap, scan_blocks;
};
KnnLayout knn_layout(int n) {
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    KnnLayout L;
    L.cap = max(64, n);
    L.part = 256;                                   // kBoundsBlocks x 6 doubles (3 KB)
    L.cell = L.part + al((size_t)kBoundsBlocks * 48);
    L.sidx = L.cell + al((size_t)n * 4);
    L.sxyz = L.sidx + al((size_t)n * 4);
    L.cnt = L.sxyz + al((size_t)n * 24);
    L.fill = L.cnt + al((size_t)(L.cap + 1) * 4);
    L.stat = L.fill + al((size_t)(L.cap + 1) * 4);
    L.scan_blocks = (L.cap + 1 + kScanTile) / kScanTile;  // cells <= cap; start[ncell] too
    L.start = L.stat + al((size_t)L.scan_blocks * 8);
    L.rbnd = L.start + al((size_t)(L.cap + 1) * 4);
    L.bytes = L.rbnd + al((size_t)std::max(n, 1) * 8);
    return L;
}

epp_status last(const char* what);

#ifdef EPP_KNN_DIAG
// the k_knn_tile phase timeline (diagnostics builds): 16 u64 per block, see the kernel
unsigned long long* knn_tl_buffer() {
    static unsigned long long* buf = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        if (hipMalloc(&buf, (size_t)16 * 8 * kKnnTlBlocks) != hipSuccess) buf = nullptr;
    });
    return buf;
}
#endif

epp_status knn_grid_launch(const double* nodes, int n, int k, double max_dist, int32_t* nbr, char* buf,
                           const KnnLayout& L, hipStream_t s, const double* box_lo = nullptr,
                           const double* box_hi = nullptr, const double* ellipse = nullptr) {
    KnnGrid* g = reinterpret_cast<KnnGrid*>(buf);
    int* cell_of = reinterpret_cast<int*>(buf + L.cell);
    int* sidx = reinterpret_cast<int*>(buf + L.sidx);
    double* sxyz = reinterpret_cast<double*>(buf + L.sxyz);
    int* cnt = reinterpret_cast<int*>(buf + L.cnt);
    int* start = reinterpret_cast<int*>(buf + L.start);
    int* fill = reinterpret_cast<int*>(buf + L.fill);
    const double r2 = max_dist > 0 ? max_dist * max_dist : 1e300;
    const dim3 g256((n + 255) / 256), b256(256);
    const int nb = std::max(1, std::min(kBoundsBlocks, (n + kBoundsThreads - 1) / kBoundsThreads));
#ifdef EPP_KNN_DIAG
    // (diagnostics builds only) EPP_KNN_NPC: the grid density, an exact-either-way A/B knob
    const char* npc_env = std::getenv("EPP_KNN_NPC");
    const double npc = npc_env && *npc_env ? std::max(0.5, std::atof(npc_env)) : kNodesPerCell;
#else
    const double npc = kNodesPerCell;
#endif
    // cnt, fill and the scan's status words are adjacent: cleared together by the first
    // kernel (never run the scatter on stale counters, never let the look-back take a stale
    // word for a published one)
    const int nclr = (int)((L.start - L.cnt) / sizeof(int));
    if (box_lo && box_hi) {  // the caller's box: the grid shape on the host, one kernel
        KnnGrid gv{};
        const double mn[3] = {box_lo[0], box_lo[1], box_lo[2]}, mx[3] = {box_hi[0], box_hi[1], box_hi[2]};
        knn_grid_shape(mn, mx, n, L.cap, npc, &gv);
        if (ellipse) {  // (the row-restricted k-NN: k_knn_list_ellipse + k_knn_retry)
            for (int d = 0; d < 3; ++d) {
                gv.qs[d] = ellipse[d];
                gv.qg[d] = ellipse[3 + d];
            }
            gv.qbound = ellipse[6];
        }
        hipLaunchKernelGGL(k_knn_prep, dim3(nb), dim3(kBoundsThreads), 0, s, gv, g, cnt, nclr);
    } else {
        double* part = reinterpret_cast<double*>(buf + L.part);
        hipLaunchKernelGGL(k_knn_bounds_part, dim3(nb), dim3(kBoundsThreads), 0, s, nodes, n, part, cnt, nclr);
        hipLaunchKernelGGL(k_knn_setup, dim3(1), dim3(64), 0, s, part, nb, n, L.cap, npc, g);
    }
    hipLaunchKernelGGL(k_knn_count, g256, b256, 0, s, nodes, n, g, cell_of, cnt);
    hipLaunchKernelGGL(k_knn_scan, dim3(L.scan_blocks), dim3(kScanThreads), 0, s, g, cnt, start,
                       reinterpret_cast<unsigned long long*>(buf + L.stat), next_scan_tag());
    hipLaunchKernelGGL(k_knn_scatter, g256, b256, 0, s, nodes, n, cell_of, start, fill, sxyz, sidx);
    // EPP_KNN_TILE=0 selects the untiled grid walk, 2 the wave-per-query k_knn_wave (same
    // answers; test hooks); the default is k_knn_tile.  The timing ablations and the
    // per-block dump exist only in a -DEPP_KNN_DIAG diagnostics build.  (A one-query-per-
    // lane variant that keeps the exact
    // top-K in registers straight out of an LDS copy of the halo was tried: 425 us per
    // 63k-node table against k_knn_tile's 134 us -- the sorted insert then runs for nearly
    // every candidate of every lane.)
    // one wave per retried query: EPP_KNN_RETRY_PER_CU per CU (waves without a query
    // exit at once; more retries than waves loop)
#ifndef EPP_KNN_RETRY_PER_CU
#define EPP_KNN_RETRY_PER_CU 8
#endif
    const char* tile_env = std::getenv("EPP_KNN_TILE");
    const int tile_sel = tile_env && *tile_env ? std::atoi(tile_env) : kKnnDefaultTile;
    const bool tiled = tile_sel != 0;
    int* const retry = cell_of;  // free once the scatter has run
    double* const retry_b = reinterpret_cast<double*>(buf + L.rbnd);
    if (ellipse && (k == 4 || k == 8 || k == 16)) {  // the planner's row-restricted k-NN
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipLaunchKernelGGL(k_knn_list_ellipse, g256, b256, 0, s, g, nodes, n, retry, retry_b);
        const dim3 gr((unsigned)std::max(1, cus * EPP_KNN_RETRY_PER_CU)), br(64);
        if (k == 4) hipLaunchKernelGGL(k_knn_retry<4>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else if (k == 8) hipLaunchKernelGGL(k_knn_retry<8>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else hipLaunchKernelGGL(k_knn_retry<16>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        return last("epp_knn_grid");
    }
    // (node ids share a word with the halo x index in k_knn_wave: below 2^29)
    if (tile_sel == 2 && (k == 4 || k == 8 || k == 16) && n < (1 << 29)) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const dim3 gw((unsigned)std::max(1, cus * 3)), bw(kWaveThreads);  // (LDS: three workgroups per CU)
#ifdef EPP_KNN_DIAG
        unsigned long long* d = knn_tl_buffer();
        if (d) (void)hipMemsetAsync(d, 0, (size_t)16 * 8 * kKnnTlBlocks, s);
#else
        unsigned long long* d = nullptr;
#endif
        if (k == 4) hipLaunchKernelGGL(k_knn_wave<4>, gw, bw, 0, s, g, r2, sxyz, sidx, start, retry, retry_b, nbr, d);
        else if (k == 8) hipLaunchKernelGGL(k_knn_wave<8>, gw, bw, 0, s, g, r2, sxyz, sidx, start, retry, retry_b, nbr, d);
        else hipLaunchKernelGGL(k_knn_wave<16>, gw, bw, 0, s, g, r2, sxyz, sidx, start, retry, retry_b, nbr, d);
        const dim3 gr((unsigned)std::max(1, cus * EPP_KNN_RETRY_PER_CU)), br(64);
        if (k == 4) hipLaunchKernelGGL(k_knn_retry<4>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else if (k == 8) hipLaunchKernelGGL(k_knn_retry<8>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else hipLaunchKernelGGL(k_knn_retry<16>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
    } else if (tiled && (k == 4 || k == 8 || k == 16)) {
        // persistent: the block count is only known on the device (grid shape)
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const dim3 gt((unsigned)std::max(1, cus * 3)), bt(kTileThreads);  // (LDS: three workgroups per CU)
#ifdef EPP_KNN_DIAG
        const int mode = tile_env ? std::atoi(tile_env) : 1;  // 4: timing ablation (inexact)
        unsigned long long* d = knn_tl_buffer();
        if (d) (void)hipMemsetAsync(d, 0, (size_t)16 * 8 * kKnnTlBlocks, s);
#else
        const int mode = 1;
        unsigned long long* d = nullptr;
#endif
        if (k == 4) hipLaunchKernelGGL(k_knn_tile<4>, gt, bt, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr, mode, d);
        else if (k == 8) hipLaunchKernelGGL(k_knn_tile<8>, gt, bt, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr, mode, d);
        else hipLaunchKernelGGL(k_knn_tile<16>, gt, bt, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr, mode, d);
        const dim3 gr((unsigned)std::max(1, cus * EPP_KNN_RETRY_PER_CU)), br(64);
        if (k == 4) hipLaunchKernelGGL(k_knn_retry<4>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else if (k == 8) hipLaunchKernelGGL(k_knn_retry<8>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
        else hipLaunchKernelGGL(k_knn_retry<16>, gr, br, 0, s, g, r2, nodes, sxyz, sidx, start, retry, retry_b, nbr);
    } else {
        switch (k) {
            case 4: hipLaunchKernelGGL(k_knn_grid<4>, g256, b256, 0, s, g, n, r2, sxyz, sidx, start, nbr); break;
            case 8: hipLaunchKernelGGL(k_knn_grid<8>, g256, b256, 0, s, g, n, r2, sxyz, sidx, start, nbr); break;
            case 16: hipLaunchKernelGGL(k_knn_grid<16>, g256, b256, 0, s, g, n, r2, sxyz, sidx, start, nbr); break;
            default: hipLaunchKernelGGL(k_knn_grid<32>, g256, b256, 0, s, g, n, r2, sxyz, sidx, start, nbr); break;
        }
    }
    return last("epp_knn_grid");
}

CachedWs g_knn_ws[64];
CachedWs g_compact_ws[64];

// ---- ordered compaction of the valid states ----------------------------------------
// One pass: block b owns states [b C, (b+1) C) (C = kCompactChunk) in kCompactRounds rounds
// of one state per thread (coalesced flag loads and row copies); ranks from wave ballots
// and the per-(round, wave) counts in LDS, the block's offset by look-back.  The valid
// states are written in index order.  Deterministic: the planner's node order (and with
// it k-NN tie breaks and the search) does not depend on scheduling.
constexpr int kCompactThreads = 256;
constexpr int kCompactRounds = 4;
constexpr int kCompactChunk = kCompactThreads * kCompactRounds;

// (block b of nb; the last block writes *n_out = the valid count + add)
__device__ __forceinline__ void compact_block(const double* __restrict__ xyz, const uint8_t* __restrict__ valid,
                                              int64_t n, unsigned long long* __restrict__ st, uint32_t tag,
                                              double* __restrict__ out, int64_t* __restrict__ n_out, int64_t add,
                                              const int b, const int nb) {
    constexpr int NW = kCompactThreads / 64;
    __shared__ int wcnt[kCompactRounds * NW];
    __shared__ long long s_excl;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t i0 = (int64_t)b * kCompactChunk + threadIdx.x;
    bool v[kCompactRounds];
    unsigned long long bal[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        const int64_t i = i0 + r * kCompactThreads;
        v[r] = i < n && valid[i] != 0;
    }
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        bal[r] = __ballot(v[r]);
        if (lane == 0) wcnt[r * NW + wv] = __popcll(bal[r]);
    }
    __syncthreads();
    // (round, wave) slots in index order: round-major
    int before[kCompactRounds], total = 0;
#pragma unroll
    for (int q = 0; q < kCompactRounds * NW; ++q) {
#pragma unroll
        for (int r = 0; r < kCompactRounds; ++r)
            if (q == r * NW + wv) before[r] = total;
        total += wcnt[q];
    }
    if (wv == 0) {
        if (lane == 0) lb_publish(st, b, tag, b == 0, total);
        const long long ex = b == 0 ? 0ll : lb_exclusive(st, b, tag);
        if (lane == 0) {
            if (b > 0) lb_publish(st, b, tag, true, ex + total);
            s_excl = ex;
            if (b == nb - 1) *n_out = ex + total + add;
        }
    }
    __syncthreads();
    const long long ex = s_excl;
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        if (v[r]) {
            const int64_t i = i0 + r * kCompactThreads;
            const int64_t p = ex + before[r] +
                              (int64_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
            out[3 * p] = xyz[3 * i];
            out[3 * p + 1] = xyz[3 * i + 1];
            out[3 * p + 2] = xyz[3 * i + 2];
        }
    }
}
__global__ __launch_bounds__(kCompactThreads) void k_compact(const double* __restrict__ xyz,
                                                             const uint8_t* __restrict__ valid, int64_t n,
                                                             unsigned long long* __restrict__ st, uint32_t tag,
                                                             double* __restrict__ out, int64_t* __restrict__ n_out) {
    compact_block(xyz, valid, n, st, tag, out, n_out, 0, blockIdx.x, gridDim.x);
}

__global__ void k_mask_edges(int32_t* __restrict__ nbr, const uint8_t* __restrict__ valid, int64_t m) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < m && !valid[e]) nbr[e] = -1;
}

// The same, plus count[0] += the surviving edges (entries >= 0 after masking) and
// count[1] += the surviving edges into node `target`.  Grid-stride over at most one
// 1024-thread block per CU, wave popcounts, one atomic per block and counter (an atomic
// per 256 edges put thousands on one address: ~45 us for 1M edges).
constexpr int kMaskThreads = 1024;
__global__ __launch_bounds__(kMaskThreads) void k_mask_edges_count(int32_t* __restrict__ nbr,
                                                                   const uint8_t* __restrict__ valid, int64_t m,
                                                                   int32_t target,
                                                                   unsigned long long* __restrict__ count,
                                                                   uint16_t* __restrict__ out16) {
    __shared__ uint32_t part[2][kMaskThreads / 64];
    uint32_t c = 0, ci = 0;
    for (int64_t e = (int64_t)blockIdx.x * kMaskThreads + threadIdx.x; e < m;
         e += (int64_t)gridDim.x * kMaskThreads) {  // (uniform trip count per wave but the last)
        const int32_t v = nbr[e];
        const bool ok = valid[e] != 0;
        if (!ok) nbr[e] = -1;
        const bool keep = ok && v >= 0;
        if (out16) out16[e] = keep ? (uint16_t)v : (uint16_t)0xFFFF;  // (a narrow copy for the download)
        c += keep ? 1u : 0u;
        ci += (keep && v == target) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) {
        c += (uint32_t)__shfl_xor((int)c, o, 64);
        ci += (uint32_t)__shfl_xor((int)ci, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = c;
        part[1][threadIdx.x >> 6] = ci;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t t = 0;
        for (int w = 0; w < kMaskThreads / 64; ++w) t += part[threadIdx.x][w];
        if (t) atomicAdd(count + threadIdx.x, (unsigned long long)t);
    }
}

// The planner's row-restricted search: the rows of the k-NN table (int32) whose node lies
// in the ellipsoid |x - s| + |x - g| <= bound, packed in arbitrary slot order: ids32 /
// ids16[slot] = the node, rows32[slot * k ..] = its row.  The test is widened by 1e-9
// relative + 1e-9 m, so every node the host's A* can expand below the bound has its row
// here.  One atomic per wave; rows past `cap` are counted, not written (the host then
// takes the whole table).
__global__ __launch_bounds__(256) void k_pack_ellipse_rows(const double* __restrict__ nodes,
                                                           const int32_t* __restrict__ tab, int32_t n,
                                                           int32_t k, double sx, double sy, double sz,
                                                           double gx, double gy, double gz, double bound,
                                                           int32_t cap, int32_t* __restrict__ ids32,
                                                           uint16_t* __restrict__ ids16,
                                                           int32_t* __restrict__ rows32,
                                                           unsigned long long* __restrict__ count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < n) {
        const double x = nodes[3 * i], y = nodes[3 * i + 1], z = nodes[3 * i + 2];
        const double ds = sqrt((x - sx) * (x - sx) + (y - sy) * (y - sy) + (z - sz) * (z - sz));
        const double dg = sqrt((x - gx) * (x - gx) + (y - gy) * (y - gy) + (z - gz) * (z - gz));
        in = ds + dg <= bound * (1.0 + 1e-9) + 1e-9;
    }
    const unsigned long long bal = __ballot(in);
    if (!bal) return;  // (uniform per wave)
    const int lane = threadIdx.x & 63;
    const int first = __ffsll(bal) - 1;
    unsigned long long base = 0;
    if (lane == first) base = atomicAdd(count, (unsigned long long)__popcll(bal));
    base = __shfl(base, first, 64);
    if (!in) return;
    const unsigned long long slot = base + __popcll(bal & ((1ull << lane) - 1ull));
    if (slot >= (unsigned long long)cap) return;
    ids32[slot] = i;
    ids16[slot] = (uint16_t)i;
    const int32_t* src = tab + (size_t)i * k;
    int32_t* dst = rows32 + (size_t)slot * k;
    if ((k & 3) == 0) {
        for (int c = 0; c < k; c += 4) *reinterpret_cast<int4*>(dst + c) = *reinterpret_cast<const int4*>(src + c);
    } else {
        for (int c = 0; c < k; ++c) dst[c] = src[c];
    }
}

// ---- the batched planner: one launch per stage for all of a batch's problems ----------
// (epp_internal.h, PlanBatchLayout).  Problem p = blockIdx.y of the per-problem stages; its
// samples at xyz + p ns, its nodes at nodes + p NS (NS = 2^ns_log >= 65536: a node's id in
// its problem is the low bits of its global id p NS + node), its k-NN grid workspace at
// kws + p kws_stride (KnnLayout for ns + 2 nodes), its queries at query + row_off.  Node
// counts stay on the device.
constexpr int kPbSegSmall = 16;  // batches of up to this many problems: no upload (k_pb_sample)
struct PlanBatchDev {
    const PlanSeg* seg;
    const PlanSeg* seg_h;         // (<= kPbSegSmall problems) the pinned host copy, else null
    uint64_t seeds[kPbSegSmall];  // (<= kPbSegSmall problems) their seeds and capacities
    int32_t caps[kPbSegSmall];
    int S, k, ns_log, nbc, cap_total, nctr;
    int64_t ns, NS;
    double lo[3], hi[3];
    double* xyz;
    uint8_t* valid;
    double* nodes;
    unsigned long long* cstat;
    unsigned long long* nstat;  // k_pb_number's look-back status words: NS / 1024 per problem
    unsigned long long* ctr;
    char* kws;
    size_t kws_stride, l_cell, l_sidx, l_sxyz, l_cnt, l_start, l_fill, l_stat;
    int l_cap, nclr;
    int32_t* query;     // per problem (at row_off): its listed nodes (node ids)
    int32_t* ids32;     // row -> global node id
    int32_t* rows32;    // row -> its k neighbours (global ids)
    uint16_t* rows16;   // the same masked (node ids, then compact indices; 0xFFFF: none)
    uint8_t* mark;      // a byte per node: referenced by a row
    int32_t* map;       // node (global id) -> compact index (referenced nodes only)
    double* need;       // 3 doubles per referenced node (at need_off + compact index)
};

struct KnnSeg {
    KnnGrid* g;
    int* cell_of;
    int* sidx;
    double* sxyz;
    int* cnt;
    int* start;
    int* fill;
    unsigned long long* stat;
};
__device__ __forceinline__ KnnSeg knn_seg(const PlanBatchDev& P, int p) {
    char* b = P.kws + (size_t)p * P.kws_stride;
    return {reinterpret_cast<KnnGrid*>(b), reinterpret_cast<int*>(b + P.l_cell), reinterpret_cast<int*>(b + P.l_sidx),
            reinterpret_cast<double*>(b + P.l_sxyz), reinterpret_cast<int*>(b + P.l_cnt),
            reinterpret_cast<int*>(b + P.l_start), reinterpret_cast<int*>(b + P.l_fill),
            reinterpret_cast<unsigned long long*>(b + P.l_stat)};
}
__device__ __forceinline__ unsigned long long& pb_ctr(const PlanBatchDev& P, int field, int p) {
    return P.ctr[kPbPerSeg + field * P.S + p];
}
enum : int { kFQueries = 0, kFKept = 1, kFGoal = 2, kFNodes = 3, kFNeed = 4, kFInexact = 5 };

// samples (k_sample_uniform's arithmetic) + clears: the problem's compaction status words
// and node marks; problem 0 also the batch counters
// A batch of <= kPbSegSmall problems needs no upload of its own (a blit dispatch, ~5 us,
// before round 6): every workgroup takes its problem's seed and capacity from the launch
// arguments (P.seeds / P.caps), and workgroup (0, p) reads problem p from the pinned host
// copy and stores it into the device copy the later stages read.  Larger batches upload
// the problems first (P.seg_h null).
static_assert(sizeof(PlanSeg) % 8 == 0, "PlanSeg copied as 8-byte words");

__global__ __launch_bounds__(256) void k_pb_sample(PlanBatchDev P) {
    const int p = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool small = P.seg_h != nullptr;  // (uniform)
    if (small && blockIdx.x == 0 && threadIdx.x < (int)(sizeof(PlanSeg) / 8))
        reinterpret_cast<uint64_t*>(const_cast<PlanSeg*>(P.seg) + p)[threadIdx.x] =
            reinterpret_cast<const uint64_t*>(P.seg_h + p)[threadIdx.x];
    if (i < P.nbc) P.cstat[(int64_t)p * P.nbc + i] = 0ull;
    if (P.cap_total > 0 && i < P.NS / kCompactChunk) P.nstat[(int64_t)p * (P.NS / kCompactChunk) + i] = 0ull;
    // (the marks exist only when some problem has restricted rows: cap_total > 0)
    if (P.cap_total > 0 && i < (P.NS >> 4))
        reinterpret_cast<uint4*>(P.mark + ((int64_t)p << P.ns_log))[i] = make_uint4(0u, 0u, 0u, 0u);
    if (p == 0 && i < P.nctr) P.ctr[i] = 0ull;
    const uint64_t seed = small ? P.seeds[p] : P.seg[p].seed;
    const int32_t cap = small ? P.caps[p] : P.seg[p].cap;
    if (cap > 0) {  // the problem's k-NN grid: cleared cell counters and its shape
        const KnnSeg ks = knn_seg(P, p);
        if (i < P.nclr) ks.cnt[i] = 0;
        if (i == 0) {
            const PlanSeg q = small ? P.seg_h[p] : P.seg[p];
            KnnGrid gv{};
            int64_t cells = 1;
            double h = q.h;
            for (;;) {  // (cells bounded by the workspace's capacity; coarser if need be)
                cells = 1;
                for (int d = 0; d < 3; ++d) {
                    gv.dims[d] = (int)fmin((q.ghi[d] - q.glo[d]) / h, 1023.0) + 1;
                    cells *= gv.dims[d];
                }
                if (cells <= P.l_cap) break;
                h *= 1.25;
            }
            for (int d = 0; d < 3; ++d) gv.lo[d] = q.glo[d];
            gv.h = h;
            gv.inv_h = 1.0 / h;
            gv.ncell = (int)cells;
            gv.qbound = 1e300;
            *ks.g = gv;
        }
    }
    if (i >= P.ns) return;
    const uint64_t c = (uint64_t)i * 3ull;
    const double u0 = (double)(splitmix64(seed ^ c) >> 11) * 0x1.0p-53;
    const double u1 = (double)(splitmix64(seed ^ (c + 1)) >> 11) * 0x1.0p-53;
    const double u2 = (double)(splitmix64(seed ^ (c + 2)) >> 11) * 0x1.0p-53;
    double* x = P.xyz + ((int64_t)p * P.ns + i) * 3;
    x[0] = P.lo[0] + (P.hi[0] - P.lo[0]) * u0;
    x[1] = P.lo[1] + (P.hi[1] - P.lo[1]) * u1;
    x[2] = P.lo[2] + (P.hi[2] - P.lo[2]) * u2;
}

__device__ __forceinline__ double pb_ellipse(const PlanSeg& q, const double* x) {
    const double ds = sqrt((x[0] - q.s[0]) * (x[0] - q.s[0]) + (x[1] - q.s[1]) * (x[1] - q.s[1]) +
                           (x[2] - q.s[2]) * (x[2] - q.s[2]));
    const double dg = sqrt((x[0] - q.g[0]) * (x[0] - q.g[0]) + (x[1] - q.g[1]) * (x[1] - q.g[1]) +
                           (x[2] - q.g[2]) * (x[2] - q.g[2]));
    return ds + dg;
}

// Per node (problems with restricted rows): inside the grid ellipsoid -> its cell counted
// (cell_of, else -1); inside the row ellipsoid (widened by 1e-8 relative + 1e-6 m) ->
// listed as a query (ranks from one atomic per workgroup).
__device__ __forceinline__ bool pb_member(const PlanBatchDev& P, const PlanSeg& q, const KnnSeg& ks, const KnnGrid& g,
                                          int p, int node, const double* x) {
    const double f = pb_ellipse(q, x);
    int c = -1;
    if (f <= q.gbound) {
        const int cx = knn_cell_axis(x[0], g, 0), cy = knn_cell_axis(x[1], g, 1), cz = knn_cell_axis(x[2], g, 2);
        c = (cz * g.dims[1] + cy) * g.dims[0] + cx;
        atomicAdd(&ks.cnt[c], 1);
    }
    ks.cell_of[node] = c;
    return f <= q.bound * (1.0 + 1e-8) + 1e-6;
}

// nodes = start, goal, the valid samples in sample order (an ordered compaction, decoupled
// look-back as compact_block); the node count into the header; each node's membership
// (pb_member) as it is written, the queries listed.
__global__ __launch_bounds__(kCompactThreads) void k_pb_compact(PlanBatchDev P, uint32_t tag) {
    const int p = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
    double* out = P.nodes + (int64_t)p * P.NS * 3;
    const PlanSeg& q = P.seg[p];
    const bool R = q.cap > 0;  // (block-uniform)
    const KnnSeg ks = knn_seg(P, p);
    KnnGrid g{};
    if (R) g = *ks.g;
    const double* xyz = P.xyz + (int64_t)p * P.ns * 3;
    const uint8_t* valid = P.valid + (int64_t)p * P.ns;
    unsigned long long* st = P.cstat + (int64_t)p * P.nbc;
    constexpr int NW = kCompactThreads / 64;
    __shared__ int wcnt[kCompactRounds * NW];
    __shared__ int qcnt[NW];
    __shared__ long long s_excl;
    __shared__ unsigned long long s_qbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    bool inq2 = false;  // start (thread 0) / goal (thread 1) of block 0: listed as queries
    if (b == 0 && threadIdx.x < 2) {
        const double* e = threadIdx.x == 0 ? q.s : q.g;
        out[3 * threadIdx.x] = e[0];
        out[3 * threadIdx.x + 1] = e[1];
        out[3 * threadIdx.x + 2] = e[2];
        if (R) inq2 = pb_member(P, q, ks, g, p, (int)threadIdx.x, e);
    }
    const int64_t i0 = (int64_t)b * kCompactChunk + threadIdx.x;
    bool v[kCompactRounds];
    unsigned long long bal[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        const int64_t i = i0 + r * kCompactThreads;
        v[r] = i < P.ns && valid[i] != 0;
    }
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        bal[r] = __ballot(v[r]);
        if (lane == 0) wcnt[r * NW + wv] = __popcll(bal[r]);
    }
    __syncthreads();
    int before[kCompactRounds], total = 0;
#pragma unroll
    for (int qq = 0; qq < kCompactRounds * NW; ++qq) {
#pragma unroll
        for (int r = 0; r < kCompactRounds; ++r)
            if (qq == r * NW + wv) before[r] = total;
        total += wcnt[qq];
    }
    if (wv == 0) {
        if (lane == 0) lb_publish(st, b, tag, b == 0, total);
        const long long ex = b == 0 ? 0ll : lb_exclusive(st, b, tag);
        if (lane == 0) {
            if (b > 0) lb_publish(st, b, tag, true, ex + total);
            s_excl = ex;
            if (b == nb - 1) pb_ctr(P, kFNodes, p) = (unsigned long long)(ex + total + 2);
        }
    }
    __syncthreads();
    const long long ex = s_excl;
    bool inq[kCompactRounds];
    int node[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        inq[r] = false;
        node[r] = 0;
        if (v[r]) {
            const int64_t i = i0 + r * kCompactThreads;
            const int64_t at = 2 + ex + before[r] +
                               (int64_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
            const double x[3] = {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
            out[3 * at] = x[0];
            out[3 * at + 1] = x[1];
            out[3 * at + 2] = x[2];
            node[r] = (int)at;
            if (R) inq[r] = pb_member(P, q, ks, g, p, (int)at, x);
        }
    }
    if (!R) return;  // (block-uniform)
    // the block's queries: one atomic per workgroup on the problem's query count
    unsigned long long qb[kCompactRounds + 1];
    int wq = 0;
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        qb[r] = __ballot(inq[r]);
        wq += __popcll(qb[r]);
    }
    qb[kCompactRounds] = __ballot(inq2);
    wq += __popcll(qb[kCompactRounds]);
    if (lane == 0) qcnt[wv] = wq;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < NW; ++w) t += qcnt[w];
        s_qbase = t ? atomicAdd(&pb_ctr(P, kFQueries, p), (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    unsigned long long rnk = s_qbase;
    for (int w = 0; w < wv; ++w) rnk += qcnt[w];
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r <= kCompactRounds; ++r) {
        const bool mine = r < kCompactRounds ? inq[r] : inq2;
        const int nd = r < kCompactRounds ? node[r] : (int)threadIdx.x;
        if (mine) {
            const unsigned long long at = rnk + __popcll(qb[r] & below);
            if (at < (unsigned long long)q.cap) P.query[q.row_off + (int64_t)at] = nd;
        }
        rnk += __popcll(qb[r]);
    }
}

__global__ __launch_bounds__(kScanThreads) void k_pb_knn_scan(PlanBatchDev P, uint32_t tag) {
    if (P.seg[blockIdx.y].cap <= 0) return;
    const KnnSeg ks = knn_seg(P, blockIdx.y);
    knn_scan_block(ks.g, ks.cnt, ks.start, ks.stat, tag, blockIdx.x);
}

__global__ __launch_bounds__(256) void k_pb_knn_scatter(PlanBatchDev P) {
    const int p = blockIdx.y;
    if (P.seg[p].cap <= 0) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (int)pb_ctr(P, kFNodes, p)) return;
    const KnnSeg ks = knn_seg(P, p);
    const int c = ks.cell_of[i];
    if (c < 0) return;
    const int pos = ks.start[c] + atomicAdd(&ks.fill[c], 1);
    if (pos >= ks.start[c + 1]) return;  // cannot happen with cleared counters
    const double* nd = P.nodes + ((int64_t)p * P.NS + i) * 3;
    ks.sidx[pos] = i;
    ks.sxyz[3 * pos] = nd[0];
    ks.sxyz[3 * pos + 1] = nd[1];
    ks.sxyz[3 * pos + 2] = nd[2];
}

// The exact k-NN row of one listed query from its problem's grid (whole wave).  Every node
// within distance r of x has |y - s| + |y - g| <= f(x) + 2 r, so while f(x) + 2 r <= gbound
// (with a margin far above the rounding) every such node is in the grid: the candidates
// within r are all the nodes within r.  r = 1.6 h first (~26 nodes at the grid's density),
// then x 1.5 until at least K are listed; each listed entry's rank in (distance, index)
// order is counted against the list (the order k_knn / the oracle use).  The box's x-runs of
// cells (one contiguous range of the cell-sorted nodes each) are laid out over all the lanes
// by a wave scan of their lengths, kU candidates per lane in flight.  Returns false when
// the radius would leave the grid ellipsoid or the list overflows (the row is then not
// exact, and the caller flags the problem).
#ifdef EPP_PB_ROWS_TL
// (diagnostics builds only: -DEPP_PB_ROWS_TL, scripts/pb_rows_timeline.py) per listed query
// d < kPbTl, lane 0's s_memrealtime (100 MHz) stamps: [0] query start, [1] first radius's
// run starts loaded, [2] its candidates listed, [3] row written, [4] radius iterations |
// candidates << 8 | wave << 32, [5] the wave's start
constexpr int kPbTl = 1 << 15;
__device__ unsigned long long g_pb_rows_tl[kPbTl][6];
#define EPP_PBTL(d, k, v)                                                     \
    do {                                                                      \
        if ((threadIdx.x & 63) == 0 && (d) < kPbTl) g_pb_rows_tl[(d)][(k)] = (v); \
    } while (0)
#define EPP_PBTL_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define EPP_PBTL(d, k, v) \
    do {                  \
    } while (0)
#define EPP_PBTL_NOW() 0ull
#endif

template <int K>
__device__ __forceinline__ bool pb_query_row(const KnnGrid& g, const double* __restrict__ sxyz,
                                             const int* __restrict__ sidx, const int* __restrict__ start,
                                             const double (&p)[3], double f, double gbound, int self,
                                             int32_t* __restrict__ out, int64_t off, int tl_d = 0) {
    constexpr int kCap = 512;
#ifndef EPP_PB_KU  // (A/B builds may override)
#define EPP_PB_KU 2
#endif
    constexpr int kU = EPP_PB_KU;  // candidates per lane in flight
    __shared__ double s_d[kCap];
    __shared__ int s_j[kCap];
    const int lane = threadIdx.x & 63;
    double r = 1.6 * g.h;
    for (int it = 0; it < 4; ++it, r *= 1.5) {  // wave-uniform
        if (!(f + 2.0 * r * (1.0 + 1e-9) + 1e-9 <= gbound)) return false;
        const double b2 = r * r;
        const double rb = r * (1.0 + 1e-9) + 1e-12 * (1.0 + fabs(p[0]) + fabs(p[1]) + fabs(p[2]));
        int lo[3], hi[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            lo[d] = knn_cell_axis(p[d] - rb, g, d);
            hi[d] = knn_cell_axis(p[d] + rb, g, d);
        }
        const int ny = hi[1] - lo[1] + 1, rows = ny * (hi[2] - lo[2] + 1);
        // (a row's x-run narrowed to the sphere's chord: the row's y / z cell ranges --
        // padded, the edge cells unbounded -- are at least dy / dz from p, so a node
        // within rb of p has |x - p.x| <= sqrt(rb^2 - dy^2 - dz^2); cells are monotone in x)
        const double pad = 1e-9 * (g.h + fabs(p[0]) + fabs(p[1]) + fabs(p[2]));
        auto gap = [&](int c, int d) {
            const double a = c == 0 ? -INFINITY : g.lo[d] + (double)c * g.h - pad;
            const double b = c == g.dims[d] - 1 ? INFINITY : g.lo[d] + (double)(c + 1) * g.h + pad;
            return p[d] < a ? a - p[d] : (p[d] > b ? p[d] - b : 0.0);
        };
        int cnt = 0;  // (wave-uniform)
        for (int rb0 = 0; rb0 < rows; rb0 += 64) {
            const int row = rb0 + lane;
            int s0 = 0, len = 0;
            if (row < rows) {
                const int cz = lo[2] + row / ny, cy = lo[1] + row % ny;
                const double dy = gap(cy, 1), dz = gap(cz, 2);
                const double rem2 = rb * rb - (dy * dy + dz * dz);
                if (rem2 >= 0.0) {
                    const double hx = sqrt(rem2) + pad;
                    const int x0 = max(lo[0], knn_cell_axis(p[0] - hx, g, 0));
                    const int x1 = min(hi[0], knn_cell_axis(p[0] + hx, g, 0));
                    const int a = (cz * g.dims[1] + cy) * g.dims[0];
                    s0 = start[a + x0];
                    len = start[a + x1 + 1] - s0;
                }
            }
            if (it == 0 && rb0 == 0) {
                [[maybe_unused]] const int lv = __shfl(len, 0, 64);  // (waits for the loads)
                EPP_PBTL(tl_d, 1, EPP_PBTL_NOW() + (unsigned long long)(lv & 0));
            }
            int incl = len;  // inclusive scan of the run lengths over the lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            const int excl = incl - len, T = __shfl(incl, 63, 64);
            for (int t0 = 0; t0 < T; t0 += 64 * kU) {
                double dd[kU];
                int jj[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int t = t0 + u * 64 + lane;
                    // the run holding candidate t: the last lane whose exclusive start <= t
                    int a = 0;
#pragma unroll
                    for (int step = 32; step > 0; step >>= 1)
                        if (__shfl(excl, a + step, 64) <= t) a += step;
                    const int q = __shfl(s0, a, 64) + (t - __shfl(excl, a, 64));
                    const bool ok = t < T;
                    const int qq = ok ? q : 0;  // (past the list: any valid entry, skipped below)
                    jj[u] = ok ? sidx[qq] : self;
                    const double ddx = sxyz[3 * qq] - p[0], ddy = sxyz[3 * qq + 1] - p[1], ddz = sxyz[3 * qq + 2] - p[2];
                    dd[u] = (ddx * ddx + ddy * ddy) + ddz * ddz;
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const bool keep = jj[u] != self && dd[u] <= b2;
                    const unsigned long long kb = __ballot(keep);
                    const int at = cnt + __popcll(kb & ((1ull << lane) - 1ull));
                    if (keep && at < kCap) {
                        s_d[at] = dd[u];
                        s_j[at] = jj[u];
                    }
                    cnt += __popcll(kb);
                }
            }
        }
        if (it == 0) EPP_PBTL(tl_d, 2, EPP_PBTL_NOW());
        EPP_PBTL(tl_d, 4, (unsigned long long)(it + 1) | ((unsigned long long)cnt << 8));
        if (cnt > kCap) return false;
        if (cnt < K) continue;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's list is complete
        // entries [0, m) of the LDS list (m <= 64), entry i on lane i: each one's rank in
        // (distance, index) order counted against the others by v_readlane; ranks < K out
        auto rank_small = [&](int m) {
            const bool mine = lane < m;
            const double di = mine ? s_d[lane] : 0.0;
            const int ji = mine ? s_j[lane] : 0;
            const int dlo = __double2loint(di), dhi = __double2hiint(di);
            int rank = 0;
            for (int f2 = 0; f2 < m; ++f2) {
                const double df = __hiloint2double(__builtin_amdgcn_readlane(dhi, f2), __builtin_amdgcn_readlane(dlo, f2));
                rank += ((df < di) | ((df == di) & (__builtin_amdgcn_readlane(ji, f2) < ji))) ? 1 : 0;
            }
            if (mine && rank < K) out[rank] = (int32_t)(off + ji);
        };
        if (cnt <= 64) {
            rank_small(cnt);
        } else if (cnt <= 4 * 64) {
            // Longer lists (a second radius: 60-100 candidates): the K-th distance is
            // bracketed by bisection on wave ballots (the list in registers, four slots per
            // lane; 10 halvings of [0, r^2]), the entries at or below the bracket's top --
            // K plus the few that share its last interval -- are listed again and ranked
            // among themselves: an entry's preceding entries all lie in that list, so its
            // rank is its rank in the whole list.  (Instead of ranking every entry against
            // every other through LDS: 20 us for the slowest queries.)
            constexpr int kSl = 4;
            double dv[kSl];
            int jv[kSl];
#pragma unroll
            for (int sl = 0; sl < kSl; ++sl) {
                const int i = sl * 64 + lane;
                dv[sl] = i < cnt ? s_d[i] : INFINITY;
                jv[sl] = i < cnt ? s_j[i] : 0;
            }
            double lo = 0.0, hi = b2;  // count(d <= hi) >= K (every entry has d <= r^2)
            for (int step = 0; step < 10; ++step) {
                const double mid = 0.5 * (lo + hi);
                int c = 0;
#pragma unroll
                for (int sl = 0; sl < kSl; ++sl) c += __popcll(__ballot(dv[sl] <= mid));
                if (c >= K) hi = mid;
                else lo = mid;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the list is read: rewritten below)
            int m = 0;
#pragma unroll
            for (int sl = 0; sl < kSl; ++sl) {
                const bool in = dv[sl] <= hi;
                const unsigned long long b = __ballot(in);
                const int at = m + __popcll(b & ((1ull << lane) - 1ull));
                if (in && at < kCap) {
                    s_d[at] = dv[sl];
                    s_j[at] = jv[sl];
                }
                m += __popcll(b);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (m <= 64) {
                rank_small(m);
            } else {  // (many entries at one distance: rank every entry of the cut list)
                for (int i = lane; i < m; i += 64) {
                    const double di = s_d[i];
                    const int ji = s_j[i];
                    int rank = 0;
                    for (int f2 = 0; f2 < m; ++f2) {
                        const double df = s_d[f2];
                        rank += ((df < di) | ((df == di) & (s_j[f2] < ji))) ? 1 : 0;
                    }
                    if (rank < K) out[rank] = (int32_t)(off + ji);
                }
            }
        } else {
            for (int i = lane; i < cnt; i += 64) {
                const double di = s_d[i];
                const int ji = s_j[i];
                int rank = 0;
                for (int f2 = 0; f2 < cnt; ++f2) {  // (every lane reads entry f2: LDS broadcast)
                    const double df = s_d[f2];
                    rank += ((df < di) | ((df == di) & (s_j[f2] < ji))) ? 1 : 0;
                }
                if (rank < K) out[rank] = (int32_t)(off + ji);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the list is rewritten by the next query)
        return true;
    }
    return false;
}

// The listed queries' rows, dense in problem order (row d of problem p: its (d - first
// row of p)-th query), one wave per query: the row (global ids) and the row's node.
template <int K>
__global__ __launch_bounds__(64) void k_pb_rows(PlanBatchDev P) {
    const int lane = threadIdx.x;
    const int wave = blockIdx.x, nwaves = gridDim.x;  // (one wave per workgroup)
    // rows per problem (lane p holds problem p's) and their inclusive prefix
    int mine = 0;
    if (lane < P.S) mine = (int)min(pb_ctr(P, kFQueries, lane), (unsigned long long)max(P.seg[lane].cap, 0));
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
    }
    const int D = __shfl(incl, 63, 64);
    if (wave == 0 && lane == 0) P.ctr[kPbRows] = (unsigned long long)D;
    // The query's node and coordinates are loaded one query ahead (wave-uniform loads in
    // flight while the current query runs: two dependent round trips off every query).
    auto locate = [&](int d, int& p, int& self, double (&pt)[3]) {
        p = __popcll(__ballot(lane < P.S && incl <= d));  // problems whose rows end at or before d
        const int first = __builtin_amdgcn_readfirstlane(__shfl(incl - mine, p, 64));
        self = __builtin_amdgcn_readfirstlane(P.query[P.seg[p].row_off + (d - first)]);
        const double* x = P.nodes + (((int64_t)p << P.ns_log) + self) * 3;
        pt[0] = x[0];
        pt[1] = x[1];
        pt[2] = x[2];
    };
    int p_n = 0, self_n = 0;
    double pt_n[3] = {0.0, 0.0, 0.0};
    [[maybe_unused]] const unsigned long long tl_w0 = EPP_PBTL_NOW();
    if (wave < D) locate(wave, p_n, self_n, pt_n);
    // (static shares, d = wave + j nwaves: handing the queries out by one atomic counter
    // serialised ~19k same-address atomics at one L2 channel -- 0.17 -> 0.37 ms per batch;
    // and every load behind a pending atomic waits for it: vmcnt counts in order)
    for (int d = wave; d < D; d += nwaves) {  // wave-uniform
        EPP_PBTL(d, 0, EPP_PBTL_NOW());
        EPP_PBTL(d, 5, tl_w0);
        const int p = p_n, self = self_n;
        const double pt[3] = {pt_n[0], pt_n[1], pt_n[2]};
        if (d + nwaves < D) locate(d + nwaves, p_n, self_n, pt_n);
        const PlanSeg& q = P.seg[p];
        const int64_t off = (int64_t)p << P.ns_log;
        const KnnSeg ks = knn_seg(P, p);
        const KnnGrid g = *ks.g;
        const double f = pb_ellipse(q, pt);
        if (lane == 0) P.ids32[d] = (int32_t)(off + self);
        if (!pb_query_row<K>(g, ks.sxyz, ks.sidx, ks.start, pt, f, q.gbound, self, P.rows32 + (int64_t)d * K, off, d)) {
            if (lane == 0) pb_ctr(P, kFInexact, p) = 1ull;
            if (lane < K) P.rows32[(int64_t)d * K + lane] = -1;  // (the problem takes the whole table)
        }
#ifdef EPP_PB_ROWS_TL
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        EPP_PBTL(d, 3, EPP_PBTL_NOW());
        if ((threadIdx.x & 63) == 0 && d < kPbTl) g_pb_rows_tl[d][4] |= (unsigned long long)wave << 32;
#endif
    }
}

// Per problem: the marked nodes numbered in node order -- an ordered compaction of the
// marks, chunks of 1024 node ids per workgroup (4 rounds of 256), the chunk's offset by
// decoupled look-back (lb_exclusive); map[node] = its index, its coordinates listed at
// need_off + index.  The workgroup holding the problem's last node writes the count.
__global__ __launch_bounds__(kCompactThreads) void k_pb_number(PlanBatchDev P, uint32_t tag) {
    const int p = blockIdx.y;
    const PlanSeg& q = P.seg[p];
    if (q.cap <= 0) return;  // (block-uniform)
    const int n = (int)pb_ctr(P, kFNodes, p);
    const int b = blockIdx.x;
    if (b * kCompactChunk >= n) return;  // (no later chunk waits on it)
    constexpr int NW = kCompactThreads / 64;
    __shared__ int wcnt[kCompactRounds * NW];
    __shared__ long long s_excl;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t off = (int64_t)p << P.ns_log;
    unsigned long long* st = P.nstat + (int64_t)p * (P.NS / kCompactChunk);
    bool v[kCompactRounds];
    unsigned long long bal[kCompactRounds];
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        const int i = b * kCompactChunk + r * kCompactThreads + threadIdx.x;
        v[r] = i < n && P.mark[off + i] != 0;
        bal[r] = __ballot(v[r]);
        if (lane == 0) wcnt[r * NW + wv] = __popcll(bal[r]);
    }
    __syncthreads();
    int before[kCompactRounds], total = 0;
#pragma unroll
    for (int qq = 0; qq < kCompactRounds * NW; ++qq) {
#pragma unroll
        for (int r = 0; r < kCompactRounds; ++r)
            if (qq == r * NW + wv) before[r] = total;
        total += wcnt[qq];
    }
    if (wv == 0) {
        if (lane == 0) lb_publish(st, b, tag, b == 0, total);
        const long long ex = b == 0 ? 0ll : lb_exclusive(st, b, tag);
        if (lane == 0) {
            if (b > 0) lb_publish(st, b, tag, true, ex + total);
            s_excl = ex;
            if ((b + 1) * kCompactChunk >= n) pb_ctr(P, kFNeed, p) = (unsigned long long)(ex + total);
        }
    }
    __syncthreads();
    const long long ex = s_excl;
#pragma unroll
    for (int r = 0; r < kCompactRounds; ++r) {
        if (v[r]) {
            const int i = b * kCompactChunk + r * kCompactThreads + threadIdx.x;
            const long long at = ex + before[r] +
                                 (long long)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal[r] >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bal[r], 0u));
            P.map[off + i] = (int32_t)at;
            if (at < q.need_cap) {
                const double* x = P.nodes + (off + i) * 3;
                double* d = P.need + (q.need_off + at) * 3;
                d[0] = x[0];
                d[1] = x[1];
                d[2] = x[2];
            }
        }
    }
}

// The results into pinned host memory, only the bytes in use: the header (counters), the
// rows' problem and compact node index (u32), the masked rows in compact indices (u16,
// renumbered here through `map` as they are copied), every problem's referenced nodes
// (24 B each, at its own offset).  16-byte stores (the device parts are 16-byte padded).
// Each workgroup then publishes `seq` in its completion slot (host memory, system scope,
// after a system fence over its stores): the host polls the slots instead of synchronising
// the stream.
__global__ __launch_bounds__(256) void k_pb_emit(PlanBatchDev P, unsigned long long* __restrict__ hdr,
                                                  uint4* __restrict__ h_slot, uint4* __restrict__ h_rows,
                                                  uint4* __restrict__ h_need, uint32_t* __restrict__ done,
                                                  uint32_t seq) {
    __shared__ long long pre[65];  // 16-byte chunks of the referenced nodes before problem p (S <= 64)
    __shared__ long long first[64];
    const int64_t rows = (int64_t)P.ctr[kPbRows];
    if (threadIdx.x == 0) {
        long long a = 0;
        for (int p = 0; p < P.S; ++p) {
            pre[p] = a;
            // problem p's slots [need_off, need_off + cnt) as 16-byte chunks (24 B per node;
            // need_off is even, so the range starts on a chunk)
            const long long cnt = min((long long)pb_ctr(P, kFNeed, p), (long long)P.seg[p].need_cap);
            first[p] = P.seg[p].need_off * 3 / 2;
            a += (cnt * 3 + 1) / 2;
        }
        pre[P.S] = a;
    }
    __syncthreads();
    const int64_t c_slot = (rows * 4 + 15) / 16, c_rows = (rows * P.k * 2 + 15) / 16, c_need = pre[P.S];
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid < P.nctr) hdr[tid] = P.ctr[tid];
    const uint4* d_rows = reinterpret_cast<const uint4*>(P.rows16);
    const uint4* d_need = reinterpret_cast<const uint4*>(P.need);
    const uint32_t lmask = (1u << P.ns_log) - 1u;
    // a row entry (node id in its problem, 0xFFFF: none) in compact indices
    auto remap = [&](int64_t e, uint32_t v) -> uint32_t {
        if (v == 0xFFFFu || e >= rows * P.k) return v;
        const int32_t u = P.ids32[e / P.k];
        return (uint32_t)P.map[(u & ~(int32_t)lmask) + (int32_t)v] & 0xFFFFu;
    };
    for (int64_t c = tid; c < c_slot + c_rows + c_need; c += (int64_t)gridDim.x * 256) {
        if (c < c_slot) {  // (p << 16 | the row's node, compact) for rows 4c .. 4c + 3
            uint32_t sv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t r = 4 * c + j;
                const int32_t u = r < rows ? P.ids32[r] : 0;
                sv[j] = r < rows ? (((uint32_t)u >> P.ns_log) << 16) | ((uint32_t)P.map[u] & 0xFFFFu) : 0u;
            }
            h_slot[c] = make_uint4(sv[0], sv[1], sv[2], sv[3]);
        } else if (c < c_slot + c_rows) {  // 8 row entries
            const int64_t cr = c - c_slot;
            const uint4 w = d_rows[cr];
            const uint32_t in[4] = {w.x, w.y, w.z, w.w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t e = 8 * cr + 2 * j;
                o[j] = remap(e, in[j] & 0xFFFFu) | (remap(e + 1, in[j] >> 16) << 16);
            }
            h_rows[cr] = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            const int64_t r = c - c_slot - c_rows;
            int p = 0;
            while (p + 1 < P.S && pre[p + 1] <= r) ++p;
            const int64_t at = first[p] + (r - pre[p]);
            h_need[at] = d_need[at];
        }
    }
    wg_stores_settled();
    if (threadIdx.x == 0) __hip_atomic_store(done + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kPbEmitMax = 1024;  // emit workgroups (one completion slot each)

// ---- the reverse edges of a k-NN table as a CSR (the planner's symmetrised search) -----
// roff[v] .. roff[v + 1]: the nodes u whose (masked) row holds v, ascending -- the order
// the host's own build gives them (rows scanned in node order), so A* relaxes them in the
// same order.  Counting sort: in-degrees by atomics, one workgroup's scan, a scatter by
// atomics, then every node's run sorted (insertion sort: ~k entries).
__global__ __launch_bounds__(256) void k_rev_count(const int32_t* __restrict__ nbr, int64_t m, int32_t* __restrict__ cnt) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e < m && nbr[e] >= 0) atomicAdd(&cnt[nbr[e]], 1);
}
__global__ __launch_bounds__(1024) void k_rev_scan(const int32_t* __restrict__ cnt, int32_t n, int32_t* __restrict__ roff,
                                                   int32_t* __restrict__ fill) {
    __shared__ int wsum[16];
    __shared__ int s_carry;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    for (int c0 = 0; c0 < n; c0 += 1024 * 16) {  // chunks of 16 counts per thread
        const int b0 = c0 + (int)threadIdx.x * 16;
        int v[16], sum = 0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            v[u] = b0 + u < n ? cnt[b0 + u] : 0;
            sum += v[u];
        }
        int incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        __syncthreads();
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int acc = s_carry + incl - sum;
        for (int w = 0; w < wv; ++w) acc += wsum[w];
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = acc + sum;
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (b0 + u < n) {
                roff[b0 + u] = acc;
                fill[b0 + u] = acc;
                acc += v[u];
            }
    }
    __syncthreads();
    if (threadIdx.x == 0) roff[n] = s_carry;
}
__global__ __launch_bounds__(256) void k_rev_fill(const int32_t* __restrict__ nbr, int64_t m, int32_t k,
                                                  int32_t* __restrict__ fill, int32_t* __restrict__ radj) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= m) return;
    const int32_t v = nbr[e];
    if (v >= 0) radj[atomicAdd(&fill[v], 1)] = (int32_t)(e / k);
}
__global__ __launch_bounds__(256) void k_rev_sort(const int32_t* __restrict__ roff, int32_t n, int32_t* __restrict__ radj,
                                                  uint16_t* __restrict__ radj16) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= n) return;
    const int a = roff[v], b = roff[v + 1];
    for (int i = a + 1; i < b; ++i) {  // (insertion sort of the node's run)
        const int32_t x = radj[i];
        int j = i - 1;
        while (j >= a && radj[j] > x) {
            radj[j + 1] = radj[j];
            --j;
        }
        radj[j + 1] = x;
    }
    if (radj16)
        for (int i = a; i < b; ++i) radj16[i] = (uint16_t)radj[i];
}

int cu_count_planner() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
}

epp_status last(const char* what) {
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

epp_status epp_sample_uniform(uint64_t seed, const double lo[3], const double hi[3], int64_t n,
                              int64_t start, double* xyz, void* stream) {
    if (n < 0 || (n > 0 && (!lo || !hi || !xyz))) {
        set_error("epp_sample_uniform: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    hipLaunchKernelGGL(k_sample_uniform, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       seed, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], n, start, xyz, nullptr, (int64_t)0);
    return last("epp_sample_uniform");
}

epp_status epp_knn_bruteforce(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr,
                              void* stream) {
    if (n < 0 || (n > 0 && (!nodes || !nbr)) || (k != 4 && k != 8 && k != 16 && k != 32)) {
        set_error("epp_knn: invalid argument (k must be 4, 8, 16 or 32)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const double r2 = max_dist > 0 ? max_dist * max_dist : 1e300;
    const dim3 grid((n + kKnnBlock - 1) / kKnnBlock), block(kKnnBlock);
    hipStream_t s = (hipStream_t)stream;
    switch (k) {
        case 4: hipLaunchKernelGGL(k_knn<4>, grid, block, 0, s, nodes, n, r2, nbr); break;
        case 8: hipLaunchKernelGGL(k_knn<8>, grid, block, 0, s, nodes, n, r2, nbr); break;
        case 16: hipLaunchKernelGGL(k_knn<16>, grid, block, 0, s, nodes, n, r2, nbr); break;
        default: hipLaunchKernelGGL(k_knn<32>, grid, block, 0, s, nodes, n, r2, nbr); break;
    }
    return last("epp_knn_bruteforce");
}

epp_status epp_knn(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* stream) {
    // the grid pays off from a few thousand nodes; both give the same answer
    // (EPP_KNN_IMPL=1 / 2 forces all-pairs / grid: diagnostics)
    const char* f = std::getenv("EPP_KNN_IMPL");
    const int impl = f && *f ? std::atoi(f) : 0;
    const bool brute = impl == 1 || (impl == 0 && n <= 2048);
    return brute ? epp_knn_bruteforce(nodes, n, k, max_dist, nbr, stream)
                 : epp_knn_grid(nodes, n, k, max_dist, nbr, stream);
}

uint64_t epp_knn_workspace_size(int32_t n) { return n <= 0 ? 0 : (uint64_t)knn_layout(n).bytes; }

#ifdef EPP_PB_ROWS_TL
// (diagnostics builds only) the last k_pb_rows launch's per-query stamps: 6 u64 each
epp_status epp_dbg_pb_rows_tl(unsigned long long* out, int64_t n) {
    if (n > kPbTl) n = kPbTl;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pb_rows_tl), (size_t)n * 48) == hipSuccess ? EPP_OK : EPP_ERR_HIP;
}
#endif

#ifdef EPP_KNN_DIAG
// (diagnostics builds only) the last k_knn_tile launch's phase timeline: 16 u64 per block
epp_status epp_dbg_knn_tl(unsigned long long* out, int64_t blocks) {
    unsigned long long* d = knn_tl_buffer();
    if (!d || blocks > kKnnTlBlocks) return EPP_ERR_RUNTIME;
    return hipMemcpy(out, d, (size_t)blocks * 16 * 8, hipMemcpyDeviceToHost) == hipSuccess ? EPP_OK : EPP_ERR_HIP;
}
// (diagnostics builds only) the last k_knn_retry launch: per retried query start, end,
// bound (f64 bits), node -- 4 u64 each
epp_status epp_dbg_knn_retry_tl(unsigned long long* out, int64_t n) {
    if (n > kKnnRetryTl) n = kKnnRetryTl;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_knn_retry_tl), (size_t)n * 32) == hipSuccess ? EPP_OK : EPP_ERR_HIP;
}
#endif

epp_status epp_knn_ws(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* ws,
                      uint64_t ws_bytes, void* stream) {
    if (n > 2048) return epp_knn_grid_ws(nodes, n, k, max_dist, nbr, ws, ws_bytes, stream);
    return epp_knn_bruteforce(nodes, n, k, max_dist, nbr, stream);
}

epp_status epp_knn_grid_ws_box(const double* nodes, int32_t n, int32_t k, double max_dist, const double lo[3],
                               const double hi[3], int32_t* nbr, void* ws, uint64_t ws_bytes, void* stream) {
    if (n < 0 || (n > 0 && (!nodes || !nbr)) || (k != 4 && k != 8 && k != 16 && k != 32) || !lo || !hi ||
        !(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2])) {
        set_error("epp_knn_grid_ws_box: invalid argument (k must be 4, 8, 16 or 32; lo <= hi)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const KnnLayout L = knn_layout(n);
    if (!ws || ws_bytes < L.bytes || (reinterpret_cast<uintptr_t>(ws) & 255)) {
        set_error("epp_knn_grid_ws_box: workspace missing, unaligned or smaller than epp_knn_workspace_size(n)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    return knn_grid_launch(nodes, n, k, max_dist, nbr, static_cast<char*>(ws), L, (hipStream_t)stream, lo, hi);
}

epp_status epp_knn_ws_box(const double* nodes, int32_t n, int32_t k, double max_dist, const double lo[3],
                          const double hi[3], int32_t* nbr, void* ws, uint64_t ws_bytes, void* stream) {
    if (n > 2048) return epp_knn_grid_ws_box(nodes, n, k, max_dist, lo, hi, nbr, ws, ws_bytes, stream);
    return epp_knn_bruteforce(nodes, n, k, max_dist, nbr, stream);
}

epp_status epp_knn_grid_ws(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* ws,
                           uint64_t ws_bytes, void* stream) {
    if (n < 0 || (n > 0 && (!nodes || !nbr)) || (k != 4 && k != 8 && k != 16 && k != 32)) {
        set_error("epp_knn_grid: invalid argument (k must be 4, 8, 16 or 32)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    const KnnLayout L = knn_layout(n);
    if (!ws || ws_bytes < L.bytes || (reinterpret_cast<uintptr_t>(ws) & 255)) {
        set_error("epp_knn_grid: workspace missing, unaligned or smaller than epp_knn_workspace_size(n)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    return knn_grid_launch(nodes, n, k, max_dist, nbr, static_cast<char*>(ws), L, (hipStream_t)stream);
}

// Without a caller workspace: one cached workspace per device.  Reuse is ordered on the
// GPU (the next user's stream waits for the previous user's completion event), growth
// frees the old buffer only after the device drained it (hipFree synchronises).
epp_status epp_knn_grid(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* stream) {
    if (n < 0 || (n > 0 && (!nodes || !nbr)) || (k != 4 && k != 8 && k != 16 && k != 32)) {
        set_error("epp_knn_grid: invalid argument (k must be 4, 8, 16 or 32)");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    CachedWs& c = g_knn_ws[dev & 63];
    std::lock_guard<std::mutex> lk(c.mu);
    hipStream_t s = (hipStream_t)stream;
    const KnnLayout L = knn_layout(n);
    hipError_t e = hipSuccess;
    e = c.acquire(s, L.bytes);
    if (e != hipSuccess) {
        set_error(std::string("epp_knn_grid: workspace: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    const epp_status rc = knn_grid_launch(nodes, n, k, max_dist, nbr, static_cast<char*>(c.buf), L, s);
    c.release(s);
    return rc;
}

epp_status epp_compact_states(const double* xyz, const uint8_t* valid, int64_t n, double* out, int64_t* n_out,
                              void* stream) {
    if (n < 0 || !n_out || (n > 0 && (!xyz || !valid || !out))) {
        set_error("epp_compact_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = (hipStream_t)stream;
    // the look-back status words live in a cached per-device workspace (stream-ordered reuse)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    CachedWs& c = g_compact_ws[dev & 63];
    std::lock_guard<std::mutex> lk(c.mu);
    hipError_t e = c.acquire(s, (size_t)epp_compact_workspace_size(n));
    if (e != hipSuccess) {
        set_error(std::string("epp_compact_states: workspace: ") + hipGetErrorString(e));
        return EPP_ERR_HIP;
    }
    const epp_status rc = epp_compact_states_ws(xyz, valid, n, out, n_out, c.buf, c.cap, stream);
    c.release(s);
    return rc;
}

uint64_t epp_compact_workspace_size(int64_t n) {
    return n <= 0 ? 8 : (uint64_t)((n + kCompactChunk - 1) / kCompactChunk) * 8;
}

epp_status epp_compact_states_ws(const double* xyz, const uint8_t* valid, int64_t n, double* out, int64_t* n_out,
                                 void* ws, uint64_t ws_bytes, void* stream) {
    if (n < 0 || !n_out || (n > 0 && (!xyz || !valid || !out)) || !ws || ws_bytes < epp_compact_workspace_size(n) ||
        (reinterpret_cast<uintptr_t>(ws) & 7)) {
        set_error("epp_compact_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int nb = (int)std::max<int64_t>(1, (n + kCompactChunk - 1) / kCompactChunk);
    // the workspace may hold anything (e.g. carved from a buffer that held other data):
    // zero its status words first, so none reads as published in this launch
    if (hipMemsetAsync(ws, 0, (size_t)nb * 8, (hipStream_t)stream) != hipSuccess) return last("epp_compact_states");
    hipLaunchKernelGGL(k_compact, dim3(nb), dim3(kCompactThreads), 0, (hipStream_t)stream, xyz, valid, n,
                       static_cast<unsigned long long*>(ws), next_scan_tag(), out, n_out);
    return last("epp_compact_states");
}

epp_status epp_mask_edges(int32_t* nbr, const uint8_t* valid, int64_t m, void* stream) {
    if (m < 0 || (m > 0 && (!nbr || !valid))) {
        set_error("epp_mask_edges: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (m == 0) return EPP_OK;
    hipLaunchKernelGGL(k_mask_edges, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, nbr,
                       valid, m);
    return last("epp_mask_edges");
}

epp_status epp_mask_edges_count(int32_t* nbr, const uint8_t* valid, int64_t m, int32_t target, int64_t* count,
                                void* stream) {
    if (m < 0 || !count || (m > 0 && (!nbr || !valid))) {
        set_error("epp_mask_edges_count: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (hipMemsetAsync(count, 0, 2 * sizeof(int64_t), (hipStream_t)stream) != hipSuccess) return last("epp_mask_edges_count");
    return epp::mask_edges_count_acc(nbr, valid, m, target, count, stream);
}

}  // extern "C"

epp_status epp::sample_uniform_and_clear(uint64_t seed, const double lo[3], const double hi[3], int64_t n, double* xyz,
                                         void* clr, uint64_t clr_bytes, void* stream) {
    const int64_t nclr = (int64_t)(clr_bytes / 8);
    if (n < 0 || (n > 0 && !xyz) || !lo || !hi || (nclr > 0 && (!clr || (reinterpret_cast<uintptr_t>(clr) & 7)))) {
        set_error("epp_sample_uniform: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int64_t m = std::max(n, nclr);
    if (m == 0) return EPP_OK;
    hipLaunchKernelGGL(k_sample_uniform, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, seed,
                       lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], n, (int64_t)0, xyz,
                       static_cast<unsigned long long*>(clr), nclr);
    return last("epp_sample_uniform");
}

epp_status epp::compact_states_cleared(const double* xyz, const uint8_t* valid, int64_t n, double* out,
                                       int64_t* n_out, void* ws, uint64_t ws_bytes, void* stream) {
    if (n < 0 || !n_out || (n > 0 && (!xyz || !valid || !out)) || !ws || ws_bytes < epp_compact_workspace_size(n) ||
        (reinterpret_cast<uintptr_t>(ws) & 7)) {
        set_error("epp_compact_states: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int nb = (int)std::max<int64_t>(1, (n + kCompactChunk - 1) / kCompactChunk);
    hipLaunchKernelGGL(k_compact, dim3(nb), dim3(kCompactThreads), 0, (hipStream_t)stream, xyz, valid, n,
                       static_cast<unsigned long long*>(ws), next_scan_tag(), out, n_out);
    return last("epp_compact_states");
}

epp_status epp::mask_edges_count_acc(int32_t* nbr, const uint8_t* valid, int64_t m, int32_t target, int64_t* count,
                                     void* stream, uint16_t* out16) {
    if (m < 0 || !count || (m > 0 && (!nbr || !valid))) {
        set_error("epp_mask_edges_count: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = (hipStream_t)stream;
    if (m == 0) return EPP_OK;
    const int64_t blocks = std::min<int64_t>((m + kMaskThreads - 1) / kMaskThreads, 256);
    hipLaunchKernelGGL(k_mask_edges_count, dim3((unsigned)blocks), dim3(kMaskThreads), 0, s, nbr, valid, m, target,
                       reinterpret_cast<unsigned long long*>(count), out16);
    return last("epp_mask_edges_count");
}

epp_status epp::pack_ellipse_rows(const double* nodes, const int32_t* tab, int32_t n, int32_t k, const double s[3],
                                  const double g[3], double bound, int32_t cap, int32_t* ids32, uint16_t* ids16,
                                  int32_t* rows32, int64_t* count, void* stream) {
    // ids16 are u16: n <= 65535 (the narrow table); 16-B aligned rows for the vector copy
    if (n < 0 || n > 65535 || k <= 0 || cap < 0 || !count || !s || !g ||
        (n > 0 && (!nodes || !tab || !ids32 || !ids16 || !rows32)) || (reinterpret_cast<uintptr_t>(tab) & 15) ||
        (reinterpret_cast<uintptr_t>(rows32) & 15)) {
        set_error("pack_ellipse_rows: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return EPP_OK;
    hipLaunchKernelGGL(k_pack_ellipse_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       nodes, tab, n, k, s[0], s[1], s[2], g[0], g[1], g[2], bound, cap, ids32, ids16, rows32,
                       reinterpret_cast<unsigned long long*>(count));
    return last("pack_ellipse_rows");
}

epp_status epp::knn_ws_box_ellipse(const double* nodes, int32_t n, int32_t k, const double lo[3], const double hi[3],
                                   const double s[3], const double g[3], double bound, int32_t* nbr, void* ws,
                                   uint64_t ws_bytes, void* stream) {
    if (n <= 2048 || (k != 4 && k != 8 && k != 16)) return epp_knn_ws_box(nodes, n, k, 0.0, lo, hi, nbr, ws, ws_bytes, stream);
    if (!nodes || !nbr || !lo || !hi || !s || !g || !(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2])) {
        set_error("knn_ws_box_ellipse: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const KnnLayout L = knn_layout(n);
    if (!ws || ws_bytes < L.bytes || (reinterpret_cast<uintptr_t>(ws) & 255)) {
        set_error("knn_ws_box_ellipse: workspace missing, unaligned or too small");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const double q[7] = {s[0], s[1], s[2], g[0], g[1], g[2], bound};
    return knn_grid_launch(nodes, n, k, 0.0, nbr, static_cast<char*>(ws), L, (hipStream_t)stream, lo, hi, q);
}

extern "C" {

epp_status epp_knn_edges(const double* nodes, const int32_t* nbr, int32_t n, int32_t k, double* s1,
                         double* s2, void* stream) {
    if (n < 0 || k <= 0 || (n > 0 && (!nodes || !nbr || !s1 || !s2))) {
        set_error("epp_knn_edges: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    const int64_t m = (int64_t)n * k;
    if (m == 0) return EPP_OK;
    hipLaunchKernelGGL(k_knn_edges, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, nodes,
                       nbr, m, k, s1, s2);
    return last("epp_knn_edges");
}

}  // extern "C"

// ---- the batched planner's host side (epp_internal.h) ---------------------------------
epp::PlanBatchLayout epp::plan_batch_layout(int32_t S, int64_t ns, int32_t k, PlanSeg* segs) {
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    PlanBatchLayout L;
    L.S = S;
    L.k = k;
    L.ns = ns;
    L.ns_log = 16;
    while ((1ll << L.ns_log) < ns + 2) ++L.ns_log;
    L.NS = 1ll << L.ns_log;
    L.nbc = (int32_t)std::max<int64_t>(1, (ns + kCompactChunk - 1) / kCompactChunk);
    // rows: the problems' capacities; referenced nodes: a row's node and its k neighbours
    // per row, at most the problem's nodes (even counts: 24-byte entries on 16-byte chunks)
    int64_t rows = 0, need = 0;
    for (int p = 0; p < S; ++p) {
        segs[p].cap = std::max(0, segs[p].cap);
        segs[p].row_off = rows;
        rows += segs[p].cap;
        segs[p].need_off = need;
        segs[p].need_cap =
            segs[p].cap > 0 ? (int32_t)((std::min<int64_t>((int64_t)segs[p].cap * (k + 1) + 2, ns + 2) + 1) & ~1ll) : 0;
        need += segs[p].need_cap;
    }
    L.cap_total = (int32_t)rows;
    L.need_cap = need;
    L.nctr = kPbPerSeg + 6 * S;
    const bool R = rows > 0;
    const KnnLayout kl = knn_layout((int)(ns + 2));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += al(bytes);
        return at;
    };
    L.o_seg = take((size_t)S * sizeof(PlanSeg));
    L.o_ctr = take((size_t)L.nctr * 8);
    L.o_xyz = take((size_t)S * ns * 24);
    L.o_valid = take((size_t)S * ns);
    L.o_nodes = take((size_t)S * L.NS * 24);
    L.o_cstat = take((size_t)S * L.nbc * 8);
    L.kws_stride = R ? al(kl.bytes) : 0;
    L.o_kws = take((size_t)S * L.kws_stride);
    const size_t capr = ((size_t)rows + 3) & ~size_t(3);
    L.o_query = take(capr * 4);
    L.o_ids32 = take(capr * 4);
    L.o_rows32 = take(capr * k * 4);
    L.o_rows16 = take(capr * k * 2);
    L.o_ev = take(capr * k);
    L.o_mark = take(R ? (size_t)S * L.NS : 0);
    L.o_map = take(R ? (size_t)S * L.NS * 4 : 0);
    L.o_nstat = take(R ? (size_t)S * (L.NS / kCompactChunk) * 8 : 0);
    L.o_need = take((size_t)L.need_cap * 24 + 16);
    L.dev_bytes = o;
    o = 0;
    L.h_seg = take((size_t)S * sizeof(PlanSeg));
    L.h_hdr = take((size_t)L.nctr * 8);
    L.h_slot = take(capr * 4);
    L.h_rows = take(capr * k * 2);
    L.h_need = take((size_t)L.need_cap * 24 + 16);
    {  // emit workgroups: each one's completion release writes back its XCD's L2 (once per
       // workgroup since completion.h; kernel trace, scripts/gpu_emit_ab.sh: 64 -> 26.6 us,
       // 128 -> 21.6, 256 -> 23.3, 512 -> 29.1)
        static const int eb = [] {
            const char* e = std::getenv("EPP_PB_EMIT_BLOCKS");  // (A/B knob: same results)
            const int v = e && *e ? std::atoi(e) : 128;
            return std::max(1, std::min(kPbEmitMax, v));
        }();
        L.done_n = eb;
    }
    L.h_done = take((size_t)L.done_n * 4);
    L.host_bytes = o;
    return L;
}

// EPP_PB_TRACE=1 (diagnostics knob, read once): events between the batch's stages on its
// stream; plan_batch_trace_print() (after the batch completed) prints each stage's time in
// microseconds to stderr, one line per batch.
namespace {
struct PbTrace {
    bool on = false;
    int n = 0;
    hipEvent_t ev[16] = {};
    const char* name[16] = {};
};
PbTrace& pb_trace() {
    static const bool on = [] {
        const char* e = std::getenv("EPP_PB_TRACE");
        return e && std::atoi(e) == 1;
    }();
    thread_local PbTrace t;
    if (on && !t.on) {
        t.on = true;
        for (auto& e : t.ev) (void)hipEventCreate(&e);
    }
    return t;
}
void pb_mark(hipStream_t s, const char* name) {
    PbTrace& t = pb_trace();
    if (!t.on || t.n >= 16) return;
    t.name[t.n] = name;
    (void)hipEventRecord(t.ev[t.n++], s);
}
}  // namespace

void epp::plan_batch_trace_print() {
    PbTrace& t = pb_trace();
    if (!t.on || t.n < 2) return;
    (void)hipEventSynchronize(t.ev[t.n - 1]);
    std::string line = "pb_trace:";
    float tot = 0;
    for (int i = 1; i < t.n; ++i) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, t.ev[i - 1], t.ev[i]);
        tot += ms;
        line += std::string(" ") + t.name[i] + "=" + std::to_string((int)(ms * 1000.0f + 0.5f));
    }
    line += " total=" + std::to_string((int)(tot * 1000.0f + 0.5f));
    std::fprintf(stderr, "%s\n", line.c_str());
    t.n = 0;
}

epp_status epp::plan_batch_launch(const epp_world* world, int32_t can_pass_gate, const double lo[3], const double hi[3],
                                  const PlanBatchLayout& L, void* dev, void* host, uint32_t seq, void* stream) {
    if (!world || !dev || !host || L.S < 1 || L.S > 64 || L.ns < 1 || (L.k != 4 && L.k != 8 && L.k != 16) ||
        ((int64_t)L.S << L.ns_log) >= (1ll << 31) || (reinterpret_cast<uintptr_t>(dev) & 255) ||
        (reinterpret_cast<uintptr_t>(host) & 255)) {
        set_error("plan_batch_launch: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    char* d = static_cast<char*>(dev);
    char* h = static_cast<char*>(host);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const KnnLayout kl = knn_layout((int)(L.ns + 2));
    PlanBatchDev P{};
    P.seg = reinterpret_cast<const PlanSeg*>(d + L.o_seg);
    P.S = L.S;
    P.k = L.k;
    P.ns_log = L.ns_log;
    P.nbc = L.nbc;
    P.cap_total = L.cap_total;
    P.nctr = L.nctr;
    P.ns = L.ns;
    P.NS = L.NS;
    for (int i = 0; i < 3; ++i) {
        P.lo[i] = lo[i];
        P.hi[i] = hi[i];
    }
    P.xyz = reinterpret_cast<double*>(d + L.o_xyz);
    P.valid = reinterpret_cast<uint8_t*>(d + L.o_valid);
    P.nodes = reinterpret_cast<double*>(d + L.o_nodes);
    P.cstat = reinterpret_cast<unsigned long long*>(d + L.o_cstat);
    P.ctr = reinterpret_cast<unsigned long long*>(d + L.o_ctr);
    P.kws = d + L.o_kws;
    P.kws_stride = L.kws_stride;
    P.l_cell = kl.cell;
    P.l_sidx = kl.sidx;
    P.l_sxyz = kl.sxyz;
    P.l_cnt = kl.cnt;
    P.l_start = kl.start;
    P.l_fill = kl.fill;
    P.l_stat = kl.stat;
    P.l_cap = kl.cap;
    P.nclr = (int)((kl.start - kl.cnt) / sizeof(int));
    P.query = reinterpret_cast<int32_t*>(d + L.o_query);
    P.ids32 = reinterpret_cast<int32_t*>(d + L.o_ids32);
    P.rows32 = reinterpret_cast<int32_t*>(d + L.o_rows32);
    P.rows16 = reinterpret_cast<uint16_t*>(d + L.o_rows16);
    P.mark = reinterpret_cast<uint8_t*>(d + L.o_mark);
    P.nstat = reinterpret_cast<unsigned long long*>(d + L.o_nstat);
    P.map = reinterpret_cast<int32_t*>(d + L.o_map);
    P.need = reinterpret_cast<double*>(d + L.o_need);
    const unsigned S = (unsigned)L.S;
    const bool R = L.cap_total > 0;
    // the problems: in k_pb_sample's arguments (<= kPbSegArgMax), else uploaded first; then
    // every stage on this stream
    P.seg_h = nullptr;
    if (L.S <= kPbSegSmall) {
        P.seg_h = reinterpret_cast<const PlanSeg*>(h + L.h_seg);
        for (int p = 0; p < L.S; ++p) {
            P.seeds[p] = P.seg_h[p].seed;
            P.caps[p] = P.seg_h[p].cap;
        }
    } else {
        if (hipMemcpyAsync(d + L.o_seg, h + L.h_seg, (size_t)L.S * sizeof(PlanSeg), hipMemcpyHostToDevice, s) !=
            hipSuccess)
            return last("plan_batch_launch");
    }
    const int64_t clr = std::max<int64_t>({L.ns, R ? L.NS >> 4 : 0, R ? (int64_t)P.nclr : 0, (int64_t)L.nbc, (int64_t)L.nctr});
    pb_mark(s, "begin");
    hipLaunchKernelGGL(k_pb_sample, dim3((unsigned)((clr + 255) / 256), S), dim3(256), 0, s, P);
    if (const epp_status st = epp_check_states(world, P.xyz, (int64_t)L.S * L.ns, can_pass_gate, P.valid, nullptr,
                                               nullptr, stream))
        return st;
    pb_mark(s, "states");
    hipLaunchKernelGGL(k_pb_compact, dim3((unsigned)L.nbc, S), dim3(kCompactThreads), 0, s, P, next_scan_tag());
    if (R) {
        const unsigned gn = (unsigned)((L.ns + 2 + 255) / 256);
        pb_mark(s, "compact_member");
        hipLaunchKernelGGL(k_pb_knn_scan, dim3((unsigned)kl.scan_blocks, S), dim3(kScanThreads), 0, s, P, next_scan_tag());
        hipLaunchKernelGGL(k_pb_knn_scatter, dim3(gn, S), dim3(256), 0, s, P);
        pb_mark(s, "scan_scatter");
        // one wave per workgroup, 28 per CU (16 resident at ~110 VGPRs; a variant with four
        // queries per wave, 16 lanes each, was 1.9x slower: its 16-lane shuffles and LDS
        // ranking cost more issue than the overlapped loads saved)
        static const int rows_wg = [] {  // (A/B knob: one-wave workgroups per CU)
            const char* e = std::getenv("EPP_PB_ROWS_WG");
            const int v = e && *e ? std::atoi(e) : 28;
            return std::max(1, std::min(64, v));
        }();
        const dim3 gr((unsigned)std::max(1, cu_count_planner() * rows_wg)), br(64);
        if (L.k == 4) hipLaunchKernelGGL(k_pb_rows<4>, gr, br, 0, s, P);
        else if (L.k == 8) hipLaunchKernelGGL(k_pb_rows<8>, gr, br, 0, s, P);
        else hipLaunchKernelGGL(k_pb_rows<16>, gr, br, 0, s, P);
        pb_mark(s, "rows");
        // the motions, with the marks of the referenced nodes and the per-problem kept /
        // goal edge counts folded into the launch
        MotionMask marks;
        marks.mark = P.mark;
        marks.pkept = P.ctr + kPbPerSeg + kFKept * L.S;
        marks.pgoal = P.ctr + kPbPerSeg + kFGoal * L.S;
        marks.ns_log = L.ns_log;
        marks.nprob = L.S;
        if (const epp_status st = check_knn_motions_rows(
                world, P.nodes, P.rows32, P.ids32, reinterpret_cast<const int64_t*>(P.ctr + kPbRows), L.cap_total,
                L.k, can_pass_gate, reinterpret_cast<uint8_t*>(d + L.o_ev), P.rows16, -1, nullptr, stream, &marks))
            return st;
        pb_mark(s, "motions_marks");
        hipLaunchKernelGGL(k_pb_number, dim3((unsigned)((L.ns + 2 + kCompactChunk - 1) / kCompactChunk), S),
                           dim3(kCompactThreads), 0, s, P, next_scan_tag());
        pb_mark(s, "number");
    }
    hipLaunchKernelGGL(k_pb_emit, dim3((unsigned)L.done_n), dim3(256), 0, s, P,
                       reinterpret_cast<unsigned long long*>(h + L.h_hdr), reinterpret_cast<uint4*>(h + L.h_slot),
                       reinterpret_cast<uint4*>(h + L.h_rows), reinterpret_cast<uint4*>(h + L.h_need),
                       reinterpret_cast<uint32_t*>(h + L.h_done), seq);
    pb_mark(s, "emit");
    return last("plan_batch_launch");
}

epp_status epp::reverse_csr(const int32_t* nbr, int32_t n, int32_t k, int32_t* cnt, int32_t* fill, int32_t* roff,
                            int32_t* radj, uint16_t* radj16, void* stream) {
    if (n <= 0 || k <= 0 || !nbr || !cnt || !fill || !roff || !radj) {
        set_error("reverse_csr: invalid argument");
        return EPP_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t m = (int64_t)n * k;
    if (hipMemsetAsync(cnt, 0, (size_t)n * 4, s) != hipSuccess) return last("reverse_csr");
    hipLaunchKernelGGL(k_rev_count, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, nbr, m, cnt);
    hipLaunchKernelGGL(k_rev_scan, dim3(1), dim3(1024), 0, s, cnt, n, roff, fill);
    hipLaunchKernelGGL(k_rev_fill, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, nbr, m, k, fill, radj);
    hipLaunchKernelGGL(k_rev_sort, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, roff, n, radj, radj16);
    return last("reverse_csr");
}

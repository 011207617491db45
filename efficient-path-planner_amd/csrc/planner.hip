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

#include <string>

#include "epp_internal.h"

namespace epp {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_sample_uniform(uint64_t seed, double lox, double loy, double loz, double hix,
                                 double hiy, double hiz, int64_t n, int64_t start,
                                 double* __restrict__ xyz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
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
                       seed, lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], n, start, xyz);
    return last("epp_sample_uniform");
}

epp_status epp_knn(const double* nodes, int32_t n, int32_t k, double max_dist, int32_t* nbr, void* stream) {
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
    return last("epp_knn");
}

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

// latency_probe.hip — round-trip floors of the host-driven latency path (diagnostics only;
// not part of the product).  Build + run:
//   hipcc --offload-arch=gfx950 -O2 -o scripts/latency_probe scripts/latency_probe.hip && scripts/latency_probe
// Prints p50 / p99 microseconds per host call for:
//   sync       empty kernel + hipStreamSynchronize
//   devsync    hipDeviceSynchronize on an idle device
//   poll       empty kernel that publishes a pinned completion word; the host polls it
//   poll_r1    as poll, after one 8-byte read of pinned host memory per lane
//   poll_r4    four dependent pinned-host reads before the completion word
//   poll_d1    one read of device memory (an 8.7 KB record table staged by 256 lanes)
//   poll_h1    the same table read from pinned host memory (the stale-index small path)
//   poll_h1w   as poll_h1, the host rewriting the table before every call
//   karg2k     as poll, with a 2 KB kernel-argument struct
//   poll_w8k   as poll, after writing 8 KB of rows to pinned host memory
//   memcpy8k   hipMemcpyAsync H2D of 8 KB + empty kernel + poll
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__device__ __forceinline__ void publish(uint32_t* done, uint32_t seq) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_empty() {}

__global__ void k_poll(uint32_t* done, uint32_t seq) { publish(done, seq); }

// `dep` dependent reads of src (host or device), then publish
__global__ void k_read(const double* src, int dep, int nd, double* sink, uint32_t* done, uint32_t seq) {
    __shared__ double s[2048];
    double acc = 0.0;
    int idx = threadIdx.x;
    for (int d = 0; d < dep; ++d) {
        double v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = idx + q * 256 < nd ? src[idx + q * 256] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (idx + q * 256 < nd) s[idx + q * 256] = v[q];
        acc += v[0];
        idx = (idx + (acc > 1e300 ? 1 : 0)) % 256;  // dependent address
    }
    __syncthreads();
    if (acc == 12345.0) sink[0] = s[threadIdx.x];
    publish(done, seq);
}

struct Big {
    double v[256];
};
__global__ void k_karg(Big b, double* sink, uint32_t* done, uint32_t seq) {
    if (b.v[threadIdx.x & 255] == 12345.0) sink[0] = 1.0;
    publish(done, seq);
}

__global__ void k_write(double* out, int nd, uint32_t* done, uint32_t seq) {
    for (int i = threadIdx.x; i < nd; i += blockDim.x) out[i] = (double)i;
    publish(done, seq);
}

static void wait_word(volatile uint32_t* w, uint32_t seq) {
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != seq) _mm_pause();
}

template <typename F>
static void timeit(const char* name, int iters, F&& f) {
    std::vector<double> t(iters);
    for (int i = 0; i < iters; ++i) {
        auto a = std::chrono::steady_clock::now();
        f(i);
        auto b = std::chrono::steady_clock::now();
        t[i] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    std::vector<double> s(t.begin() + iters / 10, t.end());
    std::sort(s.begin(), s.end());
    std::printf("%-10s p50 %7.2f us  p99 %7.2f us  min %7.2f us\n", name, s[s.size() / 2], s[(size_t)(s.size() * 0.99)],
                s[0]);
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t* done;
    CK(hipHostMalloc((void**)&done, 64, hipHostMallocDefault));
    *done = 0;
    double *h_tab, *d_tab, *sink, *h_out;
    const int nd = 64 * 17;
    CK(hipHostMalloc((void**)&h_tab, nd * 8, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_out, 8192, hipHostMallocDefault));
    for (int i = 0; i < nd; ++i) h_tab[i] = i;
    CK(hipMalloc((void**)&d_tab, nd * 8));
    CK(hipMalloc((void**)&sink, 64));
    CK(hipMemcpy(d_tab, h_tab, nd * 8, hipMemcpyHostToDevice));
    std::vector<char> src8k(8192, 1);
    char* d8k;
    CK(hipMalloc((void**)&d8k, 8192));
    char* h8k;
    CK(hipHostMalloc((void**)&h8k, 8192, hipHostMallocDefault));
    const int it = 2000;
    uint32_t seq = 0;
    for (int w = 0; w < 50; ++w) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        (void)hipStreamSynchronize(st);
    }
    timeit("sync", it, [&](int) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        (void)hipStreamSynchronize(st);
    });
    timeit("devsync", it, [&](int) { (void)hipDeviceSynchronize(); });
    timeit("poll", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_poll, dim3(1), dim3(256), 0, st, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_r1", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_read, dim3(1), dim3(256), 0, st, (const double*)h_tab, 1, 256, sink, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_r4", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_read, dim3(1), dim3(256), 0, st, (const double*)h_tab, 4, 256, sink, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_d1", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_read, dim3(1), dim3(256), 0, st, (const double*)d_tab, 1, nd, sink, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_h1w", it, [&](int i) {  // the host rewrote the table just before (a record update)
        for (int k = 0; k < nd; ++k) h_tab[k] = i + k;
        ++seq;
        hipLaunchKernelGGL(k_read, dim3(1), dim3(256), 0, st, (const double*)h_tab, 1, nd, sink, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_h1", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_read, dim3(1), dim3(256), 0, st, (const double*)h_tab, 1, nd, sink, done, seq);
        wait_word(done, seq);
    });
    Big b{};
    timeit("karg2k", it, [&](int i) {
        ++seq;
        b.v[i & 255] = i;
        hipLaunchKernelGGL(k_karg, dim3(1), dim3(256), 0, st, b, sink, done, seq);
        wait_word(done, seq);
    });
    timeit("poll_w8k", it, [&](int) {
        ++seq;
        hipLaunchKernelGGL(k_write, dim3(1), dim3(256), 0, st, h_out, 1024, done, seq);
        wait_word(done, seq);
    });
    timeit("memcpy8k", it, [&](int) {
        ++seq;
        (void)hipMemcpyAsync(d8k, h8k, 8192, hipMemcpyHostToDevice, st);
        hipLaunchKernelGGL(k_poll, dim3(1), dim3(256), 0, st, done, seq);
        wait_word(done, seq);
    });
    CK(hipStreamSynchronize(st));
    std::printf("ok\n");
    return 0;
}

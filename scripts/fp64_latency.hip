// fp64_latency.hip — dependent-instruction latencies on gfx950 (diagnostics only; not
// part of the product): one wavefront runs a chain of 256 dependent operations and the
// shader clock (s_memtime) brackets it.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o scripts/fp64_latency scripts/fp64_latency.hip && scripts/fp64_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kChain = 256;

template <int OP>
__global__ void k_chain(double* out, unsigned long long* cycles, double seed, int lanes) {
    double x = seed + threadIdx.x * 1e-9, y = 1.0000001;
    __shared__ double lds[256];
    lds[threadIdx.x] = x;
    __syncthreads();
    if ((int)threadIdx.x >= lanes) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < kChain; ++i) {
        if (OP == 0) x = fma(x, y, 1e-30);                 // v_fma_f64
        if (OP == 1) x = x * y;                            // v_mul_f64
        if (OP == 2) x = __builtin_amdgcn_rsq(x) + 0.5;    // v_rsq_f64 (+ add)
        if (OP == 3) x = __builtin_amdgcn_rcp(x) + 0.5;    // v_rcp_f64 (+ add)
        if (OP == 4) x = lds[((int)x & 1) + threadIdx.x % 64] + 1.0;  // LDS read -> add (address dependent)
        if (OP == 5) x = (float)x * 1.0000001f;            // f32 mul (+ cvts)
        if (OP == 6) x = x + 1e-30;                        // v_add_f64
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) *cycles = t1 - t0;
}

int main() {
    double* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 8);
    (void)hipMallocManaged(&cyc, 8);
    const char* names[] = {"fma_f64", "mul_f64", "rsq_f64+add", "rcp_f64+add", "lds_read+add", "f32 mul+cvt", "add_f64"};
    for (int lanes : {1, 64}) {
        for (int op = 0; op < 7; ++op) {
            unsigned long long best = ~0ull;
            for (int r = 0; r < 5; ++r) {
                switch (op) {
                    case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 3: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 4: hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 5: hipLaunchKernelGGL(k_chain<5>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                    case 6: hipLaunchKernelGGL(k_chain<6>, dim3(1), dim3(64), 0, 0, out, cyc, 1.5, lanes); break;
                }
                (void)hipDeviceSynchronize();
                if (*cyc < best) best = *cyc;
            }
            std::printf("lanes %2d  %-14s %6.1f cycles per dependent step\n", lanes, names[op], (double)best / kChain);
        }
    }
    return 0;
}

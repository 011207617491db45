// diag_stream.hip — streaming-floor probes for the 24 B/state + 1 B/flag pattern
// (diagnostics only; not part of the product library).  Build:
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/libdiag.so scripts/diag_stream.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kB = 256;

// mode 0: lane owns 4 states = 96 contiguous bytes (six 16-B loads, stride 96 B)
// mode 1: wave loads its 6 KB tile as six fully coalesced 1-KB instructions
// mode 2: mode 0 with non-temporal loads
template <int MODE>
__global__ __launch_bounds__(kB) void k_stream(const double* __restrict__ in, int64_t n_groups,
                                               uint32_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * kB;
    for (int64_t g = (int64_t)blockIdx.x * kB + threadIdx.x; g < n_groups; g += stride) {
        double acc = 0;
        if (MODE == 1) {
            const int lane = threadIdx.x & 63;
            const int64_t wbase = (g - lane) * 12;  // doubles; wave's tile = 64 * 12 doubles
            const double2* q = reinterpret_cast<const double2*>(in + wbase);
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const double2 t = q[k * 64 + lane];
                acc += t.x + t.y;
            }
        } else {
            const double2* q = reinterpret_cast<const double2*>(in + 12 * g);
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                double2 t;
                if (MODE == 2) {
                    t.x = __builtin_nontemporal_load(&q[k].x);
                    t.y = __builtin_nontemporal_load(&q[k].y);
                } else {
                    t = q[k];
                }
                acc += t.x + t.y;
            }
        }
        out[g] = acc > 1e300 ? 0u : 0x01010101u;
    }
}

extern "C" int diag_stream(int mode, const double* in, int64_t n_states, uint32_t* out, int blocks,
                           void* stream) {
    const int64_t groups = n_states / 4;
    hipStream_t s = (hipStream_t)stream;
    if (mode == 0) hipLaunchKernelGGL(k_stream<0>, dim3(blocks), dim3(kB), 0, s, in, groups, out);
    if (mode == 1) hipLaunchKernelGGL(k_stream<1>, dim3(blocks), dim3(kB), 0, s, in, groups, out);
    if (mode == 2) hipLaunchKernelGGL(k_stream<2>, dim3(blocks), dim3(kB), 0, s, in, groups, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

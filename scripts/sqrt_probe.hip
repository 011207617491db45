#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <random>
#include <vector>
#include <cstring>
__global__ void k(const double* a, double* b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { double x = a[3*i], y = a[3*i+1], z = a[3*i+2]; b[i] = sqrt((x * x + y * y) + z * z); }
}
int main() {
    const int n = 1 << 22;
    std::vector<double> a(3 * n), b(n);
    std::mt19937_64 r(1);
    std::uniform_real_distribution<double> u(-2.0, 2.0);
    for (auto& x : a) x = u(r) * (r() % 7 == 0 ? 1e-3 : 1.0);
    double *da, *db;
    hipMalloc(&da, 24 * (size_t)n); hipMalloc(&db, 8 * (size_t)n);
    hipMemcpy(da, a.data(), 24 * (size_t)n, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(da, db, n);
    hipMemcpy(b.data(), db, 8 * (size_t)n, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < n; ++i) { double x = a[3*i], y = a[3*i+1], z = a[3*i+2]; double c = std::sqrt((x * x + y * y) + z * z); if (std::memcmp(&c, &b[i], 8)) ++bad; }
    printf("sqrt mismatches: %ld of %d\n", bad, n);
    return 0;
}

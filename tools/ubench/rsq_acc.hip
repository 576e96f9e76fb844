// Dev microbenchmark: accuracy of the hardware fp64 reciprocal / rsq estimates on gfx950.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
__global__ void k(const double* x, double* rsq0, double* rsq1, double* rcp0, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double y = __builtin_amdgcn_rsq(v);
    rsq0[i] = y;
    y = y * fma(-0.5 * v * y, y, 1.5);
    rsq1[i] = y;
    rcp0[i] = __builtin_amdgcn_rcp(v);
}
int main() {
    const int n = 1 << 20;
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-30.0, 30.0);
    double* hx = new double[n];
    for (int i = 0; i < n; ++i) hx[i] = std::pow(10.0, u(g) / 3.0) * (1.0 + 1e-3 * (i % 997));
    double *dx, *a, *b, *c;
    (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&a, n * 8); (void)hipMalloc(&b, n * 8); (void)hipMalloc(&c, n * 8);
    (void)hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, a, b, c, n);
    double* ha = new double[n]; double* hb = new double[n]; double* hc = new double[n];
    (void)hipMemcpy(ha, a, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb, b, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hc, c, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double t = 1.0L / std::sqrt((long double)hx[i]);
        e0 = std::fmax(e0, (double)std::fabs((ha[i] - t) / t));
        e1 = std::fmax(e1, (double)std::fabs((hb[i] - t) / t));
        const long double r = 1.0L / (long double)hx[i];
        e2 = std::fmax(e2, (double)std::fabs((hc[i] - r) / r));
    }
    printf("v_rsq_f64 max rel err %.3e (2^%.1f); after 1 Newton %.3e; v_rcp_f64 max rel err %.3e (2^%.1f)\n", e0,
           std::log2(e0), e1, e2, std::log2(e2));
    return 0;
}

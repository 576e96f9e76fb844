// PMC calibration for roofline.traffic: FETCH_SIZE / WRITE_SIZE against a known byte count for the
// access widths lmpc_qp_kernel uses (8 B per lane, coalesced within a wave).  Buffers are 512 MiB,
// past the 256 MiB Infinity Cache, so every byte reaches the memory-side counters.
// And for roofline.executed: SQ_INSTS_VALU_FLOPS_FP64 / SQ_INSTS_VALU_MFMA_MOPS_F64 against known fp64
// flop counts -- fma64 (every lane), fma64_half (half the lanes under an exec mask) and mfma64
// (v_mfma_f64_16x16x4f64, 2048 flops each).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/pmc_cal tools/ubench/pmc_cal.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d out -- tools/ubench/pmc_cal   (and again with WRITE_SIZE)
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void read8(const double* __restrict__ a, size_t n, double* __restrict__ sink) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) sink[0] = s;  // never true: keeps the loads alive without a store stream
}

__global__ void write8(double* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.0;
}

constexpr int FMA_ITERS = 4096;  // per lane, 4 independent chains each
__global__ void fma64(double* __restrict__ sink, double a, double b, int half) {
    if (half && (threadIdx.x & 1)) return;
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    for (int i = 0; i < FMA_ITERS; ++i) {
        x0 = fma(x0, a, b);
        x1 = fma(x1, a, b);
        x2 = fma(x2, a, b);
        x3 = fma(x3, a, b);
    }
    const double s = x0 + x1 + x2 + x3;
    if (s == 12345.678) sink[0] = s;
}

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int MFMA_ITERS = 1024;
__global__ void mfma64(double* __restrict__ sink, double a) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    double x = a * threadIdx.x, y = a + threadIdx.x;
    for (int i = 0; i < MFMA_ITERS; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
    const double s = acc[0] + acc[1] + acc[2] + acc[3];
    if (s == 12345.678) sink[0] = s;
}

int main() {
    const size_t bytes = 512ull << 20, n = bytes / 8;
    double *a, *sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n, sink);
    const int waves = 1024;
    hipLaunchKernelGGL(fma64, dim3(waves), dim3(64), 0, 0, sink, 0.999, 1e-3, 0);
    hipLaunchKernelGGL(fma64, dim3(waves), dim3(64), 0, 0, sink, 0.999, 1e-3, 1);
    hipLaunchKernelGGL(mfma64, dim3(waves), dim3(64), 0, 0, sink, 0.5);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("pmc_cal: write8 and read8 each move %zu bytes (512 MiB)\n", bytes);
    printf("pmc_cal: fma64 %.6e flops (every lane), fma64 half %.6e flops, mfma64 %.6e flops\n",
           2.0 * 4 * FMA_ITERS * 64.0 * waves, 2.0 * 4 * FMA_ITERS * 32.0 * waves, 2048.0 * MFMA_ITERS * waves);
    (void)hipFree(a);
    (void)hipFree(sink);
    return 0;
}

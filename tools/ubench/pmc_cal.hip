// PMC calibration for roofline.traffic: FETCH_SIZE / WRITE_SIZE against a known byte count for the
// access widths lmpc_qp_kernel uses (8 B per lane, coalesced within a wave).  Buffers are 512 MiB,
// past the 256 MiB Infinity Cache, so every byte reaches the memory-side counters.
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

int main() {
    const size_t bytes = 512ull << 20, n = bytes / 8;
    double *a, *sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("pmc_cal: write8 and read8 each move %zu bytes (512 MiB)\n", bytes);
    (void)hipFree(a);
    (void)hipFree(sink);
    return 0;
}

// Dev microbenchmark: v_mfma_f64_16x16x4f64 issue / dependent latency on gfx950, and its operand layout.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(64) k(double* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-4;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double x[8];
    for (int q = 0; q < 8; ++q) x[q] = lane + q;
    const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 1
    for (int it = 0; it < 128; ++it) {
        if (MODE == 0) {  // dependent accumulator chain
#pragma unroll
            for (int j = 0; j < 8; ++j) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        } else if (MODE == 1) {  // 4 independent accumulators
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
            }
        } else if (MODE == 3) {  // dependent chain + 8 independent VALU fma per MFMA (does VALU overlap?)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
#pragma unroll
                for (int q = 0; q < 8; ++q) x[q] = fma(x[q], 1.0000001, 1e-9);
            }
        } else if (MODE == 4) {  // only the VALU part of MODE 3 (reference)
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int q = 0; q < 8; ++q) x[q] = fma(x[q], 1.0000001, 1e-9);
        } else if (MODE == 5) {  // 2 independent accumulators
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            }
        } else {  // result used as the next B operand (accumulator -> operand dependency)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
                b = c0[0] * 1e-3;
            }
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    d4 s = c0 + c1 + c2 + c3;
    double xs = 0.0;
    for (int q = 0; q < 8; ++q) xs += x[q];
    out[lane] = s[0] + s[1] + s[2] + s[3] + b + xs;
    if (lane == 0) cyc[0] = t1 - t0;
}

// layout probe: A[i][k] = 100 i + k, B[k][j] = (k == j) -> D = A[:, 0:4] restricted; print lane->element map
__global__ void layout(double* out) {
    const int l = threadIdx.x;
    const int ai = l & 15, ak = l >> 4;           // assumed A map: A[l&15][l>>4]
    const int bk = l >> 4, bj = l & 15;           // assumed B map: B[l>>4][l&15]
    const double a = 100.0 * ai + ak;
    const double b = (bk == bj) ? 1.0 : 0.0;
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}

int main() {
    double* out; unsigned long long* cyc;
    (void)hipMalloc(&out, 4096 * sizeof(double));
    (void)hipMalloc(&cyc, 8 * sizeof(unsigned long long));
    unsigned long long h;
    const char* nm[] = {"mfma f64 16x16x4 dependent acc", "mfma f64 16x16x4 4 independent", "mfma f64 acc->operand chain",
                        "dep mfma + 8 indep VALU fma each", "the 8 VALU fma alone (per MFMA slot)", "mfma 2 independent"};
    for (int m = 0; m < 6; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            if (m == 0) k<0><<<1, 64>>>(out, cyc);
            if (m == 1) k<1><<<1, 64>>>(out, cyc);
            if (m == 2) k<2><<<1, 64>>>(out, cyc);
            if (m == 3) k<3><<<1, 64>>>(out, cyc);
            if (m == 4) k<4><<<1, 64>>>(out, cyc);
            if (m == 5) k<5><<<1, 64>>>(out, cyc);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-34s %8.1f cycles per MFMA\n", nm[m], (double)h / (128.0 * 8.0));
    }
    layout<<<1, 64>>>(out);
    double hl[256];
    (void)hipMemcpy(hl, out, 256 * sizeof(double), hipMemcpyDeviceToHost);
    // D = A[:, 0:4] * I(4x16) -> D[i][j] = A[i][j] for j < 4 (=100 i + j), 0 for j >= 4
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            const int row = (l >> 4) + 4 * i, col = l & 15;  // guide: col = lane&15, row = (lane>>4) + 4*reg
            const double want = (col < 4) ? 100.0 * row + col : 0.0;
            if (hl[l * 4 + i] != want) ++bad;
        }
    printf("layout check (A[l&15][l>>4], B[l>>4][l&15], D row=(l>>4)+4i col=l&15): %d mismatches\n", bad);
    return 0;
}

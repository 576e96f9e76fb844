// Dev microbenchmark: one wave per CU, cycle costs of fp64 VALU / transcendental / LDS ops on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) double ldouble;

template <int MODE>
__global__ void __launch_bounds__(64) k(double* out, unsigned long long* cyc, double seed) {
    __shared__ double sm[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) sm[i] = 1.0 + 1e-9 * i;
    __syncthreads();
    ldouble* L = (ldouble*)sm;
    double a = seed + lane * 1e-3, b = 1.0000001, c = 1e-7;
    double x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3, x4 = a + 4, x5 = a + 5, x6 = a + 6, x7 = a + 7;
    int idx = lane;
    const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
        if (MODE == 0) {  // dependent fma chain, 8 per iteration
#pragma unroll
            for (int j = 0; j < 8; ++j) x0 = fma(x0, b, c);
        } else if (MODE == 1) {  // 8 independent fma chains
            x0 = fma(x0, b, c); x1 = fma(x1, b, c); x2 = fma(x2, b, c); x3 = fma(x3, b, c);
            x4 = fma(x4, b, c); x5 = fma(x5, b, c); x6 = fma(x6, b, c); x7 = fma(x7, b, c);
        } else if (MODE == 2) {  // dependent rsq chain, 8 per iteration
#pragma unroll
            for (int j = 0; j < 8; ++j) x0 = __builtin_amdgcn_rsq(x0 + 1.0);
        } else if (MODE == 3) {  // dependent LDS reads (pointer chase through an index), 8 per iteration
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const double v = L[idx];
                idx = ((int)v & 0) + ((idx + 1) & 1023);
                x0 += v;
            }
        } else if (MODE == 4) {  // dependent LDS write -> read round trip by another lane, 8 per iteration
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                L[lane] = x0;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
                x0 = L[(lane + 1) & 63] * b;
            }
        } else if (MODE == 5) {  // dependent mul chain
#pragma unroll
            for (int j = 0; j < 8; ++j) x0 = x0 * b;
        } else if (MODE == 6) {  // 8 independent chains on 16 lanes only (masked)
            if (lane < 16) {
                x0 = fma(x0, b, c); x1 = fma(x1, b, c); x2 = fma(x2, b, c); x3 = fma(x3, b, c);
                x4 = fma(x4, b, c); x5 = fma(x5, b, c); x6 = fma(x6, b, c); x7 = fma(x7, b, c);
            }
        } else if (MODE == 7) {  // dependent fp32 fma chain (reference)
            float y = (float)x0;
#pragma unroll
            for (int j = 0; j < 8; ++j) y = fmaf(y, (float)b, (float)c);
            x0 = y;
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * 64 + lane] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + idx;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double* out; unsigned long long* cyc;
    hipMalloc(&out, 64 * 64 * sizeof(double));
    hipMalloc(&cyc, 64 * sizeof(unsigned long long));
    const char* names[] = {"fma f64 dependent", "fma f64 8 independent", "rsq f64 dependent (+add)", "ds_read_b64 dependent",
                           "ds_write->ds_read other lane", "mul f64 dependent", "fma f64 8 indep, 16 lanes", "fma f32 dependent"};
    unsigned long long h[64];
    for (int m = 0; m < 8; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (m) {
                case 0: k<0><<<1, 64>>>(out, cyc, 1.0); break;
                case 1: k<1><<<1, 64>>>(out, cyc, 1.0); break;
                case 2: k<2><<<1, 64>>>(out, cyc, 1.0); break;
                case 3: k<3><<<1, 64>>>(out, cyc, 1.0); break;
                case 4: k<4><<<1, 64>>>(out, cyc, 1.0); break;
                case 5: k<5><<<1, 64>>>(out, cyc, 1.0); break;
                case 6: k<6><<<1, 64>>>(out, cyc, 1.0); break;
                case 7: k<7><<<1, 64>>>(out, cyc, 1.0); break;
            }
            hipDeviceSynchronize();
        }
        hipMemcpy(h, cyc, sizeof(unsigned long long), hipMemcpyDeviceToHost);
        printf("%-32s %8.1f cycles per op\n", names[m], (double)h[0] / (256.0 * 8.0));
    }
    return 0;
}

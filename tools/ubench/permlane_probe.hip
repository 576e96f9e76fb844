// Probe of the gfx950 cross-row swaps used by diag_inverse's tile_row (lmpc_dense_common.h):
//  (1) which source row each output of v_permlane16_swap / v_permlane32_swap holds;
//  (2) tile_row / tile_at on a tile produced by an MFMA and consumed at once (hazards), checked per lane;
//  (3) diag_inverse on an SPD tile: max |L^-1 M L^-T - I| (host check).
#include "../../legged_mpc_control_amd/csrc/lmpc_dense.hip"

#include <cmath>
#include <cstdio>

__global__ void probe(unsigned* out) {
    const unsigned x = threadIdx.x;  // lane id
    const auto s16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const auto s32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    out[0 * 64 + x] = s16[0];
    out[1 * 64 + x] = s16[1];
    out[2 * 64 + x] = s32[0];
    out[3 * 64 + x] = s32[1];
}

// tile X = A'B through one MFMA (A = lane-valued, B = identity-ish), then every row broadcast / element read at once
__global__ void rows_probe(double* out, double* el) {
    const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
    lmpc::d4 X = {0.0, 0.0, 0.0, 0.0};
    // A[m][k] (lane: m = lane&15, k = lane>>4) = 1 + m + 100k; B[k][n] = (k == 0 && n == ...) -> X[m][n] = sum_k A[k][m] B[k][n]
    const double a = 1.0 + c + 100.0 * g, b = 1.0 + 0.5 * c + 7.0 * g;
    X = MFMA64(a, b, X);
    double r[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) r[q] = lmpc::tile_row(X, q);
#pragma unroll
    for (int q = 0; q < 16; ++q) out[q * 64 + lane] = r[q];
    double e[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) e[q] = lmpc::tile_at(X, q, (q * 5) & 15);
    if (lane == 0)
        for (int q = 0; q < 16; ++q) el[q] = e[q];
}

__global__ void __launch_bounds__(64) diag_check(const double* Min, double* Wout) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
    const lmpc::DSmem S = lmpc::dcarve(sm, 10);
    lmpc::d4 M;
    for (int i = 0; i < 4; ++i) M[i] = Min[(4 * i + g) * 16 + c];
    const lmpc::DiagInv di = lmpc::diag_inverse(S.scr, M, 0x1f, lane);
    for (int i = 0; i < 4; ++i) Wout[(4 * i + g) * 16 + c] = di.uit[i];
}

int main() {
    unsigned* d;
    unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* nm[4] = {"pl16[0]", "pl16[1]", "pl32[0]", "pl32[1]"};
    for (int k = 0; k < 4; ++k) {
        printf("%s source row per row group:", nm[k]);
        for (int g = 0; g < 4; ++g) printf(" %u", h[k * 64 + 16 * g + 3] / 16);
        printf("\n");
    }
    // (2)
    double *dr, *de, hr[16 * 64], he[16];
    (void)hipMalloc(&dr, sizeof(hr));
    (void)hipMalloc(&de, sizeof(he));
    hipLaunchKernelGGL(rows_probe, dim3(1), dim3(64), 0, 0, dr, de);
    (void)hipMemcpy(hr, dr, sizeof(hr), hipMemcpyDeviceToHost);
    (void)hipMemcpy(he, de, sizeof(he), hipMemcpyDeviceToHost);
    double X[16][16];
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += (1.0 + m + 100.0 * k) * (1.0 + 0.5 * n + 7.0 * k);
            X[m][n] = s;
        }
    int bad = 0;
    for (int q = 0; q < 16; ++q)
        for (int l = 0; l < 64; ++l)
            if (hr[q * 64 + l] != X[q][l & 15]) {
                if (bad < 8) printf("tile_row(%d) lane %d: %g expected %g\n", q, l, hr[q * 64 + l], X[q][l & 15]);
                ++bad;
            }
    for (int q = 0; q < 16; ++q)
        if (he[q] != X[q][(q * 5) & 15]) {
            if (bad < 16) printf("tile_at(%d,%d): %g expected %g\n", q, (q * 5) & 15, he[q], X[q][(q * 5) & 15]);
            ++bad;
        }
    printf("tile_row/tile_at after an MFMA: %d mismatches\n", bad);
    // (3)
    double Mh[256], Wh[256];
    for (int r = 0; r < 16; ++r)
        for (int cc = 0; cc < 16; ++cc)
            Mh[r * 16 + cc] = (r == 15 || cc == 15) ? (r == cc ? 1.0 : 0.0) : (r == cc ? 4.0 : 0.0) + 0.1 / (r + cc + 1);
    double *dM, *dW;
    (void)hipMalloc(&dM, sizeof(Mh));
    (void)hipMalloc(&dW, sizeof(Wh));
    (void)hipMemcpy(dM, Mh, sizeof(Mh), hipMemcpyHostToDevice);
    const size_t lds = lmpc::dense_lds_bytes(10);
    (void)hipFuncSetAttribute((const void*)diag_check, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(diag_check, dim3(1), dim3(64), lds, 0, dM, dW);
    (void)hipMemcpy(Wh, dW, sizeof(Wh), hipMemcpyDeviceToHost);
    double worst = 0.0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0.0;  // (W M W')_ij
            for (int a = 0; a < 16; ++a)
                for (int b = 0; b < 16; ++b) s += Wh[i * 16 + a] * Mh[a * 16 + b] * Wh[j * 16 + b];
            worst = fmax(worst, fabs(s - (i == j ? 1.0 : 0.0)));
        }
    printf("diag_inverse: max |W M W' - I| = %.3e (W[0][0] %.6f W[5][3] %.6f)\n", worst, Wh[0], Wh[5 * 16 + 3]);
    return 0;
}

// Probe of the gfx950 cross-row swaps used by the dense path's group_sum4 (lmpc_dense_common.h):
//  (1) which source row each output of v_permlane16_swap / v_permlane32_swap holds;
//  (2) group_sum4 / row_sum4 (the solves' cross-lane sums), checked per lane against the host;
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

// group_sum4 and row_sum4 (lmpc_dense_common.h) on lane-valued data, every lane checked on the host
__global__ void sums_probe(double* out) {
    const int lane = threadIdx.x;
    const double v = 1.0 + lane + 0.001 * lane * lane;
    out[lane] = lmpc::group_sum4(v);
    double p[4], r[4];
    for (int k = 0; k < 4; ++k) p[k] = v * (k + 1) + k;
    lmpc::row_sum4(p, r);
    for (int k = 0; k < 4; ++k) out[64 * (k + 1) + lane] = r[k];
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
    double *ds, hs[5 * 64];
    (void)hipMalloc(&ds, sizeof(hs));
    hipLaunchKernelGGL(sums_probe, dim3(1), dim3(64), 0, 0, ds);
    (void)hipMemcpy(hs, ds, sizeof(hs), hipMemcpyDeviceToHost);
    double worst = 0.0;
    for (int l = 0; l < 64; ++l) {
        double gs = 0.0;
        for (int g = 0; g < 4; ++g) {
            const int m = 16 * g + (l & 15);
            gs += 1.0 + m + 0.001 * m * m;
        }
        worst = fmax(worst, fabs(hs[l] - gs) / gs);
        for (int k = 0; k < 4; ++k) {
            double rs = 0.0;
            for (int c = 0; c < 16; ++c) {
                const int m = 16 * (l >> 4) + c;
                rs += (1.0 + m + 0.001 * m * m) * (k + 1) + k;
            }
            worst = fmax(worst, fabs(hs[64 * (k + 1) + l] - rs) / rs);
        }
    }
    printf("group_sum4 / row_sum4: max relative error %.3e over all lanes\n", worst);
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
    worst = 0.0;
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

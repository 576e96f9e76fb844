// Dev microbenchmark: the dense path's 16x16 diagonal-tile inverse (lmpc::diag_inverse) alone on
// one wave, i.e. without the register pressure of the full kernel.  Build from the repo root:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I legged_mpc_control_amd/csrc \
//         -o tools/ubench/diag tools/ubench/diag.hip
#include "../../legged_mpc_control_amd/csrc/lmpc_dense.hip"

#include <cstdio>

__global__ void __launch_bounds__(64) diag_probe(double* out, unsigned long long* cyc, int amask) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int lane = threadIdx.x;
    const lmpc::DSmem S = lmpc::dcarve(sm, 10);
    const int lc = lane & 15, lr = lane >> 4;
    lmpc::d4 M, Ui, UiT;
    for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        // SPD: 4 I + 0.1 (r + c + 1)^-1 (Hilbert-like), identity on the padding slot
        M[i] = (r == 15 || lc == 15) ? (r == lc ? 1.0 : 0.0) : (r == lc ? 4.0 : 0.0) + 0.1 / (r + lc + 1);
    }
    double chk = 0.0;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 64; ++it) {
        const lmpc::DiagInv di = lmpc::diag_inverse(S.scr, M, amask, lane);
        Ui = di.ui;
        UiT = di.uit;
        chk += Ui[0] + UiT[3];
        M[0] += 1e-300 * chk;  // dependency between iterations
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[lane] = chk;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    double* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&cyc, 8);
    const size_t lds = lmpc::dense_lds_bytes(10);
    (void)hipFuncSetAttribute((const void*)diag_probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int mask : {0x1f, 0x3, 0x1}) {
        unsigned long long h = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(diag_probe, dim3(1), dim3(64), lds, 0, out, cyc, mask);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("diag_inverse, block mask 0x%02x: %8.0f cycles per call\n", mask, (double)h / 64.0);
    }
    return 0;
}

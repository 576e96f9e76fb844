// C++ host over the multi-device C-ABI (include/lmpc/lmpc_multi.h): no PyTorch.  Solves a synthetic
// config-2 batch (Go1 trot, H = 10) generated on every device from (seed, global index), gathered to the
// root by RCCL, and prints one line per QP block so tests/test_multi.py can compare it with the
// single-device path:  "<devices> <batch> <ms> <status0> <iters0> <sum of all GRFs, %.17g>".
//   multi_test <n_devices> <batch> <seed>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lmpc/lmpc_multi.h"

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 1;
    const int batch = argc > 2 ? std::atoi(argv[2]) : 1024;
    const unsigned long long seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 20261017ull;
    const int H = 10;
    lmpc_params p;
    lmpc_params_go1(&p);
    lmpc_synth_cfg cfg;
    lmpc_synth_cfg_go1(&cfg);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = i;
    lmpc_multi* m = nullptr;
    int rc = lmpc_multi_create(&p, H, devs.data(), n, &m);
    if (rc != LMPC_OK) {
        std::fprintf(stderr, "lmpc_multi_create: %d\n", rc);
        return 1;
    }
    double* d_grf = nullptr;
    int32_t *d_st = nullptr, *d_it = nullptr;
    if (hipSetDevice(devs[0]) != hipSuccess || hipMalloc(&d_grf, (size_t)batch * 12 * H * sizeof(double)) != hipSuccess ||
        hipMalloc(&d_st, batch * sizeof(int32_t)) != hipSuccess || hipMalloc(&d_it, batch * sizeof(int32_t)) != hipSuccess)
        return 2;
    rc = lmpc_multi_solve_synth_device(m, &cfg, seed, 0, batch, -1.0, d_grf, d_st, d_it);  // warm-up
    const auto t0 = std::chrono::steady_clock::now();
    if (rc == LMPC_OK) rc = lmpc_multi_solve_synth_device(m, &cfg, seed, 0, batch, -1.0, d_grf, d_st, d_it);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc != LMPC_OK) {
        std::fprintf(stderr, "lmpc_multi_solve_synth_device: %d\n", rc);
        return 3;
    }
    std::vector<double> grf((size_t)batch * 12 * H);
    std::vector<int32_t> st(batch), it(batch);
    if (hipMemcpy(grf.data(), d_grf, grf.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(st.data(), d_st, batch * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(it.data(), d_it, batch * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return 4;
    int bad = 0;
    for (int b = 0; b < batch; ++b) bad += st[b] != 0;
    double sum = 0.0;
    for (double v : grf) sum += v;
    std::printf("%d %d %.3f %d %d %.17g\n", n, batch, ms, bad, it[0], sum);
    (void)hipFree(d_grf);
    (void)hipFree(d_st);
    (void)hipFree(d_it);
    lmpc_multi_destroy(m);
    return 0;
}

// lmpc_wbc.hip -- WBC task formulation (wbc.cpp:102-259) into hierarchical-QP records of the WBC layout
// (include/lmpc/lmpc_hoqp.h, lmpc_hoqp_dims_wbc), on the host (one robot) and on the device (one wavefront per
// robot).  One restatement, compiled for both, so the two agree bitwise (pure copies and sign flips).
#include <hip/hip_runtime.h>

#include "lmpc/lmpc_hoqp.h"

namespace lmpc {
namespace {

constexpr int WN = 42, NQ = 18, NF = 12;        // x = [qdd (18), F (12), tau (12)] (wbc.h:18)
constexpr int M0 = 30, S0 = 44, M1 = 18, M2 = 12;
constexpr int OFF_A0 = 0, OFF_B0 = M0 * WN, OFF_D0 = OFF_B0 + M0, OFF_F0 = OFF_D0 + S0 * WN;
constexpr int OFF_A1 = OFF_F0 + S0, OFF_B1 = OFF_A1 + M1 * WN, OFF_A2 = OFF_B1 + M1, OFF_B2 = OFF_A2 + M2 * WN;
constexpr int WBC_REC = OFF_B2 + M2;
static_assert(WBC_REC == 4472, "WBC record layout");
static_assert(sizeof(lmpc_wbc_input) == 4848, "lmpc_wbc_input layout (legged_mpc_control_amd/_native.py)");

// Every entry of the record; entries are independent, so lanes take them in any order (stride `step`).
__host__ __device__ inline void wbc_fill(const lmpc_wbc_input& in, double* rec, int first, int step) {
    // stance / swing orderings (wbc.cpp:140-147, :156-158, :169-171, :236-244)
    int stance[4], swing[4], ns = 0, nw = 0;
    for (int i = 0; i < 4; ++i) {
        if (in.contact[i]) stance[ns++] = i;
        else swing[nw++] = i;
    }
    for (int e = first; e < WBC_REC; e += step) {
        double v = 0.0;
        if (e < OFF_B0) {  // level 0 equalities
            const int r = e / WN, c = e % WN;
            if (r < NQ) {  // floating-base EoM [M, -J', -S'] (wbc.cpp:102-115)
                if (c < NQ) v = in.M[r * NQ + c];
                else if (c < NQ + NF) v = -in.J[(c - NQ) * NQ + r];
                else v = (r >= 6 && c - NQ - NF == r - 6) ? -1.0 : 0.0;
            } else if (r < NQ + 3 * nw) {  // swing feet's forces = 0 (friction cone eq, wbc.cpp:153-158)
                const int j = (r - NQ) / 3, a = (r - NQ) % 3;
                v = (c == NQ + 3 * swing[j] + a) ? 1.0 : 0.0;
            } else {  // stance feet: J qdd = -dJ v (no-contact motion, wbc.cpp:133-149)
                const int j = (r - NQ - 3 * nw) / 3, a = (r - NQ - 3 * nw) % 3;
                v = c < NQ ? in.J[(3 * stance[j] + a) * NQ + c] : 0.0;
            }
        } else if (e < OFF_D0) {
            const int r = e - OFF_B0;
            if (r < NQ) v = -in.nle[r];
            else if (r < NQ + 3 * nw) v = 0.0;
            else {
                const int j = (r - NQ - 3 * nw) / 3, a = (r - NQ - 3 * nw) % 3;
                v = -in.dJv[3 * stance[j] + a];
            }
        } else if (e < OFF_F0) {  // level 0 inequalities
            const int r = (e - OFF_D0) / WN, c = (e - OFF_D0) % WN;
            if (r < 12) v = (c == NQ + NF + r) ? 1.0 : 0.0;               // tau <= limits (wbc.cpp:117-131)
            else if (r < 24) v = (c == NQ + NF + r - 12) ? -1.0 : 0.0;    // -tau <= limits
            else if (r < 24 + 5 * ns) {                                   // pyramid rows (wbc.cpp:162-171)
                const int j = (r - 24) / 5, k = (r - 24) % 5, col = c - NQ - 3 * stance[j];
                // rows (0,0,-1), (1,0,-mu), (-1,0,-mu), (0,1,-mu), (0,-1,-mu) on (fx, fy, fz)
                if (col == 0) v = k == 1 ? 1.0 : k == 2 ? -1.0 : 0.0;
                else if (col == 1) v = k == 3 ? 1.0 : k == 4 ? -1.0 : 0.0;
                else if (col == 2) v = k == 0 ? -1.0 : -in.mu;
            }
        } else if (e < OFF_A1) {
            const int r = e - OFF_F0;
            v = r < 24 ? in.torque_limits[r % 3] : 0.0;
        } else if (e < OFF_B1) {  // level 1: base acceleration, swing feet
            const int r = (e - OFF_A1) / WN, c = (e - OFF_A1) % WN;
            if (r < 6) v = (c == r) ? 1.0 : 0.0;
            else if (r < 6 + 3 * nw) {
                const int j = (r - 6) / 3, a = (r - 6) % 3;
                v = c < NQ ? in.J[(3 * swing[j] + a) * NQ + c] : 0.0;
            }
        } else if (e < OFF_A2) {
            const int r = e - OFF_B1;
            if (r < 6) v = in.base_accel[r];
            else if (r < 6 + 3 * nw) {
                const int j = (r - 6) / 3, a = (r - 6) % 3;
                v = in.swing_acc[3 * swing[j] + a] - in.dJv[3 * swing[j] + a];
            }
        } else if (e < OFF_B2) {  // level 2: contact forces (wbc.cpp:248-259)
            const int r = (e - OFF_A2) / WN, c = (e - OFF_A2) % WN;
            v = (c == NQ + r) ? 1.0 : 0.0;
        } else {
            v = in.forces_des[e - OFF_B2];
        }
        rec[e] = v;
    }
}

__global__ void __launch_bounds__(256) lmpc_wbc_tasks_kernel(const lmpc_wbc_input* __restrict__ in, int batch,
                                                             double* __restrict__ rec) {
    const int robot = blockIdx.x * 4 + (threadIdx.x >> 6);  // one wavefront per robot, four per block
    if (robot >= batch) return;
    wbc_fill(in[robot], rec + (int64_t)robot * WBC_REC, threadIdx.x & 63, 64);
}

}  // namespace
}  // namespace lmpc

extern "C" int lmpc_wbc_tasks(const lmpc_wbc_input* in, double* record) {
    if (!in || !record) return LMPC_ERR_ARG;
    lmpc::wbc_fill(*in, record, 0, 1);
    return LMPC_OK;
}

extern "C" int lmpc_wbc_tasks_device(const lmpc_wbc_input* d_in, int batch, double* d_records, void* stream) {
    if (batch < 0 || (batch > 0 && (!d_in || !d_records))) return LMPC_ERR_ARG;
    if (batch == 0) return LMPC_OK;
    hipLaunchKernelGGL(lmpc::lmpc_wbc_tasks_kernel, dim3((batch + 3) / 4), dim3(256), 0, (hipStream_t)stream, d_in,
                       batch, d_records);
    return hipGetLastError() == hipSuccess ? LMPC_OK : LMPC_ERR_LAUNCH;
}

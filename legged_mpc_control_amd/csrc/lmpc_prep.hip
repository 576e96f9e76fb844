// lmpc_prep.hip -- the step before the QP, on the device.
//
//   lmpc_records_kernel   command -> record [x0 | R | feet | x_ref(H)] + contact schedule [H][4]
//                         (calc_mpc_reference ConvexQPSolver.cpp:256-276, update_bound_constraints
//                         :329-346, predict_contact_state LeggedContactFSM.cpp:280-294)
//   lmpc_synth_kernel     synthetic commands from (seed, global index)
//   lmpc_normals_kernel   synthetic terrain normals (config 4)
//   lmpc_torque_kernel    the step after the QP: GRF -> joint torque (BaseInterface.cpp:451-459, 8f-2)
//
// All three are HBM-write-bound element maps: one thread per output element (records) or per
// instance (generators), grid-stride, consecutive threads -> consecutive addresses.  The
// arithmetic is lmpc_common.h, shared with the host so that the expansion is bit-identical.
#include <hip/hip_runtime.h>

#include "lmpc/lmpc.h"
#include "lmpc_common.h"

namespace lmpc {

__global__ void __launch_bounds__(256) lmpc_records_kernel(const lmpc_command* __restrict__ cmd, int batch, int H,
                                                           double dt, double* __restrict__ rec,
                                                           uint8_t* __restrict__ contact) {
    const int RL = LMPC_REC_XREF + 12 * H;
    const size_t nrec = (size_t)batch * RL, ncon = (size_t)batch * 4 * H;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < nrec + ncon; e += stride) {
        if (e < nrec) {
            const size_t b = e / RL;
            rec[e] = lmpc_common::record_element(cmd[b].state, dt, (int)(e - b * RL));
        } else {
            const size_t c = e - nrec, b = c / (4 * H);
            const int k = (int)(c - b * 4 * H);
            contact[c] = lmpc_common::contact_element(cmd[b], dt, k >> 2, k & 3);
        }
    }
}

__global__ void __launch_bounds__(256) lmpc_synth_kernel(lmpc_synth_cfg cfg, uint64_t seed, int64_t first, int count,
                                                         lmpc_command* __restrict__ cmd) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= count) return;
    lmpc_command c;
    lmpc_common::synth_command(cfg, seed, (uint64_t)(first + b), c);
    cmd[b] = c;
}

__global__ void __launch_bounds__(256) lmpc_normals_kernel(uint64_t seed, int64_t first, int count, double theta_max,
                                                           double* __restrict__ normals) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= count) return;
    double n[12];
    lmpc_common::synth_normals(seed, (uint64_t)(first + b), theta_max, n);
#pragma unroll
    for (int k = 0; k < 12; ++k) normals[(size_t)b * 12 + k] = n[k];
}

// one thread per (instance, leg): tau = -J'(R'u0), BaseInterface.cpp:451-459
__global__ void __launch_bounds__(256) lmpc_torque_kernel(lmpc_leg_kin kin, const double* __restrict__ rec,
                                                          const double* __restrict__ joint_pos,
                                                          const double* __restrict__ grf, int batch, int H,
                                                          double* __restrict__ tau) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * batch) return;
    const int b = t >> 2, leg = t & 3;
    const double* R = rec + (size_t)b * (LMPC_REC_XREF + 12 * H) + LMPC_REC_ROT;
    double rot[9], q[3], f[3], out[3];
#pragma unroll
    for (int e = 0; e < 9; ++e) rot[e] = R[e];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        q[c] = joint_pos[(size_t)b * 12 + 3 * leg + c];
        f[c] = grf[(size_t)b * 12 * H + 3 * leg + c];  // u_0
    }
    lmpc_common::leg_torque(kin.rho_fix[leg], kin.rho_opt[leg], rot, q, f, out);
#pragma unroll
    for (int c = 0; c < 3; ++c) tau[(size_t)b * 12 + 3 * leg + c] = out[c];
}

hipError_t launch_torque(const lmpc_leg_kin& kin, const double* rec, const double* joint_pos, const double* grf,
                         int batch, int H, double* tau, hipStream_t stream) {
    hipLaunchKernelGGL(lmpc_torque_kernel, dim3((4 * batch + 255) / 256), dim3(256), 0, stream, kin, rec, joint_pos,
                       grf, batch, H, tau);
    return hipGetLastError();
}

hipError_t launch_records(const lmpc_command* cmd, int batch, int H, double dt, double* rec, uint8_t* contact,
                          hipStream_t stream) {
    const size_t n = (size_t)batch * (LMPC_REC_XREF + 16 * H);
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(lmpc_records_kernel, dim3(blocks), dim3(256), 0, stream, cmd, batch, H, dt, rec, contact);
    return hipGetLastError();
}

hipError_t launch_synth(const lmpc_synth_cfg& cfg, uint64_t seed, int64_t first, int count, lmpc_command* cmd,
                        hipStream_t stream) {
    hipLaunchKernelGGL(lmpc_synth_kernel, dim3((count + 255) / 256), dim3(256), 0, stream, cfg, seed, first, count,
                       cmd);
    return hipGetLastError();
}

hipError_t launch_normals(uint64_t seed, int64_t first, int count, double theta_max, double* normals,
                          hipStream_t stream) {
    hipLaunchKernelGGL(lmpc_normals_kernel, dim3((count + 255) / 256), dim3(256), 0, stream, seed, first, count,
                       theta_max, normals);
    return hipGetLastError();
}

}  // namespace lmpc

// lmpc_fused.hip -- the dense path and the Riccati kernel as one launch (lmpc_dense_lq_kernel), for batches of at
// most one QP per SIMD.  Its own translation unit so that it keeps the dense kernel's machine scheduler (build.py
// SCHED_FLAGS: max-ilp here and in lmpc_dense.hip, iterative-ilp in lmpc_lq.hip); the two bodies are
// lmpc_dense_kernel.h's dense_body and lmpc_lq_kernel.h's lq_body, compiled with the same floating-point contract
// as their own kernels, so the fused launch gives every QP the bits the two launches give it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

// The product build only: the diagnostic and test-variant builds (stamps, certificate residuals, re-injected bugs,
// debug dumps) keep the two launches, so their hooks and their bugs stay in one translation unit each
#if !defined(LMPC_STAMPS) && !defined(LMPC_KKT_DIAG) && !defined(LMPC_BUG_ZA) && !defined(LMPC_BUG_YAW) && \
    !defined(LMPC_KKT_OFF) && !defined(LMPC_LQ_DEBUG) && !defined(LMPC_NO_FUSED) && !defined(LMPC_REFINE_DIAG)
#define LMPC_FUSED 1
#include "lmpc_dense_kernel.h"
#include "lmpc_lq_kernel.h"
#else
#define LMPC_FUSED 0
#endif

namespace lmpc {

#if LMPC_FUSED
// The dense path and the Riccati kernel in one launch, for batches of at most one QP per SIMD (config 2: B = 1024
// on 256 CUs), where both run one wave per SIMD anyway: the dense solve of each QP, then -- in the same wave, for
// the QPs it leaves -- the lone-wave Riccati solve.  The same two solves as the two launches (bit for bit), without
// the second launch and its dispatch of a workgroup per QP that only tests the hand-over flag (~4 us + the gap
// between the launches, ~5 % of config 2's step).
template <bool TERRAIN>
__global__ void __launch_bounds__(64, 1) lmpc_dense_lq_kernel(const DevParams prm, const double* __restrict__ rec,
                                                              const uint8_t* __restrict__ contact,
                                                              const double* __restrict__ normals, int batch,
                                                              double* __restrict__ grf, int32_t* __restrict__ status,
                                                              int32_t* __restrict__ iters, uint8_t* __restrict__ done) {
    if (!dense_body<TERRAIN>(prm, rec, contact, normals, batch, grf, status, iters, done))
        lq_body<1, TERRAIN, 1>(prm, rec, contact, normals, batch, grf, status, iters, done, true);
}
template __global__ void lmpc_dense_lq_kernel<false>(const DevParams, const double*, const uint8_t*, const double*,
                                                     int, double*, int32_t*, int32_t*, uint8_t*);
template __global__ void lmpc_dense_lq_kernel<true>(const DevParams, const double*, const uint8_t*, const double*,
                                                    int, double*, int32_t*, int32_t*, uint8_t*);
#endif

// One launch for the dense path (interior point) and the Riccati solves it leaves, where both would run one wave per
// SIMD (batch <= 4 x CUs, H <= 16): lmpc_dense_lq_kernel.  hipErrorNotSupported where this build has no fused kernel
// (diagnostic builds) or the batch does not qualify: the caller then launches the two kernels.
hipError_t launch_dense_lq(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                           int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream) {
#if LMPC_FUSED
    if (4 * prm.H > 64 || batch > 4 * prm.cus) return hipErrorNotSupported;
    const size_t lds = std::max(dense_lds_bytes(prm.H), lq_lds_bytes(prm.H));
    const dim3 grid(batch), block(LMPC_WAVE);
    if (normals) {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_lq_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_lq_kernel<true>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_lq_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_lq_kernel<false>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    }
    return hipGetLastError();
#else
    (void)prm, (void)rec, (void)contact, (void)normals, (void)batch, (void)grf, (void)status, (void)iters, (void)done;
    (void)stream;
    return hipErrorNotSupported;
#endif
}

}  // namespace lmpc

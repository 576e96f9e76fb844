// lmpc_lq.hip -- the LDS-resident Riccati kernel (lmpc_lq_kernel): its instances, the host launcher and the
// diagnostic hooks.  The per-QP solve (lq_body) and the algorithm are in lmpc_lq_kernel.h; the fused dense +
// Riccati launch in lmpc_fused.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

namespace lmpc {

#ifdef LMPC_STAMPS
constexpr int LQ_STAMP_QPS = 4096;
constexpr int LQ_STAMP_N = 16;
__device__ unsigned long long lmpc_lq_stamps[LQ_STAMP_QPS][LQ_STAMP_N];
#define LQ_STAMP_DECL unsigned long long _lq_acc[LQ_STAMP_N] = {}; unsigned long long _lq_t0 = __builtin_readcyclecounter();
#define LQ_STAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _lq_acc[i] += _t - _lq_t0; _lq_t0 = _t; } while (0)
#define LQ_STAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < LQ_STAMP_QPS) for (int _i = 0; _i < LQ_STAMP_N; ++_i) lmpc_lq_stamps[qp][_i] = _lq_acc[_i]; } while (0)
#define LQ_MARK(v) const unsigned long long v = __builtin_readcyclecounter()
#define LQ_ADD_SINCE(i, v) do { _lq_acc[i] += __builtin_readcyclecounter() - (v); } while (0)
#else
#define LQ_MARK(v) do {} while (0)
#define LQ_ADD_SINCE(i, v) do {} while (0)
#define LQ_STAMP_DECL
#define LQ_STAMP(i) do {} while (0)
#define LQ_STAMP_FLUSH(qp) do {} while (0)
#endif

#ifdef LMPC_KKT_DIAG
// diagnostic build (tools/kkt_diag.py): per QP, at its last settled polish round, the stationarity residual / gscale,
// the dynamics residual / state scale, gscale and the state scale
__device__ double lmpc_kkt_diag[LMPC_KKT_DIAG_QPS][4];
extern "C" int lmpc_debug_kkt_lq(double* out, int nqp) {
    if (nqp > LMPC_KKT_DIAG_QPS) nqp = LMPC_KKT_DIAG_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_kkt_diag), (size_t)nqp * 4 * sizeof(double)) == hipSuccess ? nqp : -1;
}
extern "C" int lmpc_debug_kkt_lq_clear(void) {
    static double zeros[LMPC_KKT_DIAG_QPS * 4];
    return hipMemcpyToSymbol(HIP_SYMBOL(lmpc_kkt_diag), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LMPC_LQ_DEBUG
__device__ double lmpc_lq_dbg[8192];
__device__ double lmpc_lq_dbg_u[384];
__device__ double lmpc_lq_dbg2[8192];
extern "C" int lmpc_debug_lq_dump(double* lds, double* u, double* lds2) {
    return (hipMemcpyFromSymbol(lds, HIP_SYMBOL(lmpc_lq_dbg), sizeof(double) * 8192) == hipSuccess &&
            hipMemcpyFromSymbol(lds2, HIP_SYMBOL(lmpc_lq_dbg2), sizeof(double) * 8192) == hipSuccess &&
            hipMemcpyFromSymbol(u, HIP_SYMBOL(lmpc_lq_dbg_u), sizeof(double) * 384) == hipSuccess) ? 0 : -1;
}
#endif

}  // namespace lmpc

#include "lmpc_lq_kernel.h"

namespace lmpc {

template <int LS, bool TERRAIN, int WPE>
__global__ void __launch_bounds__(64, WPE) lmpc_lq_kernel(const DevParams prm, const double* __restrict__ rec,
                                                          const uint8_t* __restrict__ contact,
                                                          const double* __restrict__ normals, int batch,
                                                          double* __restrict__ grf, int32_t* __restrict__ status,
                                                          int32_t* __restrict__ iters,
                                                          const uint8_t* __restrict__ dense_done) {
    lq_body<LS, TERRAIN, WPE>(prm, rec, contact, normals, batch, grf, status, iters, dense_done, false);
}


#define LMPC_LQ_INST(LS_, T_, W_)                                                                                    \
    template __global__ void lmpc_lq_kernel<LS_, T_, W_>(const DevParams, const double*, const uint8_t*, const double*, \
                                                     int, double*, int32_t*, int32_t*, const uint8_t*);
LMPC_LQ_INST(1, false, 1)
LMPC_LQ_INST(1, false, 2)
LMPC_LQ_INST(2, false, 1)
LMPC_LQ_INST(1, true, 1)
LMPC_LQ_INST(1, true, 2)
#ifdef LMPC_AB_W3  // diagnostic variant: three waves per SIMD (168 registers)
LMPC_LQ_INST(1, false, 3)
LMPC_LQ_INST(1, true, 3)
#endif
LMPC_LQ_INST(2, true, 1)
LMPC_LQ_INST(2, false, 2)
LMPC_LQ_INST(2, true, 2)
#undef LMPC_LQ_INST

template <int LS, bool TERRAIN, int WPE>
static void launch_lq_variant(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                              int batch, double* grf, int32_t* status, int32_t* iters, const uint8_t* done,
                              hipStream_t stream) {
    const size_t lds = lq_lds_bytes(prm.H);
    (void)hipFuncSetAttribute((const void*)lmpc_lq_kernel<LS, TERRAIN, WPE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lmpc_lq_kernel<LS, TERRAIN, WPE>), dim3(batch), dim3(LMPC_WAVE), lds, stream, prm, rec,
                       contact, normals, batch, grf, status, iters, done);
}

// Host-side launcher (lmpc_capi.cpp): cold solves of every QP the dense kernel did not take.  Two waves per SIMD
// only where the batch has more QPs than the device has SIMDs and more than four fit a CU's LDS (up to one QP per
// SIMD the lone-wave instance, free of spills, is faster, and the two-wave one would let the dispatcher stack two
// QPs on one SIMD while others idle).  At two leg-steps per lane (H > 16) the two-wave instance spills 276 B/lane:
// where six or more QPs fit a CU's LDS (H <= 21) the waves it adds hide more than that costs -- config 3 (H = 20,
// 8192 QPs) 3.667 -> 3.454 ms -- but at five per CU (H = 22..26) it is 8 % slower than the lone wave (round 6,
// profiles/r06/ls2w2/).  At H = 30 four QPs fill the LDS.  Same arithmetic: the choice never changes a result bit.
hipError_t launch_lq(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals, int batch,
                     double* grf, int32_t* status, int32_t* iters, const uint8_t* done, hipStream_t stream) {
    const bool two = 4 * prm.H > 64;
#ifdef LMPC_AB_NO_W2  // diagnostic variant (tools/ab_bench.sh): the lone-wave instance only
    const bool w2 = false;
#else
    const bool w2 = (two ? 6 : 5) * lq_lds_bytes(prm.H) <= LMPC_CU_LDS_BYTES && batch > 4 * prm.cus;
#endif
#define LMPC_LQ_LAUNCH(LS_, T_, W_) \
    launch_lq_variant<LS_, T_, W_>(prm, rec, contact, normals, batch, grf, status, iters, done, stream)
    if (normals) {
        if (two) w2 ? LMPC_LQ_LAUNCH(2, true, 2) : LMPC_LQ_LAUNCH(2, true, 1);
#ifdef LMPC_AB_W3
        else w2 ? LMPC_LQ_LAUNCH(1, true, 3) : LMPC_LQ_LAUNCH(1, true, 1);
#else
        else w2 ? LMPC_LQ_LAUNCH(1, true, 2) : LMPC_LQ_LAUNCH(1, true, 1);
#endif
    } else {
        if (two) w2 ? LMPC_LQ_LAUNCH(2, false, 2) : LMPC_LQ_LAUNCH(2, false, 1);
        else w2 ? LMPC_LQ_LAUNCH(1, false, 2) : LMPC_LQ_LAUNCH(1, false, 1);
    }
#undef LMPC_LQ_LAUNCH
    return hipGetLastError();
}

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_lq_stamps(unsigned long long* out, int nqp) {
    if (nqp > LQ_STAMP_QPS) nqp = LQ_STAMP_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_lq_stamps), (size_t)nqp * LQ_STAMP_N * sizeof(unsigned long long)) ==
                   hipSuccess ? nqp : -1;
}
#endif

}  // namespace lmpc

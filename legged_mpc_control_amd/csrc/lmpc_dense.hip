// lmpc_dense.hip -- the condensed dense path of the batched GRF QP (gfx950), one wavefront per QP.
//
// For QPs with at most 20 stance leg-steps (every Go1 trot at H=10: 2 stance legs x 10 steps) the
// states are eliminated once per QP and the interior point / polish iterate on the condensed QP
//     min 1/2 u'Hu + g'u   s.t. per stance leg-step: friction pyramid + f_max bound,
// u = the stance forces only (swing leg-steps are exactly zero, as in the Riccati path).
//
// Condensation (once per QP, ConvexQPSolver.cpp:198-313 restated in condensed form):
//   free response  c_{m+1} = A_m c_m - g dt e11,  c_0 = x0
//   adjoint        mu_m = Q (c_m - xref_{m-1}) + A_m' mu_{m+1}          -> g_i = B' mu_{i+1}
//   cost-to-go     P~_H = Q,  P~_m = Q + A_m' P~_{m+1} A_m              (fp64 MFMA, 12x12)
//   Hessian        H[i][j] = B' (A_j ... A_{i+1})' P~_{j+1} B  (i <= j), + R on the diagonal blocks,
//                  one column per lane: L = P~_{j+1} B e_c, then L <- A_{i+1}' L down the steps.
// Variables are laid out 5 leg-steps (15 variables + 1 padding slot) per 16-wide tile, so every
// 3x3 leg block sits inside one tile and N <= 64 fits 4x4 tiles.  H is kept in LDS as its upper
// tiles in the MFMA accumulator layout (lane l, register i <-> row (l>>4)+4i, column l&15).
//
// Newton system (H + C'WC) u = -(g + C'W(s-b)) (IPM) or T'HT y = -T'(H up + g) (polish), solved by
// a tiled Cholesky M = U'U on the fp64 matrix cores:
//   diagonal tile   16x16 block Cholesky by leg blocks (3x3 pivots) with U_bb^-T = L^-1 built alongside:
//                   per pivot one rank-3 MFMA update of the tile and one of L^-1 (diag_inverse) -- the
//                   only serial part;
//   row panel       U_bc = U_bb^-T M_bc and its transpose (v_mfma_f64_16x16x4f64, X'Y form);
//   trailing        M_cd -= U_bc' U_bd;
//   solves          U'y = r, U x = y tile by tile on the matrix cores (vectors replicated across
//                   the 16 accumulator columns, so every product feeds the next without LDS).
// The leg-level interior point and active-set polish are those of the Riccati path
// (lmpc_kernels.hip), with one stance leg-step per lane.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"
#include "lmpc_dense_common.h"

namespace lmpc {

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of QP 0..4095 (tools/dense_check.py).
#ifdef LMPC_STAMPS
constexpr int DSTAMP_N = 14;
__device__ unsigned long long lmpc_dense_stamps[4096][DSTAMP_N];
#define DSTAMP_DECL unsigned long long _ds_acc[DSTAMP_N] = {}; unsigned long long _ds_t0 = __builtin_readcyclecounter();
#define DSTAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _ds_acc[i] += _t - _ds_t0; _ds_t0 = _t; } while (0)
#define DSTAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < 4096) for (int _i = 0; _i < DSTAMP_N; ++_i) lmpc_dense_stamps[qp][_i] = _ds_acc[_i]; } while (0)
#define DS_PARAMS , unsigned long long (&_ds_acc)[DSTAMP_N], unsigned long long& _ds_t0
#define DS_ARGS , _ds_acc, _ds_t0
#else
#define DS_PARAMS
#define DS_ARGS
#define DSTAMP_DECL
#define DSTAMP(i) do {} while (0)
#define DSTAMP_FLUSH(qp) do {} while (0)
#endif

#ifdef LMPC_KKT_DIAG
// diagnostic build (tools/kkt_diag.py): per QP, at its last settled polish round, stationarity residual / gscale
__device__ double lmpc_kkt_diag_dense[LMPC_KKT_DIAG_QPS][4];
extern "C" int lmpc_debug_kkt_dense(double* out, int nqp) {
    if (nqp > LMPC_KKT_DIAG_QPS) nqp = LMPC_KKT_DIAG_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_kkt_diag_dense), (size_t)nqp * 4 * sizeof(double)) == hipSuccess
               ? nqp : -1;
}
extern "C" int lmpc_debug_kkt_dense_clear(void) {
    static double zeros[LMPC_KKT_DIAG_QPS * 4];
    return hipMemcpyToSymbol(HIP_SYMBOL(lmpc_kkt_diag_dense), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef LMPC_REFINE_DIAG
// diagnostic build (tools/refine_diag.py): per QP whose verified round was a range-space one, [stationarity residual
// / gscale, K's smallest pivot ratio, max |refinement correction|, 1 accepted / 2 rejected]
__device__ double lmpc_refine_diag[LMPC_KKT_DIAG_QPS][4];
extern "C" int lmpc_debug_refine(double* out, int nqp) {
    if (nqp > LMPC_KKT_DIAG_QPS) nqp = LMPC_KKT_DIAG_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_refine_diag), (size_t)nqp * 4 * sizeof(double)) == hipSuccess
               ? nqp : -1;
}
extern "C" int lmpc_debug_refine_clear(void) {
    static double zeros[LMPC_KKT_DIAG_QPS * 4];
    return hipMemcpyToSymbol(HIP_SYMBOL(lmpc_refine_diag), zeros, sizeof(zeros)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace lmpc

#include "lmpc_dense_kernel.h"

namespace lmpc {

template <bool TERRAIN>
__global__ void __launch_bounds__(64) lmpc_dense_kernel(const DevParams prm, const double* __restrict__ rec,
                                                        const uint8_t* __restrict__ contact,
                                                        const double* __restrict__ normals, int batch,
                                                        double* __restrict__ grf, int32_t* __restrict__ status,
                                                        int32_t* __restrict__ iters, uint8_t* __restrict__ done_out) {
    (void)dense_body<TERRAIN>(prm, rec, contact, normals, batch, grf, status, iters, done_out);
}

template __global__ void lmpc_dense_kernel<false>(const DevParams, const double*, const uint8_t*, const double*, int,
                                                  double*, int32_t*, int32_t*, uint8_t*);
template __global__ void lmpc_dense_kernel<true>(const DevParams, const double*, const uint8_t*, const double*, int,
                                                 double*, int32_t*, int32_t*, uint8_t*);

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_condense_stamps(unsigned long long* out, int nqp) {
    if (nqp > 4096) nqp = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_condense_stamps), (size_t)nqp * 5 * sizeof(unsigned long long)) ==
                   hipSuccess ? nqp : -1;
}
extern "C" int lmpc_debug_dense_stamps(unsigned long long* out, int nqp) {
    if (nqp > 4096) nqp = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_dense_stamps), (size_t)nqp * DSTAMP_N * sizeof(unsigned long long)) ==
                   hipSuccess ? nqp : -1;
}
#endif

size_t dense_lds_bytes(int H) {
    const int scr = 72 * H > DN_SCR_MIN ? 72 * H : DN_SCR_MIN;
    const int doubles = 40 + 72 + 24 + 36 + 10 * DN_TILE + 64 * 3 + 180 + 20 + 60 + 64 + 2 * H + 12 * H + 12 * H + 64 + scr;
    return (size_t)doubles * sizeof(double) + (20 + 33) * sizeof(int);
}

hipError_t launch_dense(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                        int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream) {
    const size_t lds = dense_lds_bytes(prm.H);
    const dim3 grid(batch), block(LMPC_WAVE);
    if (normals) {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_kernel<true>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_kernel<false>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    }
    return hipGetLastError();
}

}  // namespace lmpc

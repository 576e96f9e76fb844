// lmpc_device.h -- device-side parameter block shared by the kernels and the C-ABI.
#pragma once
#include <cstddef>
#include <cstdint>

namespace lmpc {

// Kernel argument block (by value).  All fp64, as in the reference (Eigen double).
struct DevParams {
    double q[12];      // state weights  (ConvexQPSolver.cpp:30)
    double r[12];      // input weights  (ConvexQPSolver.cpp:31)
    double mass;       // robot_mass     (ConvexQPSolver.cpp:280)
    double Ib[9];      // body inertia, row-major
    double mu;         // 0.3            (ConvexQPSolver.cpp:25)
    double fmax;       // 180            (ConvexQPSolver.cpp:171)
    double grav;       // 9.8            (ConvexQPSolver.cpp:175)
    double dt;         // 0.01           (ConvexQPSolver.cpp:26)
    double tol_mu;     // IPM stop: mean complementarity
    double tol_p;      // polish primal tolerance (relative to fmax)
    double tol_d;      // polish dual tolerance (relative to gradient scale)
    double tol_x;      // polish certificate: trajectory vs the forces' dynamics (relative to the state scale)
    int H;             // horizon
    int max_iter;      // IPM iteration cap (per attempt)
    int max_rounds;    // polish rounds per attempt
    int max_attempts;  // IPM+polish attempts (the stop tightened per attempt: retry_tol, lmpc_kernel_common.h)
    int dense;         // QPs with 1..DENSE_MAX_LS stance leg-steps: 0 Riccati kernel, 1 condensed interior
                       // point (lmpc_dense.hip), 2 condensed dual active set (lmpc_gi.hip)
    int gi_max_steps;  // dual active-set step cap; a QP that reaches it is solved by the Riccati kernel
    int dense_polish_iter;  // condensed interior point: iterations of the first attempt before the active-set polish
    int dense_iter_cap;  // condensed interior point: IPM iterations after which a QP is handed to the Riccati
                         // kernel (lmpc_options.dense_iter_cap; default: never, max_iter governs)
    int cus;           // compute units of the device (launch shaping only)
    // warm start of the Riccati kernel (per QP and leg-step [B][H][4]: bits 0-4 = active pyramid faces and
    // bound, 15 = lift-off apex).  warm_act != nullptr: the kernel starts in the active-set polish from it and
    // falls back to the cold interior point if the polish does not verify within max_rounds; act_out receives
    // the verified active set.  Both null by default.
    const uint8_t* warm_act;
    uint8_t* act_out;
    int warm_rounds;   // polish rounds a warm start may take before the cold fallback
};
constexpr int DENSE_MAX_LS = 20;  // 5 leg-steps per 16-wide tile x 4 tiles (lmpc_dense.hip)
constexpr int DENSE_MAX_H = 16;   // the dense path's per-step LDS arrays

constexpr size_t LMPC_CU_LDS_BYTES = 160 * 1024;  // LDS per CU on gfx950

// LDS footprint (doubles) of one QP for horizon H; carve() in lmpc_kernels.hip static_asserts both constants.
constexpr int LDS_FIXED_DOUBLES = 464;  // per-QP matrices and buffers
constexpr int LDS_STAGE_DOUBLES = 150;  // per-stage slot (SK)
constexpr int LDS_TERRAIN_DOUBLES = 60;  // terrain extension: 4 contact frames (36) + 4 packed R'diag(r)R (24)
inline int lds_doubles(int H, bool terrain = false) {
    return LDS_FIXED_DOUBLES + 2 * H + LDS_STAGE_DOUBLES * H + (terrain ? LDS_TERRAIN_DOUBLES : 0);
}
inline size_t lds_bytes(int H, bool terrain = false) { return (size_t)lds_doubles(H, terrain) * sizeof(double); }
// Global scratch (doubles) per QP: V, K, Z, Bt, input Hessian blocks, L^-1, dv, leg flags per stage (GS in lmpc_kernels.hip, static_asserted).
constexpr int SCRATCH_STAGE_DOUBLES = 380;
inline size_t scratch_doubles_per_qp(int H) { return (size_t)SCRATCH_STAGE_DOUBLES * H; }

}  // namespace lmpc

// lmpc_kernels.hip -- fused batched convex-MPC GRF QP solve for CDNA4 (gfx950).
//
// One 64-lane wavefront owns one QP end to end (one workgroup = one wave):
//   1. reads its packed record (x0 | R | feet | x_ref) and contact schedule once,
//      coalesced, into LDS;
//   2. builds the single-rigid-body model on the fly:
//        B  = [0; G0],  G0 = dt [I_w^-1 skew(r_j) ; I/m]      (ConvexQPSolver.cpp:198-212)
//        A_k = I + dt N(yaw_ref_k)                             (ConvexQPSolver.cpp:214-228)
//        x_{k+1} = A_k x_k + B u_k - g dt e11                  (ConvexQPSolver.cpp:174-176,294-297)
//        cost 1/2 sum(u'Ru + x'Qx) - sum x_ref' Q x            (ConvexQPSolver.cpp:29-50,308)
//        friction pyramid mu=0.3 and 0 <= fz <= 180*contact    (ConvexQPSolver.cpp:131-172,329-346)
//   3. solves the QP with a Mehrotra predictor-corrector interior point whose
//      Newton step is an LQR Riccati recursion over the horizon (condensation
//      done stage-wise by dynamic programming: O(H 12^3), not O((12H)^3));
//   4. polishes: takes the IPM active set, re-solves the equality-constrained
//      LQR exactly (per-leg null-space parametrisation f = up + T y), verifies
//      primal feasibility and multiplier signs and repeats if needed, so the
//      answer is the exact optimum of the reference's QP;
//   5. writes u_0..u_{H-1} (world-frame GRFs); grf[0..11] is what the
//      reference's compute_grfs returns (ConvexQPSolver.cpp:314-327).
//
// Riccati stage (critical path, everything 12x12 or smaller, all in LDS):
//   Guu = blockdiag(T'RtT) + Bt' P22 Bt          (Bt = G0 T, per-leg blocks)
//   block-Cholesky of Guu by legs (3x3 pivots) with [Bt' | I] eliminated in the
//   same sweep -> V = L^-1 Bt', L^-1 ;  K = V'V (6x6 wrench compliance)
//   Z = P2 A, P_k = Q + A'PA - Z'(KZ)
// Vector passes are affine recursions through the closed-loop matrix
//   N_k = A_k - [0; KZ_k]   (x_{k+1} = N_k x_k + n_k,  p_k = N_k' s + c_k)
// with every per-stage triangular solve moved into stage-parallel pre/post passes.
//
// Per-leg state (f, s, z, T, up, Rt, rt) lives in the registers of the lane
// that owns the leg-step (lane = (4k + leg) mod 64).  L^-1, V, K, P2 go to a
// per-QP global scratch (L2-resident); everything on the recursion's critical
// path is in LDS.  All arithmetic is fp64.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

namespace lmpc {

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of QP 0..STAMP_QPS-1,
// written to a buffer no other code reads.  Never compiled into the product library.
#ifdef LMPC_STAMPS
constexpr int STAMP_QPS = 4096;
__device__ unsigned long long lmpc_stamps[STAMP_QPS][8];
#define STAMP_DECL unsigned long long _st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _st_t0 = __builtin_readcyclecounter();
#define STAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _st_acc[i] += _t - _st_t0; _st_t0 = _t; } while (0)
#define STAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < STAMP_QPS) for (int _i = 0; _i < 8; ++_i) lmpc_stamps[qp][_i] = _st_acc[_i]; } while (0)
// sub-phase stamps inside the outlined factor / solve functions and the main loop (slot < 24)
__device__ unsigned long long lmpc_substamps[STAMP_QPS][24];
#define SUB_DECL unsigned long long _sb_t0 = __builtin_readcyclecounter();
#define SUB(i) do { const unsigned long long _t = __builtin_readcyclecounter(); \
    if (threadIdx.x == 0 && blockIdx.x < STAMP_QPS) \
        __hip_atomic_fetch_add(&lmpc_substamps[blockIdx.x][i], _t - _sb_t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    _sb_t0 = _t; } while (0)
#else
#define SUB_DECL
#define SUB(i) do {} while (0)
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(qp) do {} while (0)
#endif
__device__ __forceinline__ int pk(int r, int c) { return r * (r + 1) / 2 + c; }  // packed lower, c <= r

// inverse of pk: packed index -> (r, c)
__device__ __forceinline__ void unpk(int e, int& r, int& c) {
    r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    if (r * (r + 1) / 2 > e) --r;
    if ((r + 1) * (r + 2) / 2 <= e) ++r;
    c = e - r * (r + 1) / 2;
}

// ---- LDS layout (doubles) --------------------------------------------------
// per-stage slot: only what the serial sweeps and the stage-parallel levels read at LDS latency.
// 150 doubles, so that 4 QPs share a CU at H = 30 (the matrices the factorisation
// streams -- Bt, the input Hessian blocks, L^-1 -- live in the per-QP global scratch below and are
// fetched one stage ahead).
constexpr int SO_RRV = 0;    // 12  input linear term rr (later: y)
constexpr int SO_KZ = 12;    // 6 x 12 rows 6-11 of K^Z^: closed loop N_k = A_k - [0; KZ] (A_k from the yaw)
constexpr int SO_VV = 84;    // 12  v = P_{k+1} d_k
constexpr int SO_CST = 96;   // 12  q_k - Z' psi + N' v (dead after the backward sweep)
constexpr int SO_LAM = 96;   // 12  lambda_{k+1}: the adjoint after a solve, read before the next one (aliases CST)
constexpr int SO_PSI = 108;  // 6   V' L^-1 rr (dead once the mid level has read it)
constexpr int SO_N6 = 108;   // 6   K s2 + psi - dv, later q2 (aliases PSI: each mid task reads its own psi entry)
constexpr int SO_RHO = 114;  // 12  L^-1 rr (later: t)
constexpr int SO_PN = 126;   // 12  p_{k+1}
constexpr int SO_XS = 138;   // 12  x_k
constexpr int SK = 150;
// global scratch per stage
constexpr int GO_V = 0;      // 6 x 12 V' (column m of V = L^-1 Bt' contiguous)
constexpr int GO_K = 72;     // 6 x 6 K = V'V
constexpr int GO_Z = 108;    // 6 x 12 Z = P2_{k+1} A_k
constexpr int GO_BT = 180;   // 6 x 12 Bt = G0 T
constexpr int GO_RR = 252;   // 4 x 3x3 input Hessian blocks T'RtT
constexpr int GO_LINV = 288; // 78  L^-1 of Guu, row-packed
constexpr int GO_DV = 366;   // 6   d_k[6:12] = G0 up - g dt e5
constexpr int GO_ACT = 372;  // 4   leg block coupled (1) or decoupled identity block (0: T = 0)
constexpr int GO_ZERO = 376; // 2   always 0.0
constexpr int GO_DUMMY = 378;  // sink for the branch-free masked stores
constexpr int GS = 380;

struct Smem {
    ldouble* G0;   // 72
    ldouble* hdr;  // 40: x0(12) R(9) feet(12)
    ldouble* cs;   // 2H
    const gdouble* xr;  // 12H x_ref, read from the input record in global memory (L2-resident after first use)
    ldouble* xH;   // 12
    ldouble* GT;   // 144  Guu, column-major
    ldouble* PNL;  // 72   pivot block columns (3 columns x 12 rows), double-buffered
    ldouble* VL;   // 72   V = L^-1 Bt', column-major
    ldouble* pa;   // 12
    ldouble* pb;   // 12
    ldouble* qw;   // 12  state weights q
    ldouble* zero; // 16  always 0.0
    ldouble* st;   // H * SK
};

// fixed-size LDS members, in carve order; the total must equal LDS_FIXED_DOUBLES (lmpc_device.h)
constexpr int LDS_SIZES[] = {72, 40, 12, 144, 72, 72, 12, 12, 12, 16};  // G0 hdr xH GT PNL VL pa pb qw zero
constexpr int lds_fixed_sum() {
    int t = 0;
    for (int v : LDS_SIZES) t += v;
    return t;
}
static_assert(lds_fixed_sum() == LDS_FIXED_DOUBLES, "LDS carve and lds_doubles() disagree");
static_assert(SK == LDS_STAGE_DOUBLES, "per-stage LDS slot and lds_doubles() disagree");
static_assert(GS == SCRATCH_STAGE_DOUBLES, "per-stage global scratch and scratch_doubles_per_qp() disagree");

__device__ __forceinline__ Smem carve(double* sm, int H) {
    Smem s;
    ldouble* p = (ldouble*)sm;
    s.G0 = p; p += 72;
    s.hdr = p; p += 40;
    s.xH = p; p += 12;
    s.GT = p; p += 144;
    s.PNL = p; p += 72;
    s.VL = p; p += 72;
    s.pa = p; p += 12;
    s.pb = p; p += 12;
    s.qw = p; p += 12;
    s.zero = p; p += 16;
    s.cs = p; p += 2 * H;
    s.xr = nullptr;  // set by the kernel
    s.st = p;  // offset LDS_FIXED_DOUBLES + 2H doubles (even: 16-B aligned)
    return s;
}

// M(yaw)[i][j] for a lane-static j and per-stage (c, s)
__device__ __forceinline__ void Mcol(double c, double s, int j, double m[3]) {
    m[0] = (j == 0) ? c : (j == 1) ? s : 0.0;
    m[1] = (j == 0) ? -s : (j == 1) ? c : 0.0;
    m[2] = (j == 2) ? 1.0 : 0.0;
}

// (A x)[c] for the stage yaw (c, s)
template <class Ptr>
__device__ __forceinline__ double Ax_el(Ptr x, int c, double ck, double sk, double dt) {
    if (c < 3) return x[c] + dt * (Myaw(ck, sk, c, 0) * x[6] + Myaw(ck, sk, c, 1) * x[7] + Myaw(ck, sk, c, 2) * x[8]);
    if (c < 6) return x[c] + dt * x[c + 6];
    return x[c];
}

// (A' w)[r]
template <class Ptr>
__device__ __forceinline__ double Atw_el(Ptr w, int r, double ck, double sk, double dt) {
    if (r >= 6 && r < 9)
        return w[r] + dt * (Myaw(ck, sk, 0, r - 6) * w[0] + Myaw(ck, sk, 1, r - 6) * w[1] + Myaw(ck, sk, 2, r - 6) * w[2]);
    if (r >= 9) return w[r] + dt * w[r - 6];
    return w[r];
}

// ---------------------------------------------------------------------------
// Riccati factorisation (backward, matrix part).
//
// The dense 12x12 products run on the fp64 matrix cores (v_mfma_f64_16x16x4f64,
// 12x12 padded to 16x16).  Accumulator layout: lane l, register i holds row
// (l>>4)+4i, column l&15 -- which is also the B operand of k-block i, and, for a
// symmetric matrix, the A operand of k-block i.  So P_{k+1} stays in registers and
// every product feeds the next without an LDS round trip:
//   C^ = P B^            (B^ = [0; Bt | dv]: rows 6-11 hold Bt, column 12 dv -> v = P d)
//   Guu = Rr + B^' C^     (the 12x12 input Hessian block plus the lifted state cost)
//   PA = P A_k = P + P (dt N)         (dt N: rows 0-5 only -> 2 k-blocks)
//   [block Cholesky of Guu with [Bt' | I] eliminated alongside, VALU, one column per lane]
//   K^ = V^' V^           (V^ = [0 | V]: K lands in rows/columns 6-11, aligned with PA's rows)
//   KZ^ = K^ PA           (rows 6-11 = K Z,  Z = P2 A = rows 6-11 of PA)
//   P_k = Q + PA + (dt N)'PA - PA' KZ^ ;  N_k = A_k - KZ^ (closed-loop matrix for the vector pass)
// ---------------------------------------------------------------------------
// entry (r, c) of dt N(yaw) = A_k - I (nonzero only in rows 0-5, columns 6-11)
__device__ __forceinline__ double dtN_entry(int r, int c, double ck, double sk, double dt) {
    if (r >= 12 || c >= 12) return 0.0;
    double v = 0.0;
    if (r < 3 && c >= 6 && c < 9) {
        const int j = c - 6;
        const double m = (r == 0) ? ((j == 0) ? ck : (j == 1) ? sk : 0.0)
                       : (r == 1) ? ((j == 0) ? -sk : (j == 1) ? ck : 0.0)
                                  : ((j == 2) ? 1.0 : 0.0);
        v += dt * m;
    }
    if (r >= 3 && r < 6 && c == r + 6) v += dt;
    return v;
}

// Entry (j, c) of the closed-loop N_k = A_k - [0; KZ] as a lane-static affine form in the stage's
// yaw (ck, sk) and kzv = KZ[j-6][c]:  N = b + cc ck + sc sk - kz kzv.
struct NCoef {
    double b, cc, sc, kz;
};
__device__ __forceinline__ NCoef n_coef(int j, int c, double dt) {
    NCoef n;
    n.b = (j == c) ? 1.0 : 0.0;
    n.cc = n.sc = n.kz = 0.0;
    if (j < 6) {
        n.b += dtN_entry(j, c, 0.0, 0.0, dt);           // the yaw-independent part
        n.cc = dtN_entry(j, c, 1.0, 0.0, dt) - (n.b - ((j == c) ? 1.0 : 0.0));
        n.sc = dtN_entry(j, c, 0.0, 1.0, dt) - (n.b - ((j == c) ? 1.0 : 0.0));
    } else {
        n.kz = 1.0;
    }
    return n;
}
__device__ __forceinline__ double n_eval(const NCoef& n, double ck, double sk, double kzv) {
    return fma(n.cc, ck, fma(n.sc, sk, fma(-n.kz, kzv, n.b)));
}

// W: the calling kernel's waves-per-SIMD budget -- one copy per budget, so each copy is register-
// allocated for its caller's occupancy (a shared callee would take the larger budget into both)
template <int W>
// Diagnostic builds only (tools/build, -DLMPC_FACTOR_INLINE / -DLMPC_SOLVE_INLINE): the factor / solve inlined at
// their one call site instead of outlined (A/B of the call-saved register traffic).
#ifdef LMPC_FACTOR_INLINE
#define LMPC_FACTOR_ATTR always_inline
#else
#define LMPC_FACTOR_ATTR noinline
#endif
#ifdef LMPC_SOLVE_INLINE
#define LMPC_SOLVE_ATTR always_inline
#else
#define LMPC_SOLVE_ATTR noinline
#endif
__device__ __attribute__((LMPC_FACTOR_ATTR)) void riccati_factor(const Smem S, gdouble* __restrict__ gs, int H, const double dt,
                                                         const int lane) {
    H = __builtin_amdgcn_readfirstlane(H);  // wave-uniform (arguments arrive in VGPRs): scalar loop control
    const int lc = lane & 15, lr = lane >> 4;  // accumulator layout: column lc, rows lr + 4i
    d4 P;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        P[i] = (r == lc && r < 12) ? S.qw[r < 12 ? r : 0] : 0.0;
    }
    const d4 Qd = P;
    // ---- lane-static operand maps, hoisted out of the stage loop ----
    // dt N(yaw) entries of k-blocks 0-1: dt (nc cos + ns sin + n1)
    double nc[2], ns[2], n1[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int r = 4 * kk + lr, c = lc;
        nc[kk] = ns[kk] = n1[kk] = 0.0;
        if (r < 3 && c >= 6 && c < 9) {  // M(yaw)[r][c-6]: [c s 0; -s c 0; 0 0 1]
            const int j = c - 6;
            if (r == 0) { nc[kk] = (j == 0) ? dt : 0.0; ns[kk] = (j == 1) ? dt : 0.0; }
            if (r == 1) { ns[kk] = (j == 0) ? -dt : 0.0; nc[kk] = (j == 1) ? dt : 0.0; }
            if (r == 2) n1[kk] = (j == 2) ? dt : 0.0;
        }
        if (r >= 3 && r < 6 && c == r + 6) n1[kk] = dt;
    }
    // B^ (k-blocks 1-2: Bt from the global scratch, dv from the stage slot) and Rr operand offsets;
    // out-of-range -> the zero words
    int boff[2], roff[4];
#pragma unroll
    for (int kk = 1; kk < 3; ++kk) {
        const int r = 4 * kk + lr;
        const bool brow = r >= 6 && r < 12;
        boff[kk - 1] = (brow && lc < 12) ? GO_BT + (r - 6) * 12 + lc : (brow && lc == 12) ? GO_DV + (r - 6) : GO_ZERO;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        roff[i] = (r < 12 && lc < 12 && (r / 3) == (lc / 3)) ? GO_RR + (r / 3) * 9 + (r % 3) * 3 + (lc % 3) : GO_ZERO;
    }
    // Bt' in columns 6-11 of the V^ tile (accumulator layout): lane (lr, lc), register i <- Bt[lc-6][lr+4i]
    const bool vcol = lc >= 6 && lc < 12;
    int btof[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) btof[i] = vcol ? GO_BT + (lc - 6) * 12 + lr + 4 * i : GO_ZERO;
    // the global operands of a stage do not depend on P: fetched one stage ahead, their latency
    // hides behind the previous stage's products
    double bgn[2], rgn[4], btn[3], agn[4];
    auto fetch = [&](const gdouble* g) {
        bgn[0] = g[boff[0]];
        bgn[1] = g[boff[1]];
#pragma unroll
        for (int j = 0; j < 4; ++j) agn[j] = g[GO_ACT + j];
#pragma unroll
        for (int i = 0; i < 4; ++i) rgn[i] = g[roff[i]];
#pragma unroll
        for (int i = 0; i < 3; ++i) btn[i] = g[btof[i]];
    };
    fetch(gs + (H - 1) * GS);
    // lane-static destinations of the factor outputs (branch-free stores; the rest go to the dummy word):
    // V column m = lc - 6 contiguous (GO_V), packed lower L^-1 row r = lr + 4i, column lc <= r (GO_LINV)
    int vofs[3], lofs[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int r = lr + 4 * i;
        vofs[i] = vcol ? GO_V + (lc - 6) * 12 + r : GO_DUMMY;
        lofs[i] = (lc <= r) ? GO_LINV + r * (r + 1) / 2 + lc : GO_DUMMY;
    }
    ldouble* const pv = S.GT;     // 144: pivot rows of Guu, L^-1 and V^ (48 each)
    ldouble* const sink = S.PNL;  // 64: stores of lanes that hold no pivot row
    SUB_DECL
    for (int k = H - 1; k >= 0; --k) {
        const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
        ldouble* sl = S.st + k * SK;
        gdouble* g = gs + k * GS;
        double bg[2], rg[4], bt[3], ag[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) bg[i] = bgn[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) ag[j] = agn[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) rg[i] = rgn[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) bt[i] = btn[i];
        // ---- operands: dt N(yaw) (k-blocks 0-1: rows 0-7) and B^ (k-blocks 1-2) ----
        double nh[2], bh[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) nh[kk] = fma(nc[kk], ck, fma(ns[kk], sk, n1[kk]));
        bh[0] = bg[0];
        bh[1] = bg[1];
        // ---- C^ = P B^ ; PA = P A_k = P + P (dt N) ----
        d4 C = {0.0, 0.0, 0.0, 0.0};
        C = MFMA64(P[1], bh[0], C);
        C = MFMA64(P[2], bh[1], C);
        d4 PA = P;
        PA = MFMA64(P[0], nh[0], PA);
        PA = MFMA64(P[1], nh[1], PA);
        // ---- Guu = Rr + B^' C^ (Rr: 3x3 leg blocks on the diagonal) ----
        d4 G;
#pragma unroll
        for (int i = 0; i < 4; ++i) G[i] = rg[i];
        G = MFMA64(bh[0], C[1], G);
        G = MFMA64(bh[1], C[2], G);
        // next stage's global operands: issued while the matrix cores work through the chain above
        __builtin_amdgcn_sched_barrier(0);
        fetch(gs + (k > 0 ? k - 1 : 0) * GS);
        __builtin_amdgcn_sched_barrier(0);
        // ---- out: v = C^[:, 12], Z = rows 6-11 of PA ----
        if (lc < 12) {
#pragma unroll
            for (int i = 1; i < 3; ++i) {
                const int r = lr + 4 * i;
                if (r >= 6) g[GO_Z + (r - 6) * 12 + lc] = PA[i];
            }
        } else if (lc == 12) {
#pragma unroll
            for (int i = 0; i < 3; ++i) sl[SO_VV + lr + 4 * i] = C[i];
        }
        SUB(5);
        // ---- block Cholesky of Guu by legs, with L^-1 (from I) and V^ = L^-1 [0 | Bt'] eliminated alongside,
        //      all three 16x16 tiles in the accumulator layout (the dense path's diag_inverse, lmpc_dense_common.h).
        // Per coupled 3x3 leg block: its rows of the three tiles go through LDS, every lane factors the pivot
        // P = L_p L_p', and one rank-3 v_mfma_f64_16x16x4f64 per tile applies it: Guu -= L_C L_C', and
        // L^-1, V^ -= L_C (L_p^-1 X_p) with their pivot rows replaced by L_p^-1 X_p.  Leg blocks with T = 0
        // (swing legs; apex legs in the polish) have Guu block = I and no coupling: skipped (amask, wave-uniform).
        d4 Tg, Li, X;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = lr + 4 * i;
            Tg[i] = (r < 12 && lc < 12) ? G[i] : 0.0;  // row / column 12 of G carries dv' C^: not part of Guu
            Li[i] = (r == lc) ? 1.0 : 0.0;
            X[i] = (i < 3) ? bt[i < 3 ? i : 0] : 0.0;
        }
        int amask;
        {
            amask = (ag[0] != 0.0 ? 1 : 0) | (ag[1] != 0.0 ? 2 : 0) | (ag[2] != 0.0 ? 4 : 0) | (ag[3] != 0.0 ? 8 : 0);
            amask = __builtin_amdgcn_readfirstlane(amask);
        }
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            if (!((amask >> blk) & 1)) continue;
            const int o = 3 * blk;
            const int i0 = o >> 2, i1 = (o + 2) >> 2;  // registers holding rows o..o+2 (static)
            const int ra = 4 * i0 + lr - o, rb = 4 * i1 + lr - o;
            const bool ina = ra >= 0 && ra < 3, inb = i1 != i0 && rb >= 0 && rb < 3;
            LMPC_SYNC();
            {
                ldouble* da = ina ? pv + 16 * ra + lc : sink + lane;
                da[0] = Tg[i0];
                if (i1 != i0) {
                    ldouble* db = inb ? pv + 16 * rb + lc : sink + lane;
                    db[0] = Tg[i1];
                }
            }
            LMPC_SYNC();
            const double p00 = pv[o], p10 = pv[16 + o], p11 = pv[16 + o + 1];
            const double p20 = pv[32 + o], p21 = pv[32 + o + 1], p22 = pv[32 + o + 2];
            const double t0 = pv[lc], t1 = pv[16 + lc], t2 = pv[32 + lc];  // Guu[o+a][lc] = Guu[lc][o+a]
            {
                ldouble* da = ina ? pv + 48 + 16 * ra + lc : sink + lane;
                da[0] = Li[i0];
                ldouble* dx = ina ? pv + 96 + 16 * ra + lc : sink + lane;
                dx[0] = X[i0];
                Li[i0] = ina ? 0.0 : Li[i0];
                X[i0] = ina ? 0.0 : X[i0];
                if (i1 != i0) {
                    ldouble* db = inb ? pv + 48 + 16 * rb + lc : sink + lane;
                    db[0] = Li[i1];
                    ldouble* dy = inb ? pv + 96 + 16 * rb + lc : sink + lane;
                    dy[0] = X[i1];
                    Li[i1] = inb ? 0.0 : Li[i1];
                    X[i1] = inb ? 0.0 : X[i1];
                }
            }
            LMPC_SYNC();
            const double w0 = pv[48 + lc], w1 = pv[64 + lc], w2 = pv[80 + lc];
            const double y0 = pv[96 + lc], y1 = pv[112 + lc], y2 = pv[128 + lc];
            const double i00 = rsq_nr(p00);
            const double l10 = p10 * i00, l20 = p20 * i00;
            const double i11 = rsq_nr(fma(-l10, l10, p11));
            const double l21 = fma(-l20, l10, p21) * i11;
            const double i22 = rsq_nr(fma(-l21, l21, fma(-l20, l20, p22)));
            // row lc of L_C (zero in and above the pivot rows)
            const double x0 = t0 * i00;
            const double x1 = fma(-l10, x0, t1) * i11;
            const double x2 = fma(-l21, x1, fma(-l20, x0, t2)) * i22;
            const double xs = lr == 0 ? x0 : lr == 1 ? x1 : x2;
            const double av = (lc > o + 2 && lr < 3) ? xs : 0.0;
            // column lc of L_p^-1 W_p and of L_p^-1 X_p
            const double v0 = w0 * i00;
            const double v1 = fma(-l10, v0, w1) * i11;
            const double v2 = fma(-l21, v1, fma(-l20, v0, w2)) * i22;
            const double q0 = y0 * i00;
            const double q1 = fma(-l10, q0, y1) * i11;
            const double q2 = fma(-l21, q1, fma(-l20, q0, y2)) * i22;
            const double bw = lr == 0 ? v0 : lr == 1 ? v1 : lr == 2 ? v2 : 0.0;
            const double bx = lr == 0 ? q0 : lr == 1 ? q1 : lr == 2 ? q2 : 0.0;
            const bool cp = lc >= o && lc <= o + 2;
            const double aw = cp ? (lr == lc - o ? 1.0 : 0.0) : -av;
            Tg = MFMA64(-av, av, Tg);
            Li = MFMA64(aw, bw, Li);
            X = MFMA64(aw, bx, X);
            SUB(9 + blk);
        }
        // factor outputs: V (columns 6-11 of V^) and packed L^-1 to the global scratch (branch-free)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            g[vofs[i]] = X[i];
            g[lofs[i]] = Li[i];
        }
        SUB(7);
        // ---- K^ = V^' V^ (V^ = [0 | V], columns 6-11; rows 0-11 = k-blocks 0-2) ----
        d4 KH = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) KH = MFMA64(X[kk], X[kk], KH);
        // ---- KZ^ = K^ PA (k-blocks 1-2: K^ is zero outside rows/columns 6-11) ----
        d4 KZ = {0.0, 0.0, 0.0, 0.0};
        KZ = MFMA64(KH[1], PA[1], KZ);
        KZ = MFMA64(KH[2], PA[2], KZ);
        // K -> global (for the vector pass), rows 6-11 of KZ^ -> stage slot (N_k = A_k - [0; KZ])
        if (lc >= 6 && lc < 12) {
#pragma unroll
            for (int i = 1; i < 3; ++i) {
                const int r = lr + 4 * i;
                if (r >= 6) g[GO_K + (r - 6) * 6 + (lc - 6)] = KH[i];
            }
        }
        if (lc < 12) {
#pragma unroll
            for (int i = 1; i < 3; ++i) {
                const int r = lr + 4 * i;
                if (r >= 6) sl[SO_KZ + (r - 6) * 12 + lc] = KZ[i];
            }
        }
        // ---- P_k = Q + A'PA - PA' KZ^,  A'PA = PA + (dt N)' PA ----
        if (k > 0) {
            d4 Pn = Qd + PA;
            Pn = MFMA64(nh[0], PA[0], Pn);
            Pn = MFMA64(nh[1], PA[1], Pn);
            Pn = MFMA64(-PA[1], KZ[1], Pn);
            Pn = MFMA64(-PA[2], KZ[2], Pn);
            P = Pn;
        }
        SUB(8);
    }
    LMPC_GSYNC();  // V, K, Z, L^-1 in the global scratch visible to every lane of the vector pass
}

// ---------------------------------------------------------------------------
// Vector pass.  Reads rr (SO_RRV) per stage; leaves y in SO_RRV and x_k in SO_XS / xH.
//   pre   rho = L^-1 rr ; psi = V' rho ; cst'_k = q_k - Z'psi + N_k' v
//   back  p_k = N_k' p_{k+1} + cst'_k,  N_k = A_k - [0; KZ_k]       (serial, lanes 0-11)
//   mid   n6'_k = K (v6 + p_{k+1}[6:12]) + psi - dv
//   fwd   x_{k+1} = N_k x_k - [0; n6'_k]                              (serial, lanes 0-11)
//   post  q2 = Z x_k + v6 + p_{k+1}[6:12] ; t = V q2 + rho ; y = -L^-T t
// Stage-parallel levels are unrolled NT12 = ceil(12H/64) times with clamped task
// indices so that every global load is unconditional and issued before any use;
// the pre-pass data are fetched at entry, the post-pass data at the start of the
// forward sweep (their L2 latency hides behind the serial recursion).
// ---------------------------------------------------------------------------
template <int NT12, int W>
__device__ __attribute__((LMPC_SOLVE_ATTR)) void riccati_solve(const Smem S, const gdouble* __restrict__ gs, int H,
                                                        const double dt, const int lane) {
    constexpr int NT6 = (NT12 + 1) / 2;
    H = __builtin_amdgcn_readfirstlane(H);  // wave-uniform (arguments arrive in VGPRs): scalar loop control
    const int n12 = 12 * H, n6 = 6 * H;
    SUB_DECL
    int k12[NT12], r12[NT12];
    bool v12[NT12];
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const int e = lane + 64 * i;
        v12[i] = e < n12;
        const int ec = v12[i] ? e : n12 - 1;
        k12[i] = ec / 12;
        r12[i] = ec - 12 * k12[i];
    }
    int k6[NT6], m6[NT6];
    bool v6[NT6];
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const int e = lane + 64 * i;
        v6[i] = e < n6;
        const int ec = v6[i] ? e : n6 - 1;
        k6[i] = ec / 6;
        m6[i] = ec - 6 * k6[i];
    }
    // ---- prefetch from the global scratch: V columns, Z columns (L^-1 is LDS-resident) ----
    double zc[NT12][6], vc[NT6][12];
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const gdouble* Z = gs + k12[i] * GS + GO_Z + r12[i];
#pragma unroll
        for (int m = 0; m < 6; ++m) zc[i][m] = Z[m * 12];
    }
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const gdouble* V = gs + k6[i] * GS + GO_V + m6[i] * 12;
#pragma unroll
        for (int r = 0; r < 12; ++r) vc[i][r] = V[r];
    }
    // pre 1: rho = L^-1 rr (masked arithmetic on unconditional loads)
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const ldouble* rr = S.st + k12[i] * SK + SO_RRV;
        const gdouble* Li = gs + k12[i] * GS + GO_LINV + pk(r12[i], 0);  // pk(r, c) < 78 for every c < 12
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < 12; ++c) v += Li[c] * ((c <= r12[i]) ? rr[c] : 0.0);  // unconditional global loads
        if (v12[i]) S.st[k12[i] * SK + SO_RHO + r12[i]] = v;
    }
    LMPC_SYNC();
    // pre 2: psi = V' rho
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const ldouble* rho = S.st + k6[i] * SK + SO_RHO;
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 12; ++r) v += vc[i][r] * rho[r];
        if (v6[i]) S.st[k6[i] * SK + SO_PSI + m6[i]] = v;
    }
    LMPC_SYNC();
    // pre 3: cst'_k = -q x_ref,k-1 - Z'psi + N_k' v   (k >= 1)
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const int k = k12[i], r = r12[i];
        const ldouble* sl = S.st + k * SK;
        double v = -S.qw[r] * S.xr[(k > 0 ? k - 1 : 0) * 12 + r];
#pragma unroll
        for (int m = 0; m < 6; ++m) v -= zc[i][m] * sl[SO_PSI + m];
        // N_k' v = A_k' v - KZ' v[6:12]
        v += Atw_el(sl + SO_VV, r, S.cs[2 * k], S.cs[2 * k + 1], dt);
#pragma unroll
        for (int m = 0; m < 6; ++m) v -= sl[SO_KZ + m * 12 + r] * sl[SO_VV + 6 + m];
        if (v12[i] && k > 0) S.st[k * SK + SO_CST + r] = v;
    }
    if (lane < 12) S.st[(H - 1) * SK + SO_PN + lane] = -S.qw[lane] * S.xr[(H - 1) * 12 + lane];
    double kk[NT6][6];
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const gdouble* Kp = gs + k6[i] * GS + GO_K + m6[i] * 6;
#pragma unroll
        for (int n = 0; n < 6; ++n) kk[i][n] = Kp[n];
    }
    LMPC_SYNC();
    SUB(0);
    // ---- backward: p_k = N_k' p_{k+1} + cst'_k (into stage k-1's PN slot).  Row r is split over the
    // 4 lanes (r, part): each sums 3 of the 12 terms, a DPP quad reduction combines them.  The lane's
    // 3 entries of N_k (column r: rows j0..j0+2) are formed one step ahead -- from the yaw for rows
    // 0-5, from KZ for rows 6-11 -- so only 3 broadcast reads of p_{k+1} sit on the critical path ----
    {
        const int r = (lane < 48) ? (lane >> 2) : 0, part = lane & 3, j0 = 3 * part;
        const bool wr = lane < 48 && part == 0;
        const int kzo = SO_KZ + (j0 >= 6 ? j0 - 6 : 0) * 12 + r;  // KZ[j0-6+q][r] at kzo + 12q (rows 6-11)
        NCoef co[3];
        double nc[3], rw[5];  // rw: raw operands (yaw cos/sin, 3 KZ entries) of the stage after next
        const int k1 = H > 1 ? H - 2 : 0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            co[q] = n_coef(j0 + q, r, dt);
            nc[q] = n_eval(co[q], S.cs[2 * (H - 1)], S.cs[2 * (H - 1) + 1], S.st[(H - 1) * SK + kzo + 12 * q]);
        }
        rw[0] = S.cs[2 * k1];
        rw[1] = S.cs[2 * k1 + 1];
#pragma unroll
        for (int q = 0; q < 3; ++q) rw[2 + q] = S.st[k1 * SK + kzo + 12 * q];
        for (int k = H - 1; k >= 1; --k) {
            const ldouble* sl = S.st + k * SK;
            double pv[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) pv[q] = sl[SO_PN + j0 + q];
            const double cst = sl[SO_CST + r];
            // N_{k-1} from the raw operands fetched last step, and the raw operands of k-2, both
            // while the reads of p_{k+1} are in flight (pinned: the chain below stays clear)
            __builtin_amdgcn_sched_barrier(0);
            double nn[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) nn[q] = n_eval(co[q], rw[0], rw[1], rw[2 + q]);
            const int k2 = k > 2 ? k - 2 : 0;
            rw[0] = S.cs[2 * k2];
            rw[1] = S.cs[2 * k2 + 1];
#pragma unroll
            for (int q = 0; q < 3; ++q) rw[2 + q] = S.st[k2 * SK + kzo + 12 * q];
            __builtin_amdgcn_sched_barrier(0);
            double v = nc[0] * pv[0] + nc[1] * pv[1] + nc[2] * pv[2];
            v = quad_sum(v);
            ldouble* dst = wr ? S.st + (k - 1) * SK + SO_PN + r : S.pa;  // branch-free: others write a dummy word
            *dst = v + cst;
#pragma unroll
            for (int q = 0; q < 3; ++q) nc[q] = nn[q];
            LMPC_SYNC();
        }
    }
    SUB(1);
    // mid: n6'_k = K (v6 + p6) + psi - dv
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const ldouble* sl = S.st + k6[i] * SK;
        double v = sl[SO_PSI + m6[i]] - gs[k6[i] * GS + GO_DV + m6[i]];
#pragma unroll
        for (int n = 0; n < 6; ++n) v += kk[i][n] * (sl[SO_VV + 6 + n] + sl[SO_PN + 6 + n]);
        if (v6[i]) S.st[k6[i] * SK + SO_N6 + m6[i]] = v;
    }
    if (lane < 12) S.st[SO_XS + lane] = S.hdr[lane];
    LMPC_SYNC();
    SUB(2);
    // post-pass data from the global scratch, fetched now so that its latency hides behind the forward sweep
    double zr[NT6][12], vr[NT12][6];
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const gdouble* Z = gs + k6[i] * GS + GO_Z + m6[i] * 12;
#pragma unroll
        for (int c = 0; c < 12; ++c) zr[i][c] = Z[c];
    }
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const gdouble* V = gs + k12[i] * GS + GO_V + r12[i];
#pragma unroll
        for (int m = 0; m < 6; ++m) vr[i][m] = V[m * 12];
    }
    // ---- forward: x_{k+1} = N_k x_k - [0; n6'_k]; row r split over 4 lanes as in the backward sweep ----
    {
        const int r = (lane < 48) ? (lane >> 2) : 0, part = lane & 3, j0 = 3 * part;
        const bool wr = lane < 48 && part == 0;
        const int r6 = (r >= 6) ? r - 6 : 0;
        const double sel = (r >= 6) ? 1.0 : 0.0;
        const int kzo = SO_KZ + r6 * 12 + j0;  // KZ[r-6][j0+q] (rows 6-11)
        NCoef co[3];
        double nr[3], rw[5];  // rw: raw operands of the stage after next (as in the backward sweep)
        const int k1 = H > 1 ? 1 : 0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            co[q] = n_coef(r, j0 + q, dt);
            nr[q] = n_eval(co[q], S.cs[0], S.cs[1], S.st[kzo + q]);
        }
        rw[0] = S.cs[2 * k1];
        rw[1] = S.cs[2 * k1 + 1];
#pragma unroll
        for (int q = 0; q < 3; ++q) rw[2 + q] = S.st[k1 * SK + kzo + q];
        for (int k = 0; k < H; ++k) {
            const ldouble* sl = S.st + k * SK;
            ldouble* xo = (k + 1 < H) ? S.st + (k + 1) * SK + SO_XS : S.xH;
            double x[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) x[q] = sl[SO_XS + j0 + q];
            const double n6 = sl[SO_N6 + r6];
            __builtin_amdgcn_sched_barrier(0);
            double nn[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) nn[q] = n_eval(co[q], rw[0], rw[1], rw[2 + q]);
            const int k2 = k + 2 < H ? k + 2 : H - 1;
            rw[0] = S.cs[2 * k2];
            rw[1] = S.cs[2 * k2 + 1];
#pragma unroll
            for (int q = 0; q < 3; ++q) rw[2 + q] = S.st[k2 * SK + kzo + q];
            __builtin_amdgcn_sched_barrier(0);
            double v = nr[0] * x[0] + nr[1] * x[1] + nr[2] * x[2];
            v = quad_sum(v);
            ldouble* dst = wr ? xo + r : S.pa;
            *dst = v - sel * n6;
#pragma unroll
            for (int q = 0; q < 3; ++q) nr[q] = nn[q];
            LMPC_SYNC();
        }
    }
    SUB(3);
    // post 1: q2 = Z x_k + v6 + p6   -> SO_N6
#pragma unroll
    for (int i = 0; i < NT6; ++i) {
        const ldouble* sl = S.st + k6[i] * SK;
        double v = sl[SO_VV + 6 + m6[i]] + sl[SO_PN + 6 + m6[i]];
#pragma unroll
        for (int c = 0; c < 12; ++c) v += zr[i][c] * sl[SO_XS + c];
        if (v6[i]) S.st[k6[i] * SK + SO_N6 + m6[i]] = v;
    }
    LMPC_SYNC();
    // post 2: t = V q2 + rho  -> SO_RHO (in place: each entry is read by its own task only)
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const ldouble* sl = S.st + k12[i] * SK;
        double v = sl[SO_RHO + r12[i]];
#pragma unroll
        for (int m = 0; m < 6; ++m) v += vr[i][m] * sl[SO_N6 + m];
        if (v12[i]) S.st[k12[i] * SK + SO_RHO + r12[i]] = v;
    }
    LMPC_SYNC();
    // post 3: y = -L^-T t  -> SO_RRV
#pragma unroll
    for (int i = 0; i < NT12; ++i) {
        const ldouble* t = S.st + k12[i] * SK + SO_RHO;
        const gdouble* Li = gs + k12[i] * GS + GO_LINV;
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 12; ++r) v += Li[pk(r, r12[i])] * ((r >= r12[i]) ? t[r] : 0.0);  // pk < 78 for all r
        if (v12[i]) S.st[k12[i] * SK + SO_RRV + r12[i]] = -v;
    }
    LMPC_SYNC();
    SUB(4);
}

// Adjoint: lambda_{k+1} for every stage (SO_LAM) from the trajectory in SO_XS / xH.
//   lambda_H = q (x_H - xr_{H-1});  lambda_k = q (x_k - xr_{k-1}) + A_k' lambda_{k+1}
// The tracking terms do not depend on lambda: one stage-parallel level writes them (x_ref comes from
// global memory, so its latency is paid once), then the serial sweep adds A_k' lambda_{k+1} in place.
__device__ __forceinline__ void adjoint(const DevParams& prm, const Smem& S, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    const int n12 = 12 * H;
    constexpr int MAXT = (12 * 32 + 63) / 64;  // H <= 32
#pragma unroll
    for (int i = 0; i < MAXT; ++i) {
        const int e = lane + 64 * i;
        if (64 * i >= n12) break;  // wave-uniform
        const int ec = e < n12 ? e : n12 - 1;  // clamped: the load stays unconditional
        const int k = ec / 12, r = ec - 12 * k;
        const double xn = (k + 1 < H) ? S.st[(k + 1) * SK + SO_XS + r] : S.xH[r];
        const double v = prm.q[r] * (xn - S.xr[ec]);
        if (e < n12) S.st[k * SK + SO_LAM + r] = v;
    }
    LMPC_SYNC();
    for (int k = H - 1; k >= 1; --k) {
        if (lane < 12) {
            const int r = lane;
            const ldouble* lam = S.st + k * SK + SO_LAM;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            S.st[(k - 1) * SK + SO_LAM + r] += Atw_el(lam, r, ck, sk, dt);
        }
        LMPC_SYNC();
    }
}

// Interior-point stage data: T = I (stance) / 0 (swing), up = 0, so Rr = Rt (identity for a swing
// leg), Bt = G0_j masked by contact, dv = -g dt e5.
template <int LS>
__device__ __forceinline__ void leg_stage_prep_ipm(const DevParams& prm, const Smem& S, gdouble* gs, const bool (&valid)[LS],
                                                   const bool (&st)[LS], const int (&lsk)[LS], const int (&lsj)[LS],
                                                   const double (&Rt)[LS][6]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        if (!valid[t]) continue;
        const int k = lsk[t], j = lsj[t];
        gdouble* gl = gs + k * GS;
        const double on = st[t] ? 1.0 : 0.0, off = 1.0 - on;
        const double R3[9] = {Rt[t][0], Rt[t][1], Rt[t][2], Rt[t][1], Rt[t][3], Rt[t][4], Rt[t][2], Rt[t][4], Rt[t][5]};
#pragma unroll
        for (int e = 0; e < 9; ++e) gl[GO_RR + j * 9 + e] = on * R3[e] + ((e % 4 == 0) ? off : 0.0);
        gl[GO_ACT + j] = on;
#pragma unroll
        for (int m = 0; m < 6; ++m)
#pragma unroll
            for (int a = 0; a < 3; ++a) gl[GO_BT + m * 12 + 3 * j + a] = on * S.G0[m * 12 + 3 * j + a];
        if (j == 0) {
#pragma unroll
            for (int m = 0; m < 6; ++m) gl[GO_DV + m] = (m == 5) ? -prm.grav * prm.dt : 0.0;
        }
    }
}

// Per-leg-step stage data: Rr = T'RtT (fixed components -> identity), Bt = G0_j T, dv (quad-reduced).
// Rt is the symmetric input Hessian block [xx xy xz yy yz zz].  Must be called by ALL lanes.
template <int LS>
__device__ __forceinline__ void leg_stage_prep(const DevParams& prm, const Smem& S, gdouble* gs, const bool (&valid)[LS],
                                               const int (&lsk)[LS], const int (&lsj)[LS], const double (&Rt)[LS][6],
                                               const double (&T)[LS][9], const double (&up)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        double du[6] = {0, 0, 0, 0, 0, 0};
        if (valid[t]) {
            const int k = lsk[t], j = lsj[t];
            gdouble* gl = gs + k * GS;
            const double R3[9] = {Rt[t][0], Rt[t][1], Rt[t][2], Rt[t][1], Rt[t][3], Rt[t][4], Rt[t][2], Rt[t][4], Rt[t][5]};
            bool fixed[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) fixed[a] = (T[t][a] == 0.0 && T[t][3 + a] == 0.0 && T[t][6 + a] == 0.0);
            gl[GO_ACT + j] = (fixed[0] && fixed[1] && fixed[2]) ? 0.0 : 1.0;
            double RT[9];  // Rt T
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    RT[p * 3 + b] = R3[p * 3 + 0] * T[t][0 * 3 + b] + R3[p * 3 + 1] * T[t][1 * 3 + b] + R3[p * 3 + 2] * T[t][2 * 3 + b];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    double v = T[t][0 * 3 + a] * RT[0 * 3 + b] + T[t][1 * 3 + a] * RT[1 * 3 + b] + T[t][2 * 3 + a] * RT[2 * 3 + b];
                    if (fixed[a] || fixed[b]) v = (a == b) ? 1.0 : 0.0;
                    gl[GO_RR + j * 9 + a * 3 + b] = v;
                }
#pragma unroll
            for (int m = 0; m < 6; ++m) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double v = 0.0;
#pragma unroll
                    for (int p = 0; p < 3; ++p) v += S.G0[m * 12 + 3 * j + p] * T[t][p * 3 + a];
                    gl[GO_BT + m * 12 + 3 * j + a] = v;
                }
                double d = 0.0;
#pragma unroll
                for (int p = 0; p < 3; ++p) d += S.G0[m * 12 + 3 * j + p] * up[t][p];
                du[m] = d;
            }
        }
#pragma unroll
        for (int m = 0; m < 6; ++m) du[m] = quad_sum(du[m]);
        if (valid[t] && lsj[t] == 0) {
            gdouble* gl = gs + lsk[t] * GS;
#pragma unroll
            for (int m = 0; m < 6; ++m) gl[GO_DV + m] = du[m] - (m == 5 ? prm.grav * prm.dt : 0.0);
        }
    }
}

// rr = T'(Rt up + rt) per leg-step -> SO_RRV
template <int LS>
__device__ __forceinline__ void leg_rhs(const Smem& S, const bool (&valid)[LS], const int (&lsk)[LS],
                                        const int (&lsj)[LS], const double (&Rt)[LS][6], const double (&rt)[LS][3],
                                        const double (&T)[LS][9], const double (&up)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        if (!valid[t]) continue;
        const double R3[9] = {Rt[t][0], Rt[t][1], Rt[t][2], Rt[t][1], Rt[t][3], Rt[t][4], Rt[t][2], Rt[t][4], Rt[t][5]};
        double e[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
            e[p] = rt[t][p] + R3[p * 3 + 0] * up[t][0] + R3[p * 3 + 1] * up[t][1] + R3[p * 3 + 2] * up[t][2];
        ldouble* rr = S.st + lsk[t] * SK + SO_RRV + 3 * lsj[t];
#pragma unroll
        for (int a = 0; a < 3; ++a) rr[a] = T[t][a] * e[0] + T[t][3 + a] * e[1] + T[t][6 + a] * e[2];
    }
}

// interior-point variants (T = I for a stance leg, 0 for a swing leg; up = 0): rr = rt, u = y
template <int LS>
__device__ __forceinline__ void leg_rhs_ipm(const Smem& S, const bool (&valid)[LS], const bool (&st)[LS],
                                            const int (&lsk)[LS], const int (&lsj)[LS], const double (&rt)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        if (!valid[t]) continue;
        ldouble* rr = S.st + lsk[t] * SK + SO_RRV + 3 * lsj[t];
#pragma unroll
        for (int a = 0; a < 3; ++a) rr[a] = st[t] ? rt[t][a] : 0.0;
    }
}
template <int LS>
__device__ __forceinline__ void leg_u_ipm(const Smem& S, const bool (&valid)[LS], const bool (&st)[LS],
                                          const int (&lsk)[LS], const int (&lsj)[LS], double (&u)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        u[t][0] = u[t][1] = u[t][2] = 0.0;
        if (!valid[t] || !st[t]) continue;
        const ldouble* y = S.st + lsk[t] * SK + SO_RRV + 3 * lsj[t];
#pragma unroll
        for (int p = 0; p < 3; ++p) u[t][p] = y[p];
    }
}

// u = up + T y (y from SO_RRV after riccati_solve)
template <int LS>
__device__ __forceinline__ void leg_u(const Smem& S, const bool (&valid)[LS], const int (&lsk)[LS], const int (&lsj)[LS],
                                      const double (&T)[LS][9], const double (&up)[LS][3], double (&u)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        u[t][0] = u[t][1] = u[t][2] = 0.0;
        if (!valid[t]) continue;
        const ldouble* y = S.st + lsk[t] * SK + SO_RRV + 3 * lsj[t];
#pragma unroll
        for (int p = 0; p < 3; ++p) u[t][p] = up[t][p] + T[t][p * 3] * y[0] + T[t][p * 3 + 1] * y[1] + T[t][p * 3 + 2] * y[2];
    }
}

// ---------------------------------------------------------------------------
// The fused per-QP kernel.  LS = leg-steps owned per lane = ceil(4H / 64).
//
// TERRAIN (extension): each leg's force variable is its contact-frame force
// g = R_j'f (R_j = terrain_frame(n_j)), so the reference's pyramid/bound code below runs
// unchanged on g.  What changes: the input matrix G0 -> G0 blkdiag(R_j), the input Hessian
// block diag(r_j) -> R_j' diag(r_j) R_j, and the output f = R_j g.  R_j = I for n_j = e_z.
// ---------------------------------------------------------------------------
// WPE = waves per SIMD the register budget allows: 1 (512 VGPR+AGPR per lane, few spills) or 2 (256,
// some spills).  A lone wave is latency-bound, so a second one per SIMD nearly doubles the issue rate;
// it pays once the LDS admits more than 4 QPs per CU (H <= 16; launch_qp picks the instance).
template <int LS, bool TERRAIN, int WPE>
__global__ void __launch_bounds__(64, WPE) lmpc_qp_kernel(const DevParams prm, const double* __restrict__ rec,
                                                     const uint8_t* __restrict__ contact,
                                                     const double* __restrict__ normals, int batch,
                                                     double* __restrict__ grf, int32_t* __restrict__ status,
                                                     int32_t* __restrict__ iters, double* __restrict__ scratch,
                                                     const uint8_t* __restrict__ dense_done) {
    extern __shared__ __attribute__((aligned(16))) double lmpc_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    if (prm.dense) {  // QPs with 1..DENSE_MAX_LS stance leg-steps went to a dense-path kernel (H <= 16 here)
        const bool stl = lane < 4 * H && contact[(size_t)qp * 4 * H + lane] != 0;
        const int n = __popcll(__ballot(stl));
        // the GI kernel flags the QPs it solved; the ones it left (step cap, non-finite step) are solved here
        if (n >= 1 && n <= DENSE_MAX_LS && (!dense_done || dense_done[qp])) return;
    }
    const int RL = 33 + 12 * H;
    Smem S = carve(lmpc_smem, H);
    ldouble* const tf = S.st + SK * H;  // TERRAIN only: R_j (9 each, row-major) | R_j' diag(r_j) R_j packed (6 each)
    double* gs = scratch + (size_t)qp * GS * H;
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;
    STAMP_DECL

    // ---- load the record (coalesced, one pass) ----
    const double* rin = rec + (size_t)qp * RL;
    if (lane < 33) S.hdr[lane] = rin[lane];
    S.xr = (const gdouble*)(rin + 33);
    if constexpr (TERRAIN) {
        if (lane < 4) {
            // contact frame of leg `lane` (same closed form as lmpc_terrain_frame, lmpc_host.cpp)
            const double* nin = normals + (size_t)qp * 12 + 3 * lane;
            const double n0 = nin[0], n1 = nin[1], n2 = nin[2];
            const double nn = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
            const double nx = n0 / nn, ny = n1 / nn, c = n2 / nn;
            const double h = 1.0 / (1.0 + c);
            const double R[9] = {1.0 - nx * nx * h, -nx * ny * h, nx, -nx * ny * h, 1.0 - ny * ny * h, ny, -nx, -ny, c};
#pragma unroll
            for (int e = 0; e < 9; ++e) tf[9 * lane + e] = R[e];
            const double r0 = prm.r[3 * lane], r1 = prm.r[3 * lane + 1], r2 = prm.r[3 * lane + 2];
            int e = 0;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = a; b < 3; ++b)  // packed [xx xy xz yy yz zz]
                    tf[36 + 6 * lane + e++] = r0 * R[a] * R[b] + r1 * R[3 + a] * R[3 + b] + r2 * R[6 + a] * R[6 + b];
        }
    }
    LMPC_SYNC();
    double iw[9];  // (R I_b R')^-1, computed redundantly by every lane
    {
        const ldouble* R = S.hdr + LMPC_REC_ROT;
        double RI[9], Iw[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                RI[i * 3 + j] = R[i * 3 + 0] * prm.Ib[0 * 3 + j] + R[i * 3 + 1] * prm.Ib[1 * 3 + j] + R[i * 3 + 2] * prm.Ib[2 * 3 + j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Iw[i * 3 + j] = RI[i * 3 + 0] * R[j * 3 + 0] + RI[i * 3 + 1] * R[j * 3 + 1] + RI[i * 3 + 2] * R[j * 3 + 2];
        const double c00 = Iw[4] * Iw[8] - Iw[5] * Iw[7];
        const double c01 = Iw[5] * Iw[6] - Iw[3] * Iw[8];
        const double c02 = Iw[3] * Iw[7] - Iw[4] * Iw[6];
        const double id = 1.0 / (Iw[0] * c00 + Iw[1] * c01 + Iw[2] * c02);
        iw[0] = c00 * id;
        iw[1] = (Iw[2] * Iw[7] - Iw[1] * Iw[8]) * id;
        iw[2] = (Iw[1] * Iw[5] - Iw[2] * Iw[4]) * id;
        iw[3] = c01 * id;
        iw[4] = (Iw[0] * Iw[8] - Iw[2] * Iw[6]) * id;
        iw[5] = (Iw[2] * Iw[3] - Iw[0] * Iw[5]) * id;
        iw[6] = c02 * id;
        iw[7] = (Iw[1] * Iw[6] - Iw[0] * Iw[7]) * id;
        iw[8] = (Iw[0] * Iw[4] - Iw[1] * Iw[3]) * id;
    }
    for (int k = lane; k < H; k += 64) {
        double sn, cn;
        sincos(S.xr[12 * k + 2], &sn, &cn);
        S.cs[2 * k] = cn;
        S.cs[2 * k + 1] = sn;
    }
    // G0 = dt [I_w^-1 skew(r_j) ; I/m]  (Utils::skew, Utils.cpp:89-95)
    for (int e = lane; e < 72; e += 64) {
        const int r = e / 12, c = e % 12, j = c / 3, cc = c % 3;
        double v;
        if constexpr (!TERRAIN) {
            if (r < 3) {
                const ldouble* ft = S.hdr + LMPC_REC_FEET + 3 * j;
                double sk[3];  // column cc of skew(ft)
                if (cc == 0) { sk[0] = 0.0; sk[1] = ft[2]; sk[2] = -ft[1]; }
                else if (cc == 1) { sk[0] = -ft[2]; sk[1] = 0.0; sk[2] = ft[0]; }
                else { sk[0] = ft[1]; sk[1] = -ft[0]; sk[2] = 0.0; }
                v = dt * (iw[r * 3 + 0] * sk[0] + iw[r * 3 + 1] * sk[1] + iw[r * 3 + 2] * sk[2]);
            } else {
                v = (r - 3 == cc) ? dt / prm.mass : 0.0;
            }
        } else {
            // (G0 R_j)[r][cc] = sum_p G0[r][3j+p] R_j[p][cc]
            const ldouble* Rj = tf + 9 * j;
            if (r < 3) {
                const ldouble* ft = S.hdr + LMPC_REC_FEET + 3 * j;
                // row r of dt I_w^-1 skew(ft): w_p = dt (iw[r,:] . skew column p)
                const double w0 = dt * (iw[r * 3 + 1] * ft[2] - iw[r * 3 + 2] * ft[1]);
                const double w1 = dt * (-iw[r * 3 + 0] * ft[2] + iw[r * 3 + 2] * ft[0]);
                const double w2 = dt * (iw[r * 3 + 0] * ft[1] - iw[r * 3 + 1] * ft[0]);
                v = w0 * Rj[cc] + w1 * Rj[3 + cc] + w2 * Rj[6 + cc];
            } else {
                v = (dt / prm.mass) * Rj[3 * (r - 3) + cc];
            }
        }
        S.G0[e] = v;
    }
    if (lane < 12) S.qw[lane] = prm.q[lane];
    if (lane < 16) S.zero[lane] = 0.0;
    for (int k = lane; k < H; k += 64) {
        gs[k * GS + GO_ZERO] = gs[k * GS + GO_ZERO + 1] = 0.0;
    }
    LMPC_SYNC();

    // ---- leg-step ownership and IPM state ----
    bool st[LS], valid[LS];
    int lsk[LS], lsj[LS];
    double f[LS][3], s[LS][5], z[LS][5];
    double T[LS][9], up[LS][3], Rt[LS][6], rt[LS][3], u[LS][3];
    int nst_loc = 0;
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        const int ls = lane + 64 * t;
        valid[t] = ls < 4 * H;
        lsk[t] = valid[t] ? (ls >> 2) : 0;
        lsj[t] = ls & 3;
        st[t] = valid[t] && contact[(size_t)qp * 4 * H + ls] != 0;
        nst_loc += st[t] ? 1 : 0;
        f[t][0] = f[t][1] = 0.0;
        {
            // starting point: each stance leg carries its share of the weight (fz = m g / n_stance,
            // capped at fmax/2), zero tangential force; slacks from the constraints and a
            // centred z = 1/s (s z = 1).  Measured: ~0.9 fewer interior-point iterations on
            // average than fz = fmax/2, z = 1 (tools/variant_sweep.py, profiles/r01_init_sweep.log).
            const double cnt = quad_sum(st[t] ? 1.0 : 0.0);  // stance legs of this stage (all lanes: DPP)
            f[t][2] = st[t] ? fmin(0.5 * fzmax, prm.mass * prm.grav / fmax(cnt, 1.0)) : 0.0;
        }
        double o[5];
        cons_resid(f[t], mu, fzmax, o);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            s[t][i] = st[t] ? -o[i] : 1.0;
            z[t][i] = 1.0 / s[t][i];
        }
        u[t][0] = u[t][1] = u[t][2] = 0.0;
    }
    const double nst = wave_sum((double)nst_loc);
    STAMP(0);  // prologue
    int qstatus = LMPC_QP_CONVERGED;
    int ipm_it = 0, prounds = 0;
    bool done = false;
    int act_fin[LS];  // verified active set (warm-start output); 0 = none / unconstrained
#pragma unroll
    for (int t = 0; t < LS; ++t) act_fin[t] = 0;
    if (nst > 0.5) {
        // One loop, three modes, so that factor / solve / adjoint are each
        // instantiated once (keeps the code object small for the I-cache).
        enum { PRED = 0, CORR = 1, POLISH = 2 };
        const double mc = 5.0 * nst;
        double tol = prm.tol_mu;
        int att = 0, rd = 0, it_end = prm.max_iter;
        int mode = PRED;
        int act[LS];
        bool apex[LS];
        // warm start: straight into the polish from the given active set (the caller's previous solution)
        bool warm = prm.warm_act != nullptr;
        if (warm) {
#pragma unroll
            for (int t = 0; t < LS; ++t) {
                const int ls = lane + 64 * t;
                act[t] = st[t] ? (prm.warm_act[(size_t)qp * 4 * H + ls] & 31) : 0;
            }
            mode = POLISH;
        }
        double ua[LS][3];  // predictor step u_aff: the only predictor state kept across the corrector solve
#pragma unroll
        for (int t = 0; t < LS; ++t) ua[t][0] = ua[t][1] = ua[t][2] = 0.0;
        double mu_c = 0.0, smu = 0.0;
        SUB_DECL
        for (;;) {
            if (mode == PRED) {
                double loc = 0.0;
#pragma unroll
                for (int t = 0; t < LS; ++t)
                    if (st[t])
#pragma unroll
                        for (int i = 0; i < 5; ++i) loc += s[t][i] * z[t][i];
                mu_c = wave_sum(loc) / mc;
                if (mu_c < tol || ipm_it >= it_end) {
                    // active set from the interior point: z > LMPC_ACT_RATIO s, lift-off legs -> apex
#pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        act[t] = 0;
                        if (!st[t]) continue;
#pragma unroll
                        for (int i = 0; i < 5; ++i)
                            if (z[t][i] > LMPC_ACT_RATIO * s[t][i]) act[t] |= 1 << i;
                        const double fm = fmax(fabs(f[t][0]), fmax(fabs(f[t][1]), fabs(f[t][2])));
                        if (fm < 1e-6 * fzmax) act[t] = 15;
                    }
                    mode = POLISH;
                    rd = 0;
                } else {
                    // stage data: Rt = diag(r) + C'WC, rt = C'(W(s-b)), T = I (stance) / 0 (swing), up = 0
#pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        double W[5] = {0, 0, 0, 0, 0}, wv[5] = {0, 0, 0, 0, 0};
                        if (st[t]) {
#pragma unroll
                            for (int i = 0; i < 5; ++i) {
                                W[i] = z[t][i] * rcp_nr(s[t][i]);  // 1/s is recomputed where needed: keeping it
                                                                    // live across the factor/solve calls spills it
                                wv[i] = W[i] * (s[t][i] - (i == 4 ? fzmax : 0.0));
                            }
                        }
                        const double sx = W[0] + W[1], sy = W[2] + W[3];
                        const int j = lsj[t];
                        if constexpr (!TERRAIN) {
                            Rt[t][0] = prm.r[3 * j + 0] + sx;
                            Rt[t][1] = 0.0;
                            Rt[t][2] = mu * (W[0] - W[1]);
                            Rt[t][3] = prm.r[3 * j + 1] + sy;
                            Rt[t][4] = mu * (W[2] - W[3]);
                            Rt[t][5] = prm.r[3 * j + 2] + mu * mu * (sx + sy) + W[4];
                        } else {
                            const ldouble* rb = tf + 36 + 6 * j;
                            Rt[t][0] = rb[0] + sx;
                            Rt[t][1] = rb[1];
                            Rt[t][2] = rb[2] + mu * (W[0] - W[1]);
                            Rt[t][3] = rb[3] + sy;
                            Rt[t][4] = rb[4] + mu * (W[2] - W[3]);
                            Rt[t][5] = rb[5] + mu * mu * (sx + sy) + W[4];
                        }
                        cons_tw(wv, mu, rt[t]);
                    }
                }
            }
            if (mode == POLISH) {
                ++prounds;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    apex[t] = false;
                    if (st[t]) {
                        apex[t] = leg_basis(act[t], mu, fzmax, T[t], up[t]);
                    } else {
#pragma unroll
                        for (int i = 0; i < 9; ++i) T[t][i] = 0.0;
                        up[t][0] = up[t][1] = up[t][2] = 0.0;
                    }
                    const int j = lsj[t];
                    if constexpr (!TERRAIN) {
                        Rt[t][0] = prm.r[3 * j];
                        Rt[t][1] = Rt[t][2] = 0.0;
                        Rt[t][3] = prm.r[3 * j + 1];
                        Rt[t][4] = 0.0;
                        Rt[t][5] = prm.r[3 * j + 2];
                    } else {
#pragma unroll
                        for (int e = 0; e < 6; ++e) Rt[t][e] = tf[36 + 6 * j + e];
                    }
                    rt[t][0] = rt[t][1] = rt[t][2] = 0.0;
                }
            }
            SUB(13);  // (diagnostic) leg-step bookkeeping since the previous solve
            if (mode == PRED) leg_stage_prep_ipm<LS>(prm, S, (gdouble*)gs, valid, st, lsk, lsj, Rt);
            else if (mode == POLISH) leg_stage_prep<LS>(prm, S, (gdouble*)gs, valid, lsk, lsj, Rt, T, up);
            if (mode == POLISH) leg_rhs<LS>(S, valid, lsk, lsj, Rt, rt, T, up);
            else leg_rhs_ipm<LS>(S, valid, st, lsk, lsj, rt);
            LMPC_GSYNC();  // stage data (partly in the global scratch) visible to every lane
            SUB(14);  // (diagnostic) stage prep + rhs
            STAMP(1);  // leg-step work (IPM/polish bookkeeping, stage prep)
            if (mode != CORR) riccati_factor<WPE>(S, (gdouble*)gs, H, dt, lane);
            STAMP(2);  // factorisation
            switch ((12 * H + 63) / 64) {
                case 1: riccati_solve<1, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
                case 2: riccati_solve<2, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
                case 3: riccati_solve<3, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
                case 4: riccati_solve<4, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
                case 5: riccati_solve<5, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
                default: riccati_solve<6, WPE>(S, (const gdouble*)gs, H, dt, lane); break;
            }
            STAMP(3);  // vector pass
            SUB(15);   // (diagnostic) factor + solve, already split by their own stamps
            if (mode == POLISH) leg_u<LS>(S, valid, lsk, lsj, T, up, u);
            else leg_u_ipm<LS>(S, valid, st, lsk, lsj, u);
            SUB(16);   // (diagnostic) leg_u
            if (mode == PRED) {
                double amax = 1.0;
                double dsa[LS][5], dza[LS][5];
#pragma unroll
                for (int t = 0; t < LS; ++t) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) dsa[t][i] = dza[t][i] = 0.0;
#pragma unroll
                    for (int m = 0; m < 3; ++m) ua[t][m] = u[t][m];
                    if (!st[t]) continue;
                    double o[5];
                    cons_resid(u[t], mu, fzmax, o);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        dsa[t][i] = -o[i] - s[t][i];
                        dza[t][i] = -z[t][i] - z[t][i] * rcp_nr(s[t][i]) * dsa[t][i];
                        // fraction to the boundary: the hardware reciprocal estimate is ample here
                        if (dsa[t][i] < 0.0) amax = fmin(amax, -s[t][i] * __builtin_amdgcn_rcp(dsa[t][i]));
                        if (dza[t][i] < 0.0) amax = fmin(amax, -z[t][i] * __builtin_amdgcn_rcp(dza[t][i]));
                    }
                }
                const double aa = wave_min(amax);
                double loc = 0.0;
#pragma unroll
                for (int t = 0; t < LS; ++t)
                    if (st[t])
#pragma unroll
                        for (int i = 0; i < 5; ++i) loc += (s[t][i] + aa * dsa[t][i]) * (z[t][i] + aa * dza[t][i]);
                const double ratio = (wave_sum(loc) / mc) / mu_c;
                smu = ratio * ratio * ratio * mu_c;
                // corrector right-hand side
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    double wv[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        wv[i] = (z[t][i] * (s[t][i] - (i == 4 ? fzmax : 0.0)) + smu - dsa[t][i] * dza[t][i]) * rcp_nr(s[t][i]);
                    cons_tw(wv, mu, rt[t]);
                }
                mode = CORR;
                SUB(17);  // (diagnostic) predictor post-step
            } else if (mode == CORR) {
                double ds[LS][5], dz[LS][5];
                double amax = 1.0, dmax = 1.0;  // primal (s) and dual (z) distances to the boundary
#pragma unroll
                for (int t = 0; t < LS; ++t) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) ds[t][i] = dz[t][i] = 0.0;
                    if (!st[t]) continue;
                    double o[5], oa[5];
                    cons_resid(u[t], mu, fzmax, o);
                    cons_resid(ua[t], mu, fzmax, oa);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        const double is = rcp_nr(s[t][i]);
                        const double dsa = -oa[i] - s[t][i];  // predictor step, recomputed from u_aff
                        const double dza = -z[t][i] - z[t][i] * is * dsa;
                        ds[t][i] = -o[i] - s[t][i];
                        dz[t][i] = (smu - z[t][i] * s[t][i] - dsa * dza - z[t][i] * ds[t][i]) * is;
                        if (ds[t][i] < 0.0) amax = fmin(amax, -s[t][i] * __builtin_amdgcn_rcp(ds[t][i]));
                        if (dz[t][i] < 0.0) dmax = fmin(dmax, -z[t][i] * __builtin_amdgcn_rcp(dz[t][i]));
                    }
                }
#if LMPC_SPLIT_STEP
                const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(amax));
                const double alpd = fmin(1.0, LMPC_STEP_FRAC * wave_min(dmax));
#else
                const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(fmin(amax, dmax))), alpd = alpha;
#endif
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
#pragma unroll
                    for (int m = 0; m < 3; ++m) f[t][m] += alpha * (u[t][m] - f[t][m]);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        s[t][i] += alpha * ds[t][i];
                        z[t][i] += alpd * dz[t][i];
                    }
                }
                ++ipm_it;
                mode = PRED;
                SUB(18);  // (diagnostic) corrector post-step
            } else {
                // ---- polish verification, a KKT certificate independent of the factorisation (lmpc_lq.hip): the
                // trajectory is the dynamics of the forces returned, the adjoint of that trajectory gives the
                // gradient, every stance leg-step is primal feasible, stationary on its free directions and carries
                // multipliers of the right sign ----
                STAMP(1);
                double dres = 0.0, xsc = 1.0;  // dynamics residual, state scale (max |x|, at least 1)
                {
                    // B u_k per stage -> SO_N6 (dead after the solve)
#pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        const int j = lsj[t];
                        double bu[6];
#pragma unroll
                        for (int m = 0; m < 6; ++m)
                            bu[m] = quad_sum(fma(S.G0[m * 12 + 3 * j], u[t][0],
                                                 fma(S.G0[m * 12 + 3 * j + 1], u[t][1], S.G0[m * 12 + 3 * j + 2] * u[t][2])));
                        if (valid[t] && j == 0) {
#pragma unroll
                            for (int m = 0; m < 6; ++m) S.st[lsk[t] * SK + SO_N6 + m] = bu[m];
                        }
                    }
                    LMPC_SYNC();
                    constexpr int MAXT = (12 * LMPC_MAX_HORIZON + 63) / 64;
#pragma unroll 1
                    for (int i = 0; i < MAXT; ++i) {
                        if (64 * i >= 12 * H) break;  // wave-uniform
                        const int e = lane + 64 * i, ec = e < 12 * H ? e : 12 * H - 1;
                        const int k = ec / 12, r = ec - 12 * k;
                        const ldouble* xk = S.st + k * SK + SO_XS;
                        const double xn = k + 1 < H ? S.st[(k + 1) * SK + SO_XS + r] : S.xH[r];
                        const int m = r >= 6 ? r - 6 : 0;
                        const double bu = S.st[k * SK + SO_N6 + m] - (m == 5 ? prm.grav * dt : 0.0);
                        const double pred = Ax_el(xk, r, S.cs[2 * k], S.cs[2 * k + 1], dt) + (r >= 6 ? bu : 0.0);
                        if (e < 12 * H) {
                            dres = fmax(dres, fabs(xn - pred));
                            xsc = fmax(xsc, fabs(xn));
                        }
                    }
                }
                adjoint(prm, S, lane);
                STAMP(4);  // adjoint
                double g[LS][3];
                double gloc = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    g[t][0] = g[t][1] = g[t][2] = 0.0;
                    if (!valid[t]) continue;
                    const int k = lsk[t], j = lsj[t];
                    const ldouble* lam = S.st + k * SK + SO_LAM;
                    double ru[3];  // input-Hessian block times u
                    if constexpr (!TERRAIN) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) ru[p] = prm.r[3 * j + p] * u[t][p];
                    } else {
                        const ldouble* rb = tf + 36 + 6 * j;
                        ru[0] = rb[0] * u[t][0] + rb[1] * u[t][1] + rb[2] * u[t][2];
                        ru[1] = rb[1] * u[t][0] + rb[3] * u[t][1] + rb[4] * u[t][2];
                        ru[2] = rb[2] * u[t][0] + rb[4] * u[t][1] + rb[5] * u[t][2];
                    }
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        double v = ru[p];
#pragma unroll
                        for (int m = 0; m < 6; ++m) v += S.G0[m * 12 + 3 * j + p] * lam[6 + m];
                        g[t][p] = v;
                        gloc = fmax(gloc, fabs(v));
                    }
                }
                const double gscale = wave_max(gloc);
                int changed = 0;
                double sres = 0.0;  // stationarity residual on the free directions of the stance leg-steps
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    double o[5];
                    cons_resid(u[t], mu, fzmax, o);
                    int imax = -1;
                    double vmax = prm.tol_p * fzmax;
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        if (!((act[t] >> i) & 1) && o[i] > vmax) {
                            vmax = o[i];
                            imax = i;
                        }
                    if (imax >= 0) {
                        act[t] |= 1 << imax;
                        changed = 1;
                        continue;
                    }
                    if (apex[t]) {  // the cone test is the whole certificate at the apex
                        if (g[t][2] / mu < fabs(g[t][0]) + fabs(g[t][1]) - prm.tol_d * gscale) {
                            act[t] = (g[t][0] < 0.0 ? 2 : 1) | (g[t][1] < 0.0 ? 8 : 4);
                            changed = 1;
                        }
                        continue;
                    }
                    // multipliers: C_S' z = -g, C_S full row rank (<= 3 rows; act = 0: none, the residual is g)
                    const LegKkt kk = leg_kkt(act[t], g[t], mu, -prm.tol_d * gscale);
                    if (kk.drop >= 0) {
                        act[t] &= ~(1 << kk.drop);
                        changed = 1;
                    }
                    sres = fmax(sres, kk.res);
                }
                bool settled = false;  // the active set no longer changes, but the certificate failed
                if (!__any(changed)) {
                    const double sr = wave_max(sres), dr = wave_max(dres), xs = wave_max(xsc);
#ifndef LMPC_KKT_OFF
                    if (sr <= prm.tol_d * gscale && dr <= prm.tol_x * xs)
#endif
                    {
                        done = true;
#pragma unroll
                        for (int t = 0; t < LS; ++t) act_fin[t] = st[t] ? act[t] : 0;
                        break;
                    }
                    settled = true;  // another round would repeat it bit for bit: the retry ladder takes over
                }
                if (settled) rd = (warm ? prm.warm_rounds : prm.max_rounds) - 1;
                if (++rd >= (warm ? prm.warm_rounds : prm.max_rounds)) {
                    if (warm) {  // the warm active set did not verify: the cold interior point
                        warm = false;
                        rd = 0;
                        mode = PRED;
                        continue;
                    }
                    // retry: tighter interior point, then a fresh polish
                    if (++att >= prm.max_attempts) break;
                    tol = retry_tol(tol, att);
                    it_end += prm.max_iter;
                    mode = PRED;
                }
            }
        }
    } else {
        done = true;
    }
    if (!done) {
        // no verified active set: return the (feasible) interior-point iterate
        qstatus = LMPC_QP_MAX_ITER;
#pragma unroll
        for (int t = 0; t < LS; ++t) {
            u[t][0] = f[t][0];
            u[t][1] = f[t][1];
            u[t][2] = f[t][2];
        }
    }
    STAMP(1);
    // ---- NaN guard (reference: NaN -> zeros, ConvexQPSolver.cpp:321-326) and output ----
    int bad = 0;
#pragma unroll
    for (int t = 0; t < LS; ++t)
        if (valid[t]) bad |= (u[t][0] != u[t][0] || u[t][1] != u[t][1] || u[t][2] != u[t][2]) ? 1 : 0;
    const bool anybad = __any(bad);
    double* gout = grf + (size_t)qp * 12 * H;
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        if (!valid[t]) continue;
        const int ls = lane + 64 * t;
        double fo[3] = {u[t][0], u[t][1], u[t][2]};
        if constexpr (TERRAIN) {  // f = R_j g (world frame)
            const ldouble* Rj = tf + 9 * lsj[t];
#pragma unroll
            for (int p = 0; p < 3; ++p) fo[p] = Rj[3 * p] * u[t][0] + Rj[3 * p + 1] * u[t][1] + Rj[3 * p + 2] * u[t][2];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) gout[3 * ls + p] = (anybad || !st[t]) ? 0.0 : fo[p];
    }
    STAMP(5);  // epilogue
    STAMP_FLUSH(qp);
    if (prm.act_out) {
#pragma unroll
        for (int t = 0; t < LS; ++t)
            if (valid[t]) prm.act_out[(size_t)qp * 4 * H + lane + 64 * t] = (uint8_t)(anybad ? 0 : act_fin[t]);
    }
    if (lane == 0) {
        if (status) status[qp] = anybad ? LMPC_QP_NAN : qstatus;
        if (iters) iters[qp] = ipm_it | (prounds << 16);
    }
}

#define LMPC_INST(LS_, T_, W_)                                                                                         \
    template __global__ void lmpc_qp_kernel<LS_, T_, W_>(const DevParams, const double*, const uint8_t*, const double*, \
                                                         int, double*, int32_t*, int32_t*, double*, const uint8_t*);
LMPC_INST(1, false, 1)
LMPC_INST(1, false, 2)
LMPC_INST(2, false, 1)
LMPC_INST(1, true, 1)
LMPC_INST(1, true, 2)
LMPC_INST(2, true, 1)
#undef LMPC_INST

template <int LS, bool TERRAIN, int WPE>
static void launch_variant(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                           int batch, double* grf, int32_t* status, int32_t* iters, double* scratch,
                           const uint8_t* done, hipStream_t stream) {
    const size_t lds = lds_bytes(prm.H, TERRAIN);
    const dim3 grid(batch), block(LMPC_WAVE);  // LMPC_SYNC() relies on exactly one wavefront per workgroup
    (void)hipFuncSetAttribute((const void*)lmpc_qp_kernel<LS, TERRAIN, WPE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lmpc_qp_kernel<LS, TERRAIN, WPE>), grid, block, lds, stream, prm, rec, contact, normals, batch,
                       grf, status, iters, scratch, done);
}

// Host-side launcher (called from lmpc_capi.cpp).  normals == nullptr: flat ground (the reference).
hipError_t launch_qp(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                     int batch, double* grf, int32_t* status, int32_t* iters, double* scratch, const uint8_t* done,
                     hipStream_t stream) {
    const bool two = 4 * prm.H > 64;
    // two waves per SIMD when more than 4 QPs fit the CU's LDS and the batch has more QPs than the
    // device has SIMDs (up to one QP per SIMD the lone-wave instance, free of spills, is faster); H <= 16
    // only: the LS = 2 state spills too much at 256 registers (measured at H = 20, 5 QPs per CU: 22 %
    // slower than 4 at one wave per SIMD).  Same arithmetic, so the choice never changes a result bit.
#ifdef LMPC_AB_NO_W2  // diagnostic variant (tools/ab_bench.sh): the lone-wave instance only
    const bool w2 = false;
#else
    const bool w2 = !two && 5 * lds_bytes(prm.H, normals != nullptr) <= LMPC_CU_LDS_BYTES && batch > 4 * prm.cus;
#endif
#define LMPC_LAUNCH(LS_, T_, W_) \
    launch_variant<LS_, T_, W_>(prm, rec, contact, normals, batch, grf, status, iters, scratch, done, stream)
    if (normals) {
        if (two) LMPC_LAUNCH(2, true, 1);
        else w2 ? LMPC_LAUNCH(1, true, 2) : LMPC_LAUNCH(1, true, 1);
    } else {
        if (two) LMPC_LAUNCH(2, false, 1);
        else w2 ? LMPC_LAUNCH(1, false, 2) : LMPC_LAUNCH(1, false, 1);
    }
#undef LMPC_LAUNCH
    return hipGetLastError();
}

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_substamps(unsigned long long* out, int nqp) {
    if (nqp > STAMP_QPS) nqp = STAMP_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_substamps), (size_t)nqp * 24 * sizeof(unsigned long long)) == hipSuccess ? nqp : -1;
}
extern "C" int lmpc_debug_stamps(unsigned long long* out, int nqp) {
    if (nqp > STAMP_QPS) nqp = STAMP_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_stamps), (size_t)nqp * 8 * sizeof(unsigned long long)) == hipSuccess ? nqp : -1;
}
#endif

}  // namespace lmpc

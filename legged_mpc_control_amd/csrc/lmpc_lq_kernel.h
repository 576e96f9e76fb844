// lmpc_lq_kernel.h -- the LDS-resident Riccati solve of one QP (lq_body) and its helpers, shared by the Riccati
// kernel (lmpc_lq.hip) and the fused dense + Riccati kernel (lmpc_fused.hip).  The algorithm (round 4):
//
// One 64-lane wavefront per QP, no global scratch and no outlined calls: the per-stage factors the vector passes
// need are kept in a 135-double LDS slot per stage (14.4 KB per QP at H = 10: eight QPs -- two waves per SIMD --
// share a CU; 36 KB at H = 30: four), and everything else lives in registers.  The QP, the interior point and the
// polish are those of lmpc_kernels.hip (ConvexQPSolver.cpp:16-346 restated); what changes is how the
// Newton systems are solved (numpy replica step for step: tools/lq_proto.py, RED6=1):
//
//   reduced inputs (interior point): a stage's 12 inputs reach the dynamics only through f = Bt u (rows 6-11), so
//   min_u {1/2 u'Rr u + rr'u : Bt u = f} = 1/2 |v|^2 + const with f = U v - g, where W = Bt Rr^-1 Bt' = U U' (6 x 6)
//   and g = Bt Rr^-1 rr: the same value function from a Riccati step with six unit-cost inputs and d' = d - E g --
//   two 3x3 pivot blocks whatever the number of stance legs, no linear input term.  W_j and g_j come from each leg's
//   lane (Rr = L L', Y = G0_j L^-T), summed over the stage's quad; U by a 6x6 Cholesky per stage (lane k).  The polish
//   keeps the full inputs (its per-leg bases T make W ill-conditioned; the polish answer must be exact).
//   factorisation (stage k = H-1 .. 0), value function of the augmented state [x; 1] in one 16x16 MFMA tile
//   (P^ = [P p; p' c]: its column 12 is the linear term p, so the backward vector pass of the right-hand side the
//   factorisation is given comes for free):
//       C   = P^ B^,  B^ rows 6-11 = [U | 0 | dv'] or [Bt | dv]  -> v = P d (column 12)
//       Guu = B' P22 B, + I or Rr_j at each 3x3 pivot (block diagonal: it enters only its own pivot block)
//       block Cholesky with L^-1 and X = L^-1 [0 | B' | r] eliminated alongside (as lmpc_kernels.hip)
//       KH  = X'X                                          -> K = V'V (rows/cols 6-11), rho = B Guu^-1 r (col 12)
//       PA  = P^ A^,  A^ = [A d; 0 1]                       -> Z = rows 6-11 of PA (6 x 13; column 12 = za = v2 + p2)
//       P^_k = Q^_k + A^'PA - M'KH M'  (M' = PA with row 12 = e12), Q^_k column 12 = -Q x_ref,k-1
//   stored per stage: Z (78; before the factorisation U or Bt), K (21, packed), rho (6), v (12), x (12), dv (6)
//   forward sweep      w = Z x + za ;  x' = A x + d - [0; K w + rho]
//   inputs (parallel)  from the costate lambda2 = Z A^-1 x' + za - v2 (= P2 x' + p2): u_j = -Rr_j^-1 (rr_j + Bt_j' lambda2)
//                      (lane-local 3x3 solves: Rr is the leg-step's own input Hessian block)
//   corrector          the new rr changes g only: rho = dg - K P22 dg (parallel; P22 recovered from Z), then the
//                      backward sweep p_k = q_k + A'y - Z'(K za + rho), y = p + v, za = y[6:12], the forward sweep
//                      and the inputs as above
//   polish check       the adjoint lambda from the trajectory (independent of the factorisation), as lmpc_kernels.hip
//
// The stage-k operands of the factorisation come from LDS (U or Bt in the Z field, rr in the x field, dv, written
// before it) and, in the polish, from the leg-step lanes' registers (Rr_j, by readlane: wave-uniform per stage and
// leg), fetched one stage ahead.  QPs the condensed dense kernel solved are skipped (its hand-over flags).
//
// The diagnostic hooks (LQ_STAMP*, LMPC_KKT_DIAG, LMPC_LQ_DEBUG) are lmpc_lq.hip's, which defines them before
// including this header; elsewhere the stamps compile to nothing (lmpc_fused.hip is built without the others).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

#ifndef LQ_STAMP
#define LQ_MARK(v) do {} while (0)
#define LQ_ADD_SINCE(i, v) do {} while (0)
#define LQ_STAMP_DECL
#define LQ_STAMP(i) do {} while (0)
#define LQ_STAMP_FLUSH(qp) do {} while (0)
#endif

namespace lmpc {


// ---- LDS layout (doubles) ----------------------------------------------------------------------------------
// per-stage slot
constexpr int LQ_Z = 0;      // 78: Z = rows 6-11 of P^_{k+1} A^_k, 6 x 13 row-major (column 12: za = v2 + p2);
                             //     before the factorisation its input: U (21, packed lower; interior point) or
                             //     Bt = G0 T (6 x 12 row-major; polish)
constexpr int LQ_K = 78;     // 21: K = Bt Guu^-1 Bt', packed lower (pk6)
constexpr int LQ_RHO = 99;   // 6:  rho; after the forward sweep lambda2 (inputs / adjoint)
constexpr int LQ_V = 105;    // 12: v = P_{k+1} d_k
constexpr int LQ_X = 117;    // 12: x_{k+1}; before a polish factorisation rr (the input linear term, 12)
constexpr int LQ_DV = 129;   // 6:  d_k[6:12] (interior point: less g = Bt Rr^-1 rr)
constexpr int LQ_SLOT = 135;
// fixed part
constexpr int LQF_HDR = 0;     // 40: x0(12) R(9) feet(12)
constexpr int LQF_G0 = 40;     // 72: B rows 6-11 (terrain: G0 blkdiag(R_j))
constexpr int LQF_QW = 112;    // 12: state weights
constexpr int LQF_ZERO = 124;  // 4:  always 0
constexpr int LQF_TF = 128;    // 36: terrain frames R_j (row-major)
constexpr int LQF_RB = 164;    // 24: terrain R_j' diag(r_j) R_j packed [xx xy xz yy yz zz]
constexpr int LQF_PV = 188;    // 144: pivot rows of Guu, L^-1, X (48 each)
constexpr int LQF_SINK = 332;  // 64: stores of lanes that hold no pivot row / no output
constexpr int LQF_EX = 396;    // 32: exchange buffer of the serial sweeps
constexpr int LQF_CS = 428;    // 2H: cos / sin of the reference yaw per step
constexpr int LQF_FIXED = 428;
// At H <= LQ_KZ_MAXH (one leg-step per lane) the closed-loop rows KZ = K Z (6 x 12 per stage) are kept too, after the
// slots: the forward sweep is then one 12-term product per row (x' = A x + dv - KZ x - t, t = K za + rho in the rho
// field) instead of w = Z x + za followed by K w; eight QPs per CU still fit at H = 10.
#ifndef LMPC_LQ_KZ_MAXH  // diagnostic A/B: 0 = no closed-loop rows (a different forward-sweep formula, other bits)
#define LMPC_LQ_KZ_MAXH 10
#endif
constexpr int LQ_KZ_MAXH = LMPC_LQ_KZ_MAXH;
__host__ __device__ constexpr bool lq_kzs(int H) { return H <= LQ_KZ_MAXH; }
__host__ __device__ constexpr int lq_lds_doubles(int H) {
    return LQF_FIXED + 2 * H + LQ_SLOT * H + (lq_kzs(H) ? 72 * H : 0);
}
inline size_t lq_lds_bytes(int H) { return (size_t)lq_lds_doubles(H) * sizeof(double); }

__device__ __forceinline__ constexpr int pk6(int a, int b) {  // packed lower 6x6, any order
    return a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a;
}

// entries of dt N(yaw) = A_k - I (rows 0-5, columns 6-11)
__device__ __forceinline__ double lq_dtN(int r, int c, double ck, double sk, double dt) {
    // lane-static pattern: rows 0-1 x columns 6-7 the yaw rotation, (2, 8) and (r, r + 6) for r = 3..5 one
    const bool rot = r < 2 && (c == 6 || c == 7);
    const bool one = (r == 2 && c == 8) || (r >= 3 && r < 6 && c == r + 6);
    const bool cs_ = (r == 0) == (c == 6);  // (0,6), (1,7): cos; (0,7), (1,6): +-sin
    const double rv = cs_ ? ck : (r == 0 ? sk : -sk);
    return dt * (rot ? rv : (one ? 1.0 : 0.0));
}

// (A x)[r], (A^-1 x)[r] (A = I + dt N, N nilpotent: A^-1 = I - dt N) for a compile-time row r
template <class Ptr>
__device__ __forceinline__ double lq_Ax(Ptr x, int r, double ck, double sk, double dt, double sgn) {
    if (r == 0) return x[0] + sgn * dt * (ck * x[6] + sk * x[7]);
    if (r == 1) return x[1] + sgn * dt * (-sk * x[6] + ck * x[7]);
    if (r == 2) return x[2] + sgn * dt * x[8];
    if (r < 6) return x[r] + sgn * dt * x[r + 6];
    return x[r];
}

// The factorisation sweep reads the lane index once per sweep (bit 0: for the stage body, bit 1: for the operand
// fetch), so its lane-static offsets and masks are computed once per sweep instead of once per stage (478 -> 187
// instructions per stage).  That fits 256 registers at two waves per SIMD only because every other pass takes its
// own opaque copy of the lane index (no lane address lives across the sweep) and the reduced stage reads its U row
// late (LMPC_LQ_LATE); config 4 10.8 -> 9.9 ms.  0 restores the per-stage maps (diagnostic).
#ifndef LMPC_LQ_HOIST
#define LMPC_LQ_HOIST 3
#endif
// the same choice for the two-wave instance at two leg-steps per lane (round 6: H = 17..26)
#ifndef LMPC_LQ_HOIST_LS2W2
#define LMPC_LQ_HOIST_LS2W2 3
#endif
// At two waves per SIMD the reduced stage reads its U row after the pivot staging and stores Z_k after the solve
// (shorter live ranges across the 6 x 6 factor; the lone-wave instances keep the early read, 2 % faster there -- the
// same arithmetic either way, so every instance gives the same bits); 0 = the early read everywhere (diagnostic)
// 1 fences the next stage's operand fetch off from the machine scheduler (one block between the stage's first
// matrix-core chain and its leg-block work: round 4's choice under max-ilp).  Under iterative-ilp (round 5) the
// scheduler places it better on its own: configs 3/4/5 -1.7/-0.3/-1.6 % without the fence
// (profiles/r05/fused/ab_lq_fence_hoist.log), so 0 is the default; 1 is kept for A/B.
#ifndef LMPC_LQ_FETCH_FENCE
#define LMPC_LQ_FETCH_FENCE 0
#endif
// 1 loads a serial-sweep stage's operands one stage ahead in the lone-wave instance (round 4).  Under iterative-ilp
// (round 5) loading them in the stage is faster -- the second operand set's registers cost more than the load
// latency they hid: config 2 --dense off -3 %, configs 3/5 -2 % (profiles/r05/fused/ab_lq_late_prefetch.log).
// reduced-input polish stages also at two leg-steps per lane (diagnostic A/B; see LQ_RP in the kernel)
#ifndef LMPC_LQ_RP2
#define LMPC_LQ_RP2 0
#endif
#ifndef LMPC_LQ_PF
#define LMPC_LQ_PF 0
#endif
#ifndef LMPC_LQ_LATE
#define LMPC_LQ_LATE 1
#endif
constexpr bool LQ_LATE_ON = LMPC_LQ_LATE != 0;

__device__ __forceinline__ int lq_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// The lane index for the lane-static operand maps of a phase: opaque at two waves per SIMD (recomputed where used:
// 256 registers cannot hold them across the solve), plain in the lone-wave instance (512 registers: computed once).
#ifndef LMPC_LQ_OPAQUE_W1
#define LMPC_LQ_OPAQUE_W1 0
#endif
template <int WPE>
__device__ __forceinline__ int lq_lane(int lane) {
    return (WPE == 1 && !LMPC_LQ_OPAQUE_W1) ? lane : lq_opaque(lane);
}

// The same products branch-free for a runtime row r: (A x)[r] = x[r] + dt (a1 x[c1] + a2 x[c2]) and
// (A' w)[r] = w[r] + dt (a1 w[c1] + a2 w[c2]), with lane-static columns and coefficients selected from (cos, sin)
// of the stage's yaw; every operand load is unconditional (a divergent branch per row waits on its own loads).
struct LqRow {
    int c1, c2;
    double a1, a2;
};
__device__ __forceinline__ LqRow lq_ax_row(int r, double ck, double sk) {
    LqRow o;
    o.c1 = r < 2 ? 6 : (r < 6 ? r + 6 : 6);
    o.c2 = 7;
    o.a1 = r == 0 ? ck : r == 1 ? -sk : (r < 6 ? 1.0 : 0.0);
    o.a2 = r == 0 ? sk : r == 1 ? ck : 0.0;
    return o;
}
__device__ __forceinline__ LqRow lq_atw_row(int r, double ck, double sk) {
    LqRow o;
    o.c1 = r >= 8 ? r - 6 : 0;
    o.c2 = 1;
    o.a1 = r == 6 ? ck : r == 7 ? sk : (r >= 8 ? 1.0 : 0.0);
    o.a2 = r == 6 ? -sk : r == 7 ? ck : 0.0;
    return o;
}
template <class Ptr>
__device__ __forceinline__ double lq_row_apply(Ptr x, int r, const LqRow& q, double s) {
    return fma(s, fma(q.a1, x[q.c1], q.a2 * x[q.c2]), x[r]);
}

// lane-local solve of the symmetric positive definite 3x3 system R y = b (R packed [xx xy xz yy yz zz])
__device__ __forceinline__ void sym3_solve(const double R[6], const double b[3], double y[3]) {
    const double i00 = rsq_nr(R[0]);
    const double l10 = R[1] * i00, l20 = R[2] * i00;
    const double i11 = rsq_nr(fma(-l10, l10, R[3]));
    const double l21 = fma(-l20, l10, R[4]) * i11;
    const double i22 = rsq_nr(fma(-l21, l21, fma(-l20, l20, R[5])));
    const double c0 = b[0] * i00;
    const double c1 = fma(-l10, c0, b[1]) * i11;
    const double c2 = fma(-l21, c1, fma(-l20, c0, b[2])) * i22;
    y[2] = c2 * i22;
    y[1] = fma(-l21, y[2], c1) * i11;
    y[0] = fma(-l20, y[2], fma(-l10, y[1], c0)) * i00;
}

// ---------------------------------------------------------------------------------------------------------
// The kernel.  LS = leg-steps per lane (ceil(4H/64)); TERRAIN: per-leg contact frames (lmpc_kernels.hip).
// WPE = waves per SIMD the register budget allows: 2 (256 registers, LS = 1 only: eight QPs per CU at H <= 10) or 1
// (512, no spills: the instance for batches of at most one QP per SIMD, and for LS = 2).
// ---------------------------------------------------------------------------------------------------------
// The solve of QP blockIdx.x as a device function: lmpc_lq_kernel runs it alone; lmpc_dense_lq_kernel after the dense
// solve of the same QP (after_dense: the QP is one the dense solve left, so the hand-over test below is skipped).
template <int LS, bool TERRAIN, int WPE>
__device__ __forceinline__ void lq_body(const DevParams prm, const double* __restrict__ rec,
                                        const uint8_t* __restrict__ contact, const double* __restrict__ normals,
                                        int batch, double* __restrict__ grf, int32_t* __restrict__ status,
                                        int32_t* __restrict__ iters, const uint8_t* __restrict__ dense_done,
                                        bool after_dense) {
    extern __shared__ __attribute__((aligned(16))) double lq_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    if (prm.dense && !after_dense) {  // QPs with 1..DENSE_MAX_LS stance leg-steps went to a dense-path kernel (H <= 16 here)
        const bool stl = lane < 4 * H && contact[(size_t)qp * 4 * H + lane] != 0;
        const int n = __popcll(__ballot(stl));
        if (n >= 1 && n <= DENSE_MAX_LS && (!dense_done || dense_done[qp])) return;
    }
    ldouble* const sm = (ldouble*)lq_smem;
    ldouble* const hdr = sm + LQF_HDR;
    ldouble* const G0s = sm + LQF_G0;
    ldouble* const qw = sm + LQF_QW;
    ldouble* const zero = sm + LQF_ZERO;
    ldouble* const tf = sm + LQF_TF;
    ldouble* const rbt = sm + LQF_RB;
    ldouble* const pv = sm + LQF_PV;
    ldouble* const sink = sm + LQF_SINK;
    ldouble* const ex = sm + LQF_EX;
    ldouble* const cs = sm + LQF_CS;
    ldouble* const slots = sm + LQF_FIXED + 2 * H;
    ldouble* const kzr = slots + LQ_SLOT * H;  // closed-loop rows (kzs only)
    // (both instances, although it pays only at two waves per SIMD: the instance a QP runs on depends on the batch,
    // and a QP's answer must not -- test_full_size_properties checks the bits)
    const bool kzs = LS == 1 && lq_kzs(H);
    const int RL = 33 + 12 * H;
    const double* rin = rec + (size_t)qp * RL;
    const double* xr = rin + 33;  // x_ref (global, L2-resident after its first use)
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;
    // the serial sweeps can load a stage's operands one stage ahead in the lone-wave instance (LMPC_LQ_PF, off by
    // default since round 5); at two waves per SIMD the second set of registers would spill
    constexpr bool LQ_PF = LMPC_LQ_PF && WPE == 1;
    constexpr bool LQ_LATE = LQ_LATE_ON && WPE == 2;
    constexpr int LQ_HOIST = (LS == 2 && WPE == 2) ? LMPC_LQ_HOIST_LS2W2 : LMPC_LQ_HOIST;
    // reduced-input polish stages (well-conditioned W_k) at one leg-step per lane: measured -1.2 % on config 4 (stages
    // with three or four stance legs), +2.5 % on config 2 with the dense path off (a trot's full polish stage has only
    // two pivot blocks); both instances alike, as kzs above; at two leg-steps per lane the leg-step work is not repaid
    constexpr bool LQ_RP = LS == 1 || LMPC_LQ_RP2;
    LQ_STAMP_DECL

    // ---- prologue: record, terrain frames, I_w^-1, G0, yaw cos / sin ----------------------------------------
    if (lane < 33) hdr[lane] = rin[lane];
    if (lane < 12) qw[lane] = prm.q[lane];
    if (lane < 4) zero[lane] = 0.0;
    if constexpr (TERRAIN) {
        if (lane < 4) {
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
                for (int b = a; b < 3; ++b) rbt[6 * lane + e++] = r0 * R[a] * R[b] + r1 * R[3 + a] * R[3 + b] + r2 * R[6 + a] * R[6 + b];
        }
    }
    for (int k = lane; k < H; k += 64) {
        double sn, cn;
        sincos(xr[12 * k + 2], &sn, &cn);
        cs[2 * k] = cn;
        cs[2 * k + 1] = sn;
    }
    LMPC_SYNC();
    {
        double iw[9];
        const ldouble* R = hdr + LMPC_REC_ROT;
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
        // G0 = dt [I_w^-1 skew(r_j) ; I/m] (ConvexQPSolver.cpp:198-212; Utils.cpp:89-95), terrain: G0 blkdiag(R_j)
        for (int e = lane; e < 72; e += 64) {
            const int r = e / 12, c = e % 12, j = c / 3, cc = c % 3;
            double w[3];
            if (r < 3) {
                const ldouble* ft = hdr + LMPC_REC_FEET + 3 * j;
                // row r of I_w^-1 by selects (a dynamically indexed private array would live in scratch memory)
                const double a0 = r == 0 ? iw[0] : r == 1 ? iw[3] : iw[6];
                const double a1 = r == 0 ? iw[1] : r == 1 ? iw[4] : iw[7];
                const double a2 = r == 0 ? iw[2] : r == 1 ? iw[5] : iw[8];
                w[0] = dt * (a1 * ft[2] - a2 * ft[1]);
                w[1] = dt * (-a0 * ft[2] + a2 * ft[0]);
                w[2] = dt * (a0 * ft[1] - a1 * ft[0]);
            } else {
                w[0] = w[1] = w[2] = 0.0;
                w[r - 3] = dt / prm.mass;
            }
            double v = w[cc];
            if constexpr (TERRAIN) {
                const ldouble* Rj = tf + 9 * j;
                v = w[0] * Rj[cc] + w[1] * Rj[3 + cc] + w[2] * Rj[6 + cc];
            }
            G0s[e] = v;
        }
    }
    LMPC_SYNC();

    // ---- leg-step ownership, starting point (lmpc_kernels.hip) -----------------------------------------------
    bool st[LS], valid[LS];
    int lsk[LS], lsj[LS];
    double f[LS][3], s[LS][5], z[LS][5];
    // long-lived per leg-step: the iterate (f, s, z), the stage data of the current Newton system (Rr: input
    // Hessian block, rr: linear term), the last solution u and the predictor's ua.  The polish's null-space
    // basis (T, up) is recomputed where it is needed (leg_basis), so it holds no registers across the solves.
    double Rr[LS][6], rr[LS][3], u[LS][3], ua[LS][3];
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
        const double cnt = quad_sum(st[t] ? 1.0 : 0.0);
        f[t][2] = st[t] ? fmin(0.5 * fzmax, prm.mass * prm.grav / fmax(cnt, 1.0)) : 0.0;
        double o[5];
        cons_resid(f[t], mu, fzmax, o);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            s[t][i] = st[t] ? -o[i] : 1.0;
            z[t][i] = 1.0 / s[t][i];
        }
#pragma unroll
        for (int m = 0; m < 3; ++m) u[t][m] = ua[t][m] = rr[t][m] = 0.0;
#pragma unroll
        for (int e = 0; e < 6; ++e) Rr[t][e] = (e == 0 || e == 3 || e == 5) ? 1.0 : 0.0;
    }
    const double nst = wave_sum((double)nst_loc);
    LQ_STAMP(0);  // prologue

    const int lc = lane & 15, lr = lane >> 4;  // accumulator layout: column lc, rows lr + 4i

    // ---- the interior point / polish state machine -----------------------------------------------------------
    int qstatus = LMPC_QP_CONVERGED, ipm_it = 0, prounds = 0;
    bool done = false;
    if (nst > 0.5) {
        enum { PRED = 0, CORR = 1, POLISH = 2 };
        const double mc = 5.0 * nst;
        double tol = prm.tol_mu;
        int att = 0, rd = 0, it_end = prm.max_iter, mode = PRED;
        // the polish's reduced-input stages switched off for the rest of this QP (wave-uniform): set when a settled
        // active set fails the certificate's dynamics check -- a nearly rank-deficient W_k whose tiny directions the
        // reduced stage drops leaves the swept trajectory off the forces' own (2 of 65536 flat config-4 QPs, 1e-6)
        bool rp_off = false;
        int act[LS];
        bool apex[LS];
#pragma unroll
        for (int t = 0; t < LS; ++t) {
            act[t] = 0;
            apex[t] = false;
        }
        double mu_c = 0.0, smu = 0.0;
        for (;;) {
            // ======== leg-step work: stage data of the Newton system ========
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
                }
            }
            // stage data per leg-step: Rr (the input Hessian block), rr (linear term), and for the factorisation
            // Bt = G0_j T -> S slot, rr -> x slot, G0_j up (-> dv) with T the leg's null-space basis (I for a stance leg
            // in the interior point, 0 for a swing leg) and up its particular solution (polish only)
            // the tracking terms -Q x_ref,j of every stage, loaded from the record here (global memory: every load
            // issued at once, ahead of the leg-step work) and stored to slot j below -- v field before a
            // factorisation, x field before the corrector's backward sweep -- so the serial sweeps read LDS only
            // the leg-step work, specialised per mode at compile time (its three variants share no registers)
            unsigned long long cmask[LS];
            auto legwork = [&](auto mode_tag) {
                constexpr int md = decltype(mode_tag)::value;
                constexpr int NTQ = LS == 1 ? 3 : 6;
                double qxl[NTQ];
    #pragma unroll
                for (int i = 0; i < NTQ; ++i) qxl[i] = xr[min(lq_lane<WPE>(lane) + 64 * i, 12 * H - 1)];
                double du[LS][6], gq[LS][6];
                bool cpl[LS];
    #pragma unroll
                for (int t = 0; t < LS; ++t) {
                    const int j = lsj[t];
                    double rb[6];
                    if constexpr (TERRAIN) {
    #pragma unroll
                        for (int e = 0; e < 6; ++e) rb[e] = rbt[6 * j + e];
                    } else {
                        rb[0] = prm.r[3 * j]; rb[1] = 0.0; rb[2] = 0.0;
                        rb[3] = prm.r[3 * j + 1]; rb[4] = 0.0; rb[5] = prm.r[3 * j + 2];
                    }
                    double T[9], up[3] = {0.0, 0.0, 0.0};
    #pragma unroll
                    for (int e = 0; e < 9; ++e) T[e] = (e % 4 == 0 && st[t]) ? 1.0 : 0.0;
                    if (md == POLISH) {
                        apex[t] = false;
                        if (st[t]) apex[t] = leg_basis(act[t], mu, fzmax, T, up);
                        // Rr = T' Rb T (fixed components -> identity), rr = T' Rb up
                        const double R3[9] = {rb[0], rb[1], rb[2], rb[1], rb[3], rb[4], rb[2], rb[4], rb[5]};
                        bool fixed[3];
    #pragma unroll
                        for (int a = 0; a < 3; ++a) fixed[a] = T[a] == 0.0 && T[3 + a] == 0.0 && T[6 + a] == 0.0;
                        double RT[9], Ru[3];
    #pragma unroll
                        for (int q = 0; q < 3; ++q) {
    #pragma unroll
                            for (int b = 0; b < 3; ++b) RT[q * 3 + b] = R3[q * 3 + 0] * T[0 * 3 + b] + R3[q * 3 + 1] * T[1 * 3 + b] + R3[q * 3 + 2] * T[2 * 3 + b];
                            Ru[q] = R3[q * 3 + 0] * up[0] + R3[q * 3 + 1] * up[1] + R3[q * 3 + 2] * up[2];
                        }
                        int e = 0;
    #pragma unroll
                        for (int a = 0; a < 3; ++a) {
    #pragma unroll
                            for (int b = a; b < 3; ++b) {
                                double v = T[0 * 3 + a] * RT[0 * 3 + b] + T[1 * 3 + a] * RT[1 * 3 + b] + T[2 * 3 + a] * RT[2 * 3 + b];
                                if (fixed[a] || fixed[b]) v = (a == b) ? 1.0 : 0.0;
                                Rr[t][e++] = v;
                            }
                            rr[t][a] = fixed[a] ? 0.0 : T[0 * 3 + a] * Ru[0] + T[1 * 3 + a] * Ru[1] + T[2 * 3 + a] * Ru[2];
                        }
                    } else if (md == PRED) {
                        // interior point: Rr = Rb + C'WC, rr = C'W(s - b) (predictor); identity / zero on swing legs
                        double W[5] = {0, 0, 0, 0, 0}, wv[5] = {0, 0, 0, 0, 0};
                        if (st[t]) {
    #pragma unroll
                            for (int i = 0; i < 5; ++i) {
                                W[i] = z[t][i] * rcp_nr(s[t][i]);
                                wv[i] = W[i] * (s[t][i] - (i == 4 ? fzmax : 0.0));
                            }
                        }
                        const double sx = W[0] + W[1], sy = W[2] + W[3];
                        Rr[t][0] = st[t] ? rb[0] + sx : 1.0;
                        Rr[t][1] = st[t] ? rb[1] : 0.0;
                        Rr[t][2] = st[t] ? rb[2] + mu * (W[0] - W[1]) : 0.0;
                        Rr[t][3] = st[t] ? rb[3] + sy : 1.0;
                        Rr[t][4] = st[t] ? rb[4] + mu * (W[2] - W[3]) : 0.0;
                        Rr[t][5] = st[t] ? rb[5] + mu * mu * (sx + sy) + W[4] : 1.0;
                        cons_tw(wv, mu, rr[t]);
                    }
                    // (CORR: Rr unchanged; rr was set to the corrector's by the predictor step below)
                    bool cp = false;
    #pragma unroll
                    for (int e = 0; e < 9; ++e) cp |= T[e] != 0.0;
                    cpl[t] = valid[t] && cp;
    #pragma unroll
                    for (int m = 0; m < 6; ++m) du[t][m] = 0.0;
                    if (md == POLISH && valid[t]) {
                        ldouble* sl = slots + lsk[t] * LQ_SLOT;
    #pragma unroll
                        for (int m = 0; m < 6; ++m) {
                            const double g0 = G0s[m * 12 + 3 * j + 0], g1 = G0s[m * 12 + 3 * j + 1], g2 = G0s[m * 12 + 3 * j + 2];
    #pragma unroll
                            for (int a = 0; a < 3; ++a) sl[LQ_Z + m * 12 + 3 * j + a] = g0 * T[0 * 3 + a] + g1 * T[1 * 3 + a] + g2 * T[2 * 3 + a];
                            du[t][m] = g0 * up[0] + g1 * up[1] + g2 * up[2];
                        }
    #pragma unroll
                        for (int a = 0; a < 3; ++a) sl[LQ_X + 3 * j + a] = rr[t][a];
                    }
                    if (md != POLISH || LQ_RP) {
                        // the Newton systems in reduced inputs (RED6 of tools/lq_proto.py): with Rr = L L' (lane-local),
                        // Y = Bt_j L^-T (Bt_j = G0_j T: G0_j on a stance leg in the interior point): the leg's W_j = Y Y'
                        // and g_j = Y L^-1 rr, summed over the stage's legs below; swing legs add nothing.  The interior
                        // point always solves in reduced inputs (W_k -> the Z field, dv - g -> dv); the polish where W_k is
                        // well conditioned (W_k -> the K field, g_k -> the rho field; the U pre-pass decides per stage)
                        const double i00 = rsq_nr(Rr[t][0]);
                        const double l10 = Rr[t][1] * i00, l20 = Rr[t][2] * i00;
                        const double i11 = rsq_nr(fma(-l10, l10, Rr[t][3]));
                        const double l21 = fma(-l20, l10, Rr[t][4]) * i11;
                        const double i22 = rsq_nr(fma(-l21, l21, fma(-l20, l20, Rr[t][5])));
                        const double m10 = -l10 * i00 * i11, m21 = -l21 * i11 * i22, m20 = fma(l10 * l21, i11, -l20) * i00 * i22;
                        const double c0 = rr[t][0] * i00;                               // L^-1 rr
                        const double c1 = fma(m10, rr[t][0], i11 * rr[t][1]);
                        const double c2 = fma(m20, rr[t][0], fma(m21, rr[t][1], i22 * rr[t][2]));
                        double Y[6][3];
    #pragma unroll
                        for (int m = 0; m < 6; ++m) {
                            const double g0 = G0s[m * 12 + 3 * j + 0], g1 = G0s[m * 12 + 3 * j + 1], g2 = G0s[m * 12 + 3 * j + 2];
                            double b0, b1, b2;
                            if (md == POLISH) {
                                b0 = g0 * T[0] + g1 * T[3] + g2 * T[6];
                                b1 = g0 * T[1] + g1 * T[4] + g2 * T[7];
                                b2 = g0 * T[2] + g1 * T[5] + g2 * T[8];
                            } else {
                                b0 = st[t] ? g0 : 0.0;
                                b1 = st[t] ? g1 : 0.0;
                                b2 = st[t] ? g2 : 0.0;
                            }
                            Y[m][0] = b0 * i00;
                            Y[m][1] = fma(b0, m10, b1 * i11);
                            Y[m][2] = fma(b0, m20, fma(b1, m21, b2 * i22));
                            const double gm = fma(Y[m][0], c0, fma(Y[m][1], c1, Y[m][2] * c2));
                            if (md == POLISH) gq[t][m] = gm;
                            else du[t][m] = -gm;
                        }
                        if (md != CORR) {  // W_k = sum over the quad, entry by entry (U's place)
                            ldouble* wz = slots + lsk[t] * LQ_SLOT + (md == POLISH ? LQ_K : LQ_Z);
                            const bool lead = valid[t] && j == 0;
    #pragma unroll
                            for (int m = 0; m < 6; ++m)
    #pragma unroll
                                for (int n = 0; n <= m; ++n) {
                                    const double w = quad_sum(fma(Y[m][0], Y[n][0], fma(Y[m][1], Y[n][1], Y[m][2] * Y[n][2])));
                                    if (lead) wz[pk6(m, n)] = w;
                                }
                        }
                    }
                }
                // per stage, summed over its legs (lanes 4k..4k+3: a quad): polish dv_k = sum_j G0_j up_j - g dt e5; interior
                // point dv_k - g_k (predictor) and W_k, the corrector's dg = g'' - g' (to the rho slot)
    #pragma unroll
                for (int t = 0; t < LS; ++t) {
    #pragma unroll
                    for (int m = 0; m < 6; ++m) du[t][m] = quad_sum(du[t][m]);
                    if (md == POLISH && LQ_RP) {
    #pragma unroll
                        for (int m = 0; m < 6; ++m) gq[t][m] = quad_sum(gq[t][m]);
                    }
                    if (valid[t] && lsj[t] == 0) {
                        ldouble* sl = slots + lsk[t] * LQ_SLOT;
                        if (md == POLISH && LQ_RP) {
    #pragma unroll
                            for (int m = 0; m < 6; ++m) sl[LQ_RHO + m] = gq[t][m];
                        }
                        if (md == CORR) {
    #pragma unroll
                            for (int m = 0; m < 6; ++m) sl[LQ_RHO + m] = -du[t][m] + sl[LQ_DV + m] + (m == 5 ? prm.grav * dt : 0.0);
                        } else {
    #pragma unroll
                            for (int m = 0; m < 6; ++m) sl[LQ_DV + m] = du[t][m] - (m == 5 ? prm.grav * dt : 0.0);
                        }
                    }
                }
                // coupled legs per stage (T != 0): ballot, one word per leg-step slot
    #pragma unroll
                for (int t = 0; t < LS; ++t) cmask[t] = __ballot(cpl[t]);
                {
                    const int fld = md == CORR ? LQ_X : LQ_V;
    #pragma unroll
                    for (int i = 0; i < NTQ; ++i) {
                        const int e = lq_lane<WPE>(lane) + 64 * i, j = e / 12, r = e - 12 * j;
                        if (e < 12 * H) slots[j * LQ_SLOT + fld + r] = -qw[r] * qxl[i];
                    }
                }
            };
            if (mode == PRED) legwork(std::integral_constant<int, PRED>{});
            else if (mode == CORR) legwork(std::integral_constant<int, CORR>{});
            else legwork(std::integral_constant<int, POLISH>{});
            LMPC_SYNC();
            LQ_STAMP(1);  // leg-step work

            if (mode == CORR) {
                // ======== corrector: rho = dg - K P22 dg per stage (the new rr enters through g only), then the
                // backward sweep.  P22 = P_{k+1}[6:12, 6:12] from Z_k = rows 6-11 of P_{k+1} A_k (A_k's columns 0-5
                // are unit columns): P22 = Z[:, 6:12] - Z[:, 0:6] dtN[0:6, 6:12].  h = P22 dg goes to Z's column 12
                // (za, rewritten by the sweep), then rho over dg in the rho slot ========
                constexpr int NT6 = (6 * LMPC_MAX_HORIZON + 63) / 64;
#pragma unroll
                for (int i = 0; i < NT6; ++i) {
                    if (64 * i >= 6 * H) break;  // wave-uniform
                    const int e = lq_lane<WPE>(lane) + 64 * i, ec = e < 6 * H ? e : 6 * H - 1;
                    const int k = ec / 6, m = ec - 6 * k;
                    const ldouble* sl = slots + k * LQ_SLOT;
                    const double dtc = dt * cs[2 * k], dts = dt * cs[2 * k + 1];
                    const ldouble* dg = sl + LQ_RHO;
                    const ldouble* zr = sl + LQ_Z + m * 13;
                    const double e0 = fma(dtc, dg[0], dts * dg[1]), e1 = fma(dtc, dg[1], -dts * dg[0]);
                    double h = -fma(zr[0], e0, zr[1] * e1);
#pragma unroll
                    for (int n = 2; n < 6; ++n) h = fma(-zr[n], dt * dg[n], h);
#pragma unroll
                    for (int n = 0; n < 6; ++n) h = fma(zr[6 + n], dg[n], h);
                    if (e < 6 * H) slots[k * LQ_SLOT + LQ_Z + m * 13 + 12] = h;
                }
                LMPC_SYNC();
#pragma unroll
                for (int i = 0; i < NT6; ++i) {
                    if (64 * i >= 6 * H) break;  // wave-uniform
                    const int e = lq_lane<WPE>(lane) + 64 * i, ec = e < 6 * H ? e : 6 * H - 1;
                    const int k = ec / 6, m = ec - 6 * k;
                    const ldouble* sl = slots + k * LQ_SLOT;
                    double rho = sl[LQ_RHO + m];
#pragma unroll
                    for (int n = 0; n < 6; ++n) rho = fma(-sl[LQ_K + pk6(m, n)], sl[LQ_Z + n * 13 + 12], rho);
                    if (e < 6 * H) slots[k * LQ_SLOT + LQ_RHO + m] = rho;  // only this lane reads this dg
                }
                LMPC_SYNC();
                if (kzs) {
                    // closed-loop rows: p_k = q'_k + A'y - (K Z)'y[6:12] with q'_k = q_k - Z_{k+1}'rho_{k+1} formed for
                    // every stage first (parallel, into the x field), t = K za + rho afterwards (parallel, over rho)
                    constexpr int NT12 = (12 * LMPC_MAX_HORIZON + 63) / 64;
#pragma unroll
                    for (int i = 0; i < NT12; ++i) {
                        if (64 * i >= 12 * (H - 1)) break;  // wave-uniform
                        const int e = lq_lane<WPE>(lane) + 64 * i, ec = e < 12 * (H - 1) ? e : 12 * (H - 1) - 1;
                        const int k = 1 + ec / 12, r = ec - 12 * (k - 1);
                        const ldouble* sl = slots + k * LQ_SLOT;
                        double v = slots[(k - 1) * LQ_SLOT + LQ_X + r];
#pragma unroll
                        for (int mm = 0; mm < 6; ++mm) v = fma(-sl[LQ_Z + mm * 13 + r], sl[LQ_RHO + mm], v);
                        if (e < 12 * (H - 1)) slots[(k - 1) * LQ_SLOT + LQ_X + r] = v;
                    }
                    LMPC_SYNC();
                    const int lnb = lq_lane<WPE>(lane), r = lnb < 12 ? lnb : 0;  // per pass: no lane address outlives it
                    double p = lnb < 12 ? slots[(H - 1) * LQ_SLOT + LQ_X + r] : 0.0;
                    for (int k = H - 1; k >= 0; --k) {
                        const ldouble* sl = slots + k * LQ_SLOT;
                        const double y = p + sl[LQ_V + r];
                        const int kp = k > 0 ? k - 1 : 0;
                        double kz[6];
#pragma unroll
                        for (int a = 0; a < 6; ++a) kz[a] = kzr[k * 72 + a * 12 + r];
                        const double q = slots[kp * LQ_SLOT + LQ_X + r], ck = cs[2 * k], sk = cs[2 * k + 1];
                        if (lnb < 12) ex[r] = y;
                        if (lnb >= 6 && lnb < 12) slots[k * LQ_SLOT + LQ_Z + (lnb - 6) * 13 + 12] = y;
                        LMPC_SYNC();
                        if (k == 0) break;
                        double pn = q + lq_row_apply(ex, r, lq_atw_row(r, ck, sk), dt);
#pragma unroll
                        for (int a = 0; a < 6; ++a) pn = fma(-kz[a], ex[6 + a], pn);
                        p = pn;
                        LMPC_SYNC();
                    }
                    LMPC_SYNC();
                    constexpr int NT6 = (6 * LMPC_MAX_HORIZON + 63) / 64;
#pragma unroll
                    for (int i = 0; i < NT6; ++i) {
                        if (64 * i >= 6 * H) break;  // wave-uniform
                        const int e = lq_lane<WPE>(lane) + 64 * i, ec = e < 6 * H ? e : 6 * H - 1;
                        const int k = ec / 6, m = ec - 6 * k;
                        const ldouble* sl = slots + k * LQ_SLOT;
                        double t = sl[LQ_RHO + m];
#pragma unroll
                        for (int n = 0; n < 6; ++n) t = fma(sl[LQ_K + pk6(m, n)], sl[LQ_Z + n * 13 + 12], t);
                        if (e < 6 * H) slots[k * LQ_SLOT + LQ_RHO + m] = t;  // only this lane reads this rho
                    }
                } else
                // backward: y = p_{k+1} + v_k, za = y[6:12] -> Z column 12, t = K za + rho, p_k = q_k + A'y - Z't.
                // Lanes 0-11 hold p (lane r <-> p[r]); y goes through the exchange buffer, t by readlane.
                {
                    const int lnb = lq_lane<WPE>(lane), r = lnb < 12 ? lnb : 0;
                    const int m = lnb < 6 ? lnb : 0;
                    // a stage's operands are loaded while the stage before it runs: an LDS load cannot move above
                    // the fence that orders the exchange buffer, so loaded in the stage itself they would wait a
                    // round trip on the serial path
                    struct BwOps {
                        double v, rho, q, ck, sk, kr[6], zc[6];
                    };
                    auto load = [&](int k, BwOps& o) {
                        const ldouble* sl = slots + k * LQ_SLOT;
                        o.v = sl[LQ_V + r];
                        o.rho = sl[LQ_RHO + m];
                        o.q = slots[(k > 0 ? k - 1 : 0) * LQ_SLOT + LQ_X + r];
                        o.ck = cs[2 * k];
                        o.sk = cs[2 * k + 1];
#pragma unroll
                        for (int n = 0; n < 6; ++n) o.kr[n] = sl[LQ_K + pk6(m, n)];
#pragma unroll
                        for (int mm = 0; mm < 6; ++mm) o.zc[mm] = sl[LQ_Z + mm * 13 + r];
                    };
                    BwOps cur, nxt;
                    load(H - 1, cur);
                    double p = lnb < 12 ? slots[(H - 1) * LQ_SLOT + LQ_X + r] : 0.0;
                    for (int k = H - 1; k >= 0; --k) {
                        if (!LQ_PF && k < H - 1) load(k, cur);
                        const double y = p + cur.v;
                        if (lnb < 12) ex[r] = y;
                        if (lnb >= 6 && lnb < 12) slots[k * LQ_SLOT + LQ_Z + (lnb - 6) * 13 + 12] = y;
                        if (LQ_PF && k > 0) load(k - 1, nxt);
                        LMPC_SYNC();
                        if (k == 0) break;
                        // t_m = sum_n K[m][n] y[6+n] + rho_m, lanes 0-5
                        double tv = cur.rho;
#pragma unroll
                        for (int n = 0; n < 6; ++n) tv = fma(cur.kr[n], ex[6 + n], tv);
                        double pn = cur.q + lq_row_apply(ex, r, lq_atw_row(r, cur.ck, cur.sk), dt);
#pragma unroll
                        for (int mm = 0; mm < 6; ++mm) pn = fma(-cur.zc[mm], readlane_f64(tv, mm), pn);
                        p = pn;
                        if (LQ_PF) cur = nxt;
                        LMPC_SYNC();
                    }
                }
                LQ_STAMP(2);  // corrector backward
            } else {
                // ======== factorisation with the fused backward pass (stage k = H-1 .. 0) ========
                // The lane-static operand maps are recomputed in every stage from an opaque copy of the lane index
                // (integer work off the critical path): held across the loop -- or hoisted out of the solve loop by
                // loop-invariant code motion -- they would stay live through every other phase and push the kernel's
                // long-lived state past the 256 registers of two waves per SIMD.
                // interior point: reduced inputs -- B^ rows 6-11 = [U | 0 | dv'], unit input Hessian, X = L^-1 [0 | U' | 0],
                // two 3x3 pivot blocks whatever the stage's leg count; polish: Bt, Rr_j, rr as staged by the legs
                const bool red = mode != POLISH;
                LQ_MARK(_lq_fact0);
                if (red || LQ_RP) {
                    // U_k = chol(W_k) for every stage at once (lane k), in place of W (Z field; polish: K field); pivots
                    // at rounding level (W is rank-deficient with fewer than two stance legs) leave a zero column.  The
                    // polish solves a stage in reduced inputs only where W_k is well conditioned (every other pivot
                    // above 1e-6 of its diagonal: a polish answer must be exact); the flag goes to the exchange buffer
                    for (int k = lq_lane<WPE>(lane); k < H; k += 64) {
                        ldouble* wz = slots + k * LQ_SLOT + (red ? LQ_Z : LQ_K);
                        const double floor_ = red ? 1e-10 : 1e-12;
                        bool wellc = true;
                        double w[21];
#pragma unroll
                        for (int e = 0; e < 21; ++e) w[e] = wz[e];
#pragma unroll
                        for (int c = 0; c < 6; ++c) {
                            const double wd = w[pk6(c, c)];
                            double d = wd;
#pragma unroll
                            for (int b = 0; b < c; ++b) d = fma(-w[pk6(c, b)], w[pk6(c, b)], d);
                            const bool ok = d > floor_ * wd && wd > 0.0;
                            wellc = wellc && (!ok || d > 1e-6 * wd);
                            const double inv = ok ? rsq_nr(d) : 0.0;
                            w[pk6(c, c)] = ok ? d * inv : 0.0;
#pragma unroll
                            for (int r2 = c + 1; r2 < 6; ++r2) {
                                double v = w[pk6(r2, c)];
#pragma unroll
                                for (int b = 0; b < c; ++b) v = fma(-w[pk6(r2, b)], w[pk6(c, b)], v);
                                w[pk6(r2, c)] = v * inv;
                            }
                        }
#pragma unroll
                        for (int e = 0; e < 21; ++e) wz[e] = w[e];
                        if (!red) ex[k] = (wellc && !rp_off) ? 1.0 : 0.0;
                    }
                    LMPC_SYNC();
                }
                d4 P;
                {
                    const int fl = lq_lane<WPE>(lane), lc = fl & 15, lr = fl >> 4;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = lr + 4 * i;
                        P[i] = (r == lc && r < 12) ? qw[r < 12 ? r : 0] : 0.0;
                        if (lc == 12 && i < 3) P[i] = slots[(H - 1) * LQ_SLOT + LQ_V + r];
                    }
                }
                // operands of stage k: B^ k-blocks 1-2 (rows 4+lr, 8+lr: Bt (S slot) in columns 0-11, dv in column
                // 12), X = [0 | Bt' | rr] (columns 6-11: Bt[lc-6][row], column 12: rr[row] from the x slot), and
                // the column 12 of Q^_k (-q x_ref,k-1); out-of-range lanes read the zero words
                // the stage sweep, specialised for the interior point (reduced inputs) and for the polish
                auto sweep = [&](auto red_tag) {
                    constexpr bool red = decltype(red_tag)::value;
                    constexpr int UF = red ? LQ_Z : LQ_K;  // where U_k is (the polish stages Bt in the Z field)
                    const int sfl = lq_lane<WPE>(lane);  // one lane read for the whole sweep (its offsets stay in registers)
                    double bg[2], xg[3], qn[3], ckn, skn;
                    bool sfn;
                    auto fetch = [&](int k) {
                        const int fl = (LQ_HOIST & 2) ? sfl : lq_lane<WPE>(lane), lc = fl & 15, lr = fl >> 4;
                        const ldouble* sl = slots + k * LQ_SLOT;
                        ckn = cs[2 * k];
                        skn = cs[2 * k + 1];
                        // stage k in reduced inputs? (always in the interior point; the polish's per-stage flag)
                        const bool srf = red || (LQ_RP && __builtin_amdgcn_readfirstlane(ex[k] != 0.0 ? 1 : 0) != 0);
                        sfn = srf;
    #pragma unroll
                        for (int kk = 0; kk < 2; ++kk) {
                            const int r = 4 * (kk + 1) + lr;
                            const int a = r - 6;
                            // reduced: U[a][lc] (lower: lc <= a); full: Bt[a][lc]; column 12: dv (a reduced polish stage:
                            // dv - g, g in the rho field)
                            const bool in = r >= 6 && r < 12 && (lc == 12 || (srf ? lc <= a : lc < 12));
                            const int off = lc == 12 ? LQ_DV + a : (srf ? UF + pk6(a, lc) : LQ_Z + a * 12 + lc);
                            double v = (in ? sl : zero)[in ? off : 0];
                            if (!red) {
                                const int ac = r >= 6 && r < 12 ? a : 0;
                                const double gv = sl[LQ_RHO + ac];
                                v -= (srf && in && lc == 12) ? gv : 0.0;
                            }
                            bg[kk] = v;
                        }
    #pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            const int r = lr + 4 * i;
                            const int a = lc - 6;
                            // X columns 6-11: full stages Bt[a][r], column 12: rr (reduced stages: the lane-local 6x6)
                            const bool in = !srf && lc >= 6 && lc <= 12;
                            const int off = lc == 12 ? LQ_X + r : LQ_Z + a * 12 + r;
                            xg[i] = (in ? sl : zero)[in ? off : 0];
                        }
                        const int km = k > 0 ? k - 1 : 0;
    #pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            const double qv = slots[km * LQ_SLOT + LQ_V + lr + 4 * i];
                            qn[i] = lc == 12 ? qv : 0.0;
                        }
                    };
                    fetch(H - 1);
                    for (int k = H - 1; k >= 0; --k) {
                        const int fl = (LQ_HOIST & 1) ? sfl : lq_lane<WPE>(lane), lc = fl & 15, lr = fl >> 4;
                        ldouble* sl = slots + k * LQ_SLOT;
                        const double ck = ckn, sk = skn;
                        const bool sr = red || sfn;
                        double bh[2], xb[3], qc[3];
    #pragma unroll
                        for (int kk = 0; kk < 2; ++kk) bh[kk] = bg[kk];
    #pragma unroll
                        for (int i = 0; i < 3; ++i) {
                            xb[i] = xg[i];
                            qc[i] = qn[i];
                        }
                        // dt N(yaw_k), k-blocks 0-1 (rows 0-7) in the accumulator layout
                        double nh[2];
    #pragma unroll
                        for (int kk = 0; kk < 2; ++kk) nh[kk] = lq_dtN(4 * kk + lr, lc, ck, sk, dt);  // selects, no branches
                        // C = P^ B^ ; PA = P^ A (the d column below) ; Guu = B^' C
                        d4 C = {0.0, 0.0, 0.0, 0.0};
                        C = MFMA64(P[1], bh[0], C);
                        C = MFMA64(P[2], bh[1], C);
                        d4 PA = P;
                        PA = MFMA64(P[0], nh[0], PA);
                        PA = MFMA64(P[1], nh[1], PA);
                        d4 G = {0.0, 0.0, 0.0, 0.0};
                        G = MFMA64(bh[0], C[1], G);
                        G = MFMA64(bh[1], C[2], G);
                        // next stage's operands, issued while the matrix cores work through the chain above
#if LMPC_LQ_FETCH_FENCE
                        __builtin_amdgcn_sched_barrier(0);
#endif
                        fetch(k > 0 ? k - 1 : 0);
#if LMPC_LQ_FETCH_FENCE
                        __builtin_amdgcn_sched_barrier(0);
#endif
                        // reduced inputs: this lane's U row (c = lc - 6, for its X columns), read before Z_k overwrites U_k
                        double ur[6];
                        auto read_ur = [&]() {
                            const bool xc = lc >= 6 && lc < 12;
                            const int ac = xc ? lc - 6 : 0;
    #pragma unroll
                            for (int b = 0; b < 6; ++b) {
                                const bool in = xc && b <= ac;
                                ur[b] = (in ? sl : zero)[in ? UF + pk6(ac, b) : 0];
                            }
                        };
                        if constexpr (!LQ_LATE) {
                            if (sr) read_ur();
                        }
                        // PA column 12 += v = P d (C column 12); out: v, Z = rows 6-11 of PA (columns 0-12)
                        if (lc == 12) {
    #pragma unroll
                            for (int i = 0; i < 3; ++i) PA[i] += C[i];
                        }
    #pragma unroll
                        for (int i = 0; i < 3; ++i) (lc == 12 ? sl : sink)[lc == 12 ? LQ_V + lr + 4 * i : fl] = C[i];
                        if constexpr (!LQ_LATE) {
    #pragma unroll
                            for (int i = 1; i < 3; ++i) {
                                const int r = lr + 4 * i;
                                const bool o = r >= 6 && r < 12 && lc <= 12;
                                (o ? sl : sink)[o ? LQ_Z + (r - 6) * 13 + lc : fl] = PA[i];
                            }
                        }
                        LQ_STAMP(11);  // factorisation: C, PA, G, Z / v stores
                        d4 X;
                        const int ls0 = 4 * k;
                        const int lmask = (int)(((LS == 1 || ls0 < 64 ? cmask[0] : cmask[LS - 1]) >> (ls0 & 63)) & 15ull);  // static indices: a dynamically indexed array lives in scratch
                        if (sr) {
                            // ---- reduced inputs: Guu' = I + U'P22 U (6 x 6) through LDS once, factored by every lane
                            // (Guu' >= I: no pivot can fail), X = L^-1 U' (rows 0-5, columns 6-11): each lane solves L y = its U
                            // row and keeps its own rows of y; a stage without stance legs has U = 0 and X = 0 ----
                            LMPC_SYNC();  // the previous stage's reads of the staging block come first
    #pragma unroll
                            for (int i = 0; i < 2; ++i) {
                                const int r = lr + 4 * i;
                                if (lc < 6 && r < 6) pv[r * 6 + lc] = G[i];
                            }
                            LMPC_SYNC();
                            if constexpr (LQ_LATE) read_ur();  // U_k is still in place: Z_k is stored after the solve below
                            double gl[21];
    #pragma unroll
                            for (int r = 0; r < 6; ++r)
    #pragma unroll
                                for (int c = 0; c <= r; ++c) gl[pk6(r, c)] = pv[r * 6 + c] + (r == c ? 1.0 : 0.0);
                            double id[6];
    #pragma unroll
                            for (int c = 0; c < 6; ++c) {
                                double d = gl[pk6(c, c)];
    #pragma unroll
                                for (int b = 0; b < c; ++b) d = fma(-gl[pk6(c, b)], gl[pk6(c, b)], d);
                                id[c] = rsq_nr(d);
    #pragma unroll
                                for (int r = c + 1; r < 6; ++r) {
                                    double v = gl[pk6(r, c)];
    #pragma unroll
                                    for (int b = 0; b < c; ++b) v = fma(-gl[pk6(r, b)], gl[pk6(c, b)], v);
                                    gl[pk6(r, c)] = v * id[c];
                                }
                            }
                            // y = L^-1 (this lane's U row): the lane's X column, rows 0-5
                            double y[6];
    #pragma unroll
                            for (int r = 0; r < 6; ++r) {
                                double v = ur[r];
    #pragma unroll
                                for (int b = 0; b < r; ++b) v = fma(-gl[pk6(r, b)], y[b], v);
                                y[r] = v * id[r];
                            }
                            const bool xc = lc >= 6 && lc < 12 && lmask;
                            X[0] = xc ? (lr == 0 ? y[0] : lr == 1 ? y[1] : lr == 2 ? y[2] : y[3]) : 0.0;
                            X[1] = xc && lr < 2 ? (lr == 0 ? y[4] : y[5]) : 0.0;
                            X[2] = X[3] = 0.0;
                        } else {
                        // ---- block Cholesky of Guu by legs, L^-1 and X = L^-1 [0 | Bt' | rr] alongside ----
                        d4 Tg, Li;
    #pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int r = lr + 4 * i;
                            Tg[i] = (r < 12 && lc < 12) ? G[i] : 0.0;
                            Li[i] = (r == lc) ? 1.0 : 0.0;
                            X[i] = (i < 3) ? xb[i < 3 ? i : 0] : 0.0;
                        }
                        const int amask = lmask;
    #pragma unroll
                        for (int blk = 0; blk < 4; ++blk) {
                            if (!((amask >> blk) & 1)) continue;
                            const int o = 3 * blk;
                            const int i0 = o >> 2, i1 = (o + 2) >> 2;
                            const int ra = 4 * i0 + lr - o, rb = 4 * i1 + lr - o;
                            const bool ina = ra >= 0 && ra < 3, inb = i1 != i0 && rb >= 0 && rb < 3;
                            // Rr_j of this leg-step, from its lane (wave-uniform)
                            const int srcl = (ls0 + blk) & 63, srct = (ls0 + blk) >> 6;
                            double Rj[6];
    #pragma unroll
                            for (int e = 0; e < 6; ++e) Rj[e] = readlane_f64(LS == 1 || srct == 0 ? Rr[0][e] : Rr[LS - 1][e], srcl);
                            // the three tiles' pivot rows through LDS in one round trip (the fence ahead orders the
                            // previous block's reads of the staging rows before these writes)
                            LMPC_SYNC();
                            {
                                ldouble* dt0 = ina ? pv + 16 * ra + lc : sink + fl;
                                dt0[0] = Tg[i0];
                                if (i1 != i0) {
                                    ldouble* dt1 = inb ? pv + 16 * rb + lc : sink + fl;
                                    dt1[0] = Tg[i1];
                                }
                                ldouble* da = ina ? pv + 48 + 16 * ra + lc : sink + fl;
                                da[0] = Li[i0];
                                ldouble* dx = ina ? pv + 96 + 16 * ra + lc : sink + fl;
                                dx[0] = X[i0];
                                Li[i0] = ina ? 0.0 : Li[i0];
                                X[i0] = ina ? 0.0 : X[i0];
                                if (i1 != i0) {
                                    ldouble* db = inb ? pv + 48 + 16 * rb + lc : sink + fl;
                                    db[0] = Li[i1];
                                    ldouble* dy = inb ? pv + 96 + 16 * rb + lc : sink + fl;
                                    dy[0] = X[i1];
                                    Li[i1] = inb ? 0.0 : Li[i1];
                                    X[i1] = inb ? 0.0 : X[i1];
                                }
                            }
                            LMPC_SYNC();
                            const double p00 = pv[o] + Rj[0], p10 = pv[16 + o] + Rj[1], p11 = pv[16 + o + 1] + Rj[3];
                            const double p20 = pv[32 + o] + Rj[2], p21 = pv[32 + o + 1] + Rj[4], p22 = pv[32 + o + 2] + Rj[5];
                            const double t0 = pv[lc], t1 = pv[16 + lc], t2 = pv[32 + lc];
                            const double w0 = pv[48 + lc], w1 = pv[64 + lc], w2 = pv[80 + lc];
                            const double y0 = pv[96 + lc], y1 = pv[112 + lc], y2 = pv[128 + lc];
                            const double i00 = rsq_nr(p00);
                            const double l10 = p10 * i00, l20 = p20 * i00;
                            const double i11 = rsq_nr(fma(-l10, l10, p11));
                            const double l21 = fma(-l20, l10, p21) * i11;
                            const double i22 = rsq_nr(fma(-l21, l21, fma(-l20, l20, p22)));
                            const double x0 = t0 * i00;
                            const double x1 = fma(-l10, x0, t1) * i11;
                            const double x2 = fma(-l21, x1, fma(-l20, x0, t2)) * i22;
                            const double xs = lr == 0 ? x0 : lr == 1 ? x1 : x2;
                            const double av = (lc > o + 2 && lc < 12 && lr < 3) ? xs : 0.0;
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
                        }
                        }
                        if constexpr (LQ_LATE) {
                            LMPC_SYNC();  // every lane's U_k reads ahead of the Z_k stores over them
    #pragma unroll
                            for (int i = 1; i < 3; ++i) {
                                const int r = lr + 4 * i;
                                const bool o = r >= 6 && r < 12 && lc <= 12;
                                (o ? sl : sink)[o ? LQ_Z + (r - 6) * 13 + lc : fl] = PA[i];
                            }
                        }
                        LQ_STAMP(12);  // factorisation: leg blocks
                        // ---- KH = X'X: K (rows / columns 6-11, packed), rho (column 12) ----
                        d4 KH = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll
                        for (int kk = 0; kk < 2; ++kk) KH = MFMA64(X[kk], X[kk], KH);
                        // reduced inputs: X has rows 0-5 only (one leg-step per lane: the two-leg-step instance keeps
                        // the third product, whose code layout measured 1 % faster there)
                        if (LS == 2 || !sr) KH = MFMA64(X[2], X[2], KH);
    #pragma unroll
                        for (int i = 1; i < 3; ++i) {
                            const int r = lr + 4 * i;
                            const bool zr = r >= 6 && r < 12;
                            // (a reduced polish stage keeps g in the rho field: its rho is 0, and dv - g is its d)
                            const bool ko = zr && ((lc >= 6 && lc < 12 && lc <= r) || (lc == 12 && (red || !sr)));
                            const int off = lc == 12 ? LQ_RHO + (r - 6) : LQ_K + pk6(r - 6, lc - 6);
                            (ko ? sl : sink)[ko ? off : fl] = KH[i];
                        }
                        LQ_STAMP(13);  // factorisation: KH, K / rho stores
                        d4 KZ = {0.0, 0.0, 0.0, 0.0};
                        if (k > 0 || kzs) {
                            // KZ = KH M' (k-blocks 1-2; M' = PA with row 12 = e12: its k = 12 term is KH column 12 added
                            // to column 12 lane-locally)
                            KZ = MFMA64(KH[1], PA[1], KZ);
                            KZ = MFMA64(KH[2], PA[2], KZ);
                            if (lc == 12) {
    #pragma unroll
                                for (int i = 0; i < 3; ++i) KZ[i] += KH[i];
                            }
                            if (kzs) {  // rows 6-11: K Z (columns 0-11) to the KZ region, t = K za + rho (column 12) over rho
    #pragma unroll
                                for (int i = 1; i < 3; ++i) {
                                    const int r = lr + 4 * i;
                                    const bool zr = r >= 6 && r < 12 && lc <= 12;
                                    ldouble* dst = lc == 12 ? sl + LQ_RHO + (r - 6) : kzr + k * 72 + (r - 6) * 12 + lc;
                                    // t = K za + rho; a reduced polish stage: K za + g (g in the rho field)
                                    const double gadd = (!red && sr && lc == 12) ? sl[LQ_RHO + (zr && lc == 12 ? r - 6 : 0)] : 0.0;
                                    (zr ? dst : sink + fl)[0] = KZ[i] + gadd;
                                }
                            }
                        }
                        if (k > 0) {
                            // P^_k = Q^_k + A^'PA - M'KZ  (rows 0-11; row 12 is never read)
                            d4 Pn;
    #pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int r = lr + 4 * i;
                                const double qd = (r == lc && r < 12) ? qw[r < 12 ? r : 0] : 0.0;
                                Pn[i] = PA[i] + qd + ((lc == 12 && i < 3) ? qc[i < 3 ? i : 0] : 0.0);
                            }
                            Pn = MFMA64(nh[0], PA[0], Pn);
                            Pn = MFMA64(nh[1], PA[1], Pn);
                            Pn = MFMA64(-PA[1], KZ[1], Pn);
                            Pn = MFMA64(-PA[2], KZ[2], Pn);
                            P = Pn;
                        }
                        LQ_STAMP(14);  // factorisation: KZ, P
                        // the pivot staging and the next stage's slot reads are ordered by the next LMPC_SYNC
                    }
                };
                if (mode != POLISH) sweep(std::true_type{});
                else sweep(std::false_type{});
                LMPC_SYNC();
                if (!red) LQ_ADD_SINCE(15, _lq_fact0);  // the polish's factorisations (also counted in 11-14, 3)
                LQ_STAMP(3);  // factorisation
            }

#ifdef LMPC_LQ_DEBUG
            if (qp == 0 && mode == PRED && ipm_it == 0) {  // QP 0's slots right after the first factorisation
                LMPC_SYNC();
                for (int e = lane; e < lq_lds_doubles(H) && e < 8192; e += 64) lmpc_lq_dbg2[e] = sm[e];
            }
#endif
            // the forward sweep and the inputs, specialised per mode (the polish recomputes each leg's basis)
            auto fwd_inputs = [&](auto mode_tag) {
                constexpr int md = decltype(mode_tag)::value;
                (void)md;
                // ======== forward sweep: w = Z x + za ; x' = A x + d - [0; K w + rho] ========
                if (kzs) {
                    // closed-loop rows: x'[6:12] = x[6:12] + dv - t - KZ x (lanes 4a..4a+3: row a, three terms each, a
                    // quad sum), x'[0:6] = (A x)[0:6] on lanes 0-5
                    struct KzOps {
                        double kz[3], c, ck, sk;
                    };
                    auto load = [&](int k, KzOps& o) {
                        const int ln = lq_lane<WPE>(lane);
                        const int a = ln < 24 ? (ln >> 2) : 0, part = ln & 3;
                        const ldouble* sl = slots + k * LQ_SLOT;
    #pragma unroll
                        for (int i = 0; i < 3; ++i) o.kz[i] = kzr[k * 72 + a * 12 + 3 * part + i];
                        o.c = sl[LQ_DV + a] - sl[LQ_RHO + a];
#ifdef LMPC_BUG_ZA  // diagnostic variant: the same lost "+ za" here, t = K za + rho without K za
    #pragma unroll
                        for (int n = 0; n < 6; ++n) o.c += sl[LQ_K + pk6(a, n)] * sl[LQ_Z + n * 13 + 12];
#endif
#ifdef LMPC_BUG_YAW  // diagnostic variant (tests/test_gpu_kkt.py): the forward sweep reads the next stage's yaw
                        const int ky = k + 1 < H ? k + 1 : k;
#else
                        const int ky = k;
#endif
                        o.ck = cs[2 * ky];
                        o.sk = cs[2 * ky + 1];
                    };
                    KzOps cur, nxt;
                    load(0, cur);
                    if (lane < 12) ex[16 + lane] = hdr[lane];  // x0
                    LMPC_SYNC();
                    for (int k = 0; k < H; ++k) {
                        const int ln = lq_lane<WPE>(lane);
                        const int a = ln < 24 ? (ln >> 2) : 0, part = ln & 3;
                        const int r = ln < 6 ? ln : 0;
                        const ldouble* x = ex + 16;
                        if (!LQ_PF && k > 0) load(k, cur);
                        if (LQ_PF && k + 1 < H) load(k + 1, nxt);
                        double w = cur.kz[0] * x[3 * part];
                        w = fma(cur.kz[1], x[3 * part + 1], w);
                        w = fma(cur.kz[2], x[3 * part + 2], w);
                        const double xa = lq_row_apply(x, r, lq_ax_row(r, cur.ck, cur.sk), dt);
                        const double xv = x[6 + a] + cur.c;
                        w = quad_sum(w);
                        const double xb = xv - w;
                        if (LQ_PF) cur = nxt;
                        LMPC_SYNC();
                        if (ln < 6) {
                            ex[16 + r] = xa;
                            slots[k * LQ_SLOT + LQ_X + r] = xa;
                        }
                        if (ln < 24 && part == 0) {
                            ex[22 + a] = xb;
                            slots[k * LQ_SLOT + LQ_X + 6 + a] = xb;
                        }
                        LMPC_SYNC();
                    }
                } else {
                    struct FwOps {
                        double kr[6], base, za, z[3], ck, sk;
                    };
                    // lane roles from an opaque lane index (addresses computed per stage, never hoisted at 256 registers);
                    // a stage's operands are loaded while the stage before it runs (see the corrector's backward sweep)
                    auto load = [&](int k, FwOps& o) {
                        const int ln = lq_lane<WPE>(lane);
                        const int m = ln < 24 ? (ln >> 2) : 0, part = ln & 3;  // w: lanes 4m..4m+3, 3 terms each
                        const int r = ln < 12 ? ln : 0;
                        const int a = r >= 6 ? r - 6 : 0;
                        const ldouble* sl = slots + k * LQ_SLOT;
    #pragma unroll
                        for (int mm = 0; mm < 6; ++mm) o.kr[mm] = sl[LQ_K + pk6(a, mm)];
                        o.base = sl[LQ_DV + a] - sl[LQ_RHO + a];
                        o.za = sl[LQ_Z + m * 13 + 12];
    #pragma unroll
                        for (int i = 0; i < 3; ++i) o.z[i] = sl[LQ_Z + m * 13 + 3 * part + i];
#ifdef LMPC_BUG_YAW
                        const int ky = k + 1 < H ? k + 1 : k;
#else
                        const int ky = k;
#endif
                        o.ck = cs[2 * ky];
                        o.sk = cs[2 * ky + 1];
                    };
                    FwOps cur, nxt;
                    load(0, cur);
                    if (lane < 12) ex[16 + lane] = hdr[lane];  // x0
                    LMPC_SYNC();
                    for (int k = 0; k < H; ++k) {
                        const int ln = lq_lane<WPE>(lane);
                        const int part = ln & 3;
                        const int r = ln < 12 ? ln : 0;
                        const ldouble* x = ex + 16;
                        if (!LQ_PF && k > 0) load(k, cur);
                        if (LQ_PF && k + 1 < H) load(k + 1, nxt);
                        double w = cur.z[0] * x[3 * part];
                        w = fma(cur.z[1], x[3 * part + 1], w);
                        w = fma(cur.z[2], x[3 * part + 2], w);
                        const double xa = lq_row_apply(x, r, lq_ax_row(r, cur.ck, cur.sk), dt);
#ifdef LMPC_BUG_ZA  // diagnostic variant (tests/test_gpu_kkt.py): round 4's lost "+ za", w = Z x
                        w = quad_sum(w);
#else
                        w = quad_sum(w) + cur.za;
#endif
                        // w_m to every lane (readlane in uniform control flow: all lanes take part in the DPP sums
                        // above, and the broadcast reads lanes 0, 4, ..., 20)
                        double wb[6];
    #pragma unroll
                        for (int mm = 0; mm < 6; ++mm) wb[mm] = readlane_f64(w, 4 * mm);
                        // K w in two independent halves (a shorter dependent chain)
                        double k0 = cur.base, k1 = 0.0;
    #pragma unroll
                        for (int mm = 0; mm < 3; ++mm) {
                            k0 = fma(-cur.kr[mm], wb[mm], k0);
                            k1 = fma(-cur.kr[mm + 3], wb[mm + 3], k1);
                        }
                        const double xn = xa + (r >= 6 ? k0 + k1 : 0.0);
                        if (LQ_PF) cur = nxt;
                        LMPC_SYNC();
                        if (ln < 12) {
                            ex[16 + r] = xn;
                            slots[k * LQ_SLOT + LQ_X + r] = xn;
                        }
                        LMPC_SYNC();
                    }
                }
                LQ_STAMP(4);  // forward sweep
                // ======== inputs from the costate: lambda2 = Z A^-1 x' + za - v2 (-> rho slot), then per leg-step ========
                {
                    constexpr int NT6 = (6 * LMPC_MAX_HORIZON + 63) / 64;
    #pragma unroll
                    for (int i = 0; i < NT6; ++i) {
                        const int e = lq_lane<WPE>(lane) + 64 * i;
                        if (64 * i >= 6 * H) break;  // wave-uniform
                        const int ec = e < 6 * H ? e : 6 * H - 1;
                        const int k = ec / 6, m = ec - 6 * k;
                        const ldouble* sl = slots + k * LQ_SLOT;
                        const ldouble* xk = sl + LQ_X;
                        const double ck = cs[2 * k], sk = cs[2 * k + 1];
                        double lam = sl[LQ_Z + m * 13 + 12] - sl[LQ_V + 6 + m];
    #pragma unroll
                        for (int c = 0; c < 12; ++c) lam = fma(sl[LQ_Z + m * 13 + c], lq_Ax(xk, c, ck, sk, dt, -1.0), lam);
                        if (e < 6 * H) slots[k * LQ_SLOT + LQ_RHO + m] = lam;
                    }
                    LMPC_SYNC();
    #pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        u[t][0] = u[t][1] = u[t][2] = 0.0;
                        if (!st[t]) continue;
                        const int j = lsj[t];
                        const ldouble* lam = slots + lsk[t] * LQ_SLOT + LQ_RHO;
                        double l2[6];
    #pragma unroll
                        for (int mm = 0; mm < 6; ++mm) l2[mm] = lam[mm];
                        // b = rr + T' G0_j' lambda2 ; y = -Rr^-1 b ; u = up + T y
                        double gj[3], b[3], y[3];
    #pragma unroll
                        for (int p = 0; p < 3; ++p) {
                            double v = 0.0;
    #pragma unroll
                            for (int mm = 0; mm < 6; ++mm) v = fma(G0s[mm * 12 + 3 * j + p], l2[mm], v);
                            gj[p] = v;
                        }
                        double T[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}, up[3] = {0.0, 0.0, 0.0};
                        if (md == POLISH) (void)leg_basis(act[t], mu, fzmax, T, up);
    #pragma unroll
                        for (int a = 0; a < 3; ++a) b[a] = -(rr[t][a] + T[0 * 3 + a] * gj[0] + T[1 * 3 + a] * gj[1] + T[2 * 3 + a] * gj[2]);
                        sym3_solve(Rr[t], b, y);
    #pragma unroll
                        for (int p = 0; p < 3; ++p) u[t][p] = up[p] + T[p * 3] * y[0] + T[p * 3 + 1] * y[1] + T[p * 3 + 2] * y[2];
                    }
                }
                LQ_STAMP(5);  // inputs
            };
            if (mode == POLISH) fwd_inputs(std::integral_constant<int, POLISH>{});
            else fwd_inputs(std::integral_constant<int, PRED>{});
#ifdef LMPC_LQ_DEBUG
            // diagnostic build only: QP 0's LDS and inputs after the first predictor solve (tools/lq_debug.py)
            if (qp == 0 && mode == PRED && ipm_it == 0) {
                LMPC_SYNC();
                for (int e = lane; e < lq_lds_doubles(H) && e < 8192; e += 64) lmpc_lq_dbg[e] = sm[e];
#pragma unroll
                for (int t = 0; t < LS; ++t)
#pragma unroll
                    for (int m = 0; m < 3; ++m) lmpc_lq_dbg_u[(lane + 64 * t) * 3 + m] = u[t][m];
            }
#endif

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
                // corrector linear term rr' = C' w'
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    double wv[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        wv[i] = (z[t][i] * (s[t][i] - (i == 4 ? fzmax : 0.0)) + smu - dsa[t][i] * dza[t][i]) * rcp_nr(s[t][i]);
                    cons_tw(wv, mu, rr[t]);
                }
                mode = CORR;
                LQ_STAMP(6);  // predictor step
            } else if (mode == CORR) {
                double ds[LS][5], dz[LS][5];
                double amax = 1.0, dmax = 1.0;
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
                        const double dsa = -oa[i] - s[t][i];
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
                LQ_STAMP(7);  // corrector step
            } else {
                ++prounds;
                // ======== polish verification, a KKT certificate independent of the factorisation: the trajectory
                // the forward sweep produced must be the dynamics of the forces returned (x_{k+1} = A_k x_k + B u_k -
                // g dt e11, every row at once), the adjoint lambda of that trajectory gives the gradient, and every
                // stance leg-step must then be primal feasible, stationary on its free directions and carry
                // multipliers of the right sign (lmpc_kernels.hip) ========
                bool dyn_ok;  // wave-uniform: the dynamics residual within tol_p of the state scale (max |x|, >= 1)
#ifdef LMPC_KKT_DIAG
                double lmpc_kkt_dyn;
#endif
                {
                    // B u_k per stage (rows 6-11: G0 u_k, summed over the stage's legs) -> the dv field, dead until
                    // the next leg-step work rewrites it
#pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        const int j = lsj[t];
                        double bu[6];
#pragma unroll
                        for (int m = 0; m < 6; ++m)
                            bu[m] = quad_sum(fma(G0s[m * 12 + 3 * j], u[t][0],
                                                 fma(G0s[m * 12 + 3 * j + 1], u[t][1], G0s[m * 12 + 3 * j + 2] * u[t][2])));
                        if (valid[t] && j == 0) {
#pragma unroll
                            for (int m = 0; m < 6; ++m) slots[lsk[t] * LQ_SLOT + LQ_DV + m] = bu[m];
                        }
                    }
                    LMPC_SYNC();
                    // every dynamics row at once: x_{j+1} - (A_j x_j + B u_j - g dt e11), x_0 from the record
                    constexpr int NTQ = LS == 1 ? 3 : 6;
                    double dres = 0.0, xsc = 1.0;
#pragma unroll 1  // unrolled, its loads all in flight at once push the two-leg-step instances into spills
                    for (int i = 0; i < NTQ; ++i) {
                        const int e = lq_lane<WPE>(lane) + 64 * i, ec = e < 12 * H ? e : 12 * H - 1;
                        const int j = ec / 12, rr_ = ec - 12 * j;
                        const ldouble* xk = j > 0 ? slots + (j - 1) * LQ_SLOT + LQ_X : hdr;
                        const int m = rr_ >= 6 ? rr_ - 6 : 0;
                        const double pred = lq_row_apply(xk, rr_, lq_ax_row(rr_, cs[2 * j], cs[2 * j + 1]), dt) +
                                            (rr_ >= 6 ? slots[j * LQ_SLOT + LQ_DV + m] - (m == 5 ? prm.grav * dt : 0.0) : 0.0);
                        const double xn = slots[j * LQ_SLOT + LQ_X + rr_];
                        if (e < 12 * H) {
                            dres = fmax(dres, fabs(xn - pred));
                            xsc = fmax(xsc, fabs(xn));
                        }
                    }
                    {
                        const double dmax = wave_max(dres), xmax = wave_max(xsc);
                        dyn_ok = dmax <= prm.tol_x * xmax;
#ifdef LMPC_KKT_DIAG
                        lmpc_kkt_dyn = dmax / xmax;
#endif
                    }
                    LMPC_SYNC();  // every read of x ahead of the tracking terms over it
                }
                {
                    // tracking terms q (x_k - x_ref,k-1) of every stage at once -> x slot (dead after this), then the
                    // serial sweep lambda_k = q_k-term + A_k' lambda_{k+1}, lambda_{k+1}[6:12] -> rho slot k
                    const int lnv = lq_lane<WPE>(lane), r = lnv < 12 ? lnv : 0;
                    {
                        constexpr int NTQ = LS == 1 ? 3 : 6;
                        double xl[NTQ];
#pragma unroll
                        for (int i = 0; i < NTQ; ++i) xl[i] = xr[min(lq_lane<WPE>(lane) + 64 * i, 12 * H - 1)];
#pragma unroll
                        for (int i = 0; i < NTQ; ++i) {
                            const int e = lq_lane<WPE>(lane) + 64 * i, j = e / 12, rr_ = e - 12 * j;
                            if (e < 12 * H) {
                                ldouble* xs = slots + j * LQ_SLOT + LQ_X + rr_;
                                xs[0] = qw[rr_] * (xs[0] - xl[i]);
                            }
                        }
                        LMPC_SYNC();
                    }
                    double lam = lnv < 12 ? slots[(H - 1) * LQ_SLOT + LQ_X + r] : 0.0;
                    for (int k = H - 1; k >= 0; --k) {
                        if (lnv < 12) ex[r] = lam;
                        if (lnv >= 6 && lnv < 12) slots[k * LQ_SLOT + LQ_RHO + (lnv - 6)] = lam;
                        // the stage's own operands ahead of the fence (they do not depend on the exchange)
                        const int kp = k > 0 ? k - 1 : 0;
                        const double q = slots[kp * LQ_SLOT + LQ_X + r], ck = cs[2 * k], sk = cs[2 * k + 1];
                        LMPC_SYNC();
                        if (k == 0) break;
                        lam = q + lq_row_apply(ex, r, lq_atw_row(r, ck, sk), dt);
                        LMPC_SYNC();
                    }
                }
                LQ_STAMP(8);  // adjoint
                double g[LS][3];
                double gloc = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    g[t][0] = g[t][1] = g[t][2] = 0.0;
                    if (!valid[t]) continue;
                    const int j = lsj[t];
                    const ldouble* lam = slots + lsk[t] * LQ_SLOT + LQ_RHO;
                    double ru[3];
                    if constexpr (!TERRAIN) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) ru[p] = prm.r[3 * j + p] * u[t][p];
                    } else {
                        const ldouble* rb = rbt + 6 * j;
                        ru[0] = rb[0] * u[t][0] + rb[1] * u[t][1] + rb[2] * u[t][2];
                        ru[1] = rb[1] * u[t][0] + rb[3] * u[t][1] + rb[4] * u[t][2];
                        ru[2] = rb[2] * u[t][0] + rb[4] * u[t][1] + rb[5] * u[t][2];
                    }
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        double v = ru[p];
#pragma unroll
                        for (int m = 0; m < 6; ++m) v += G0s[m * 12 + 3 * j + p] * lam[m];
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
                    if (apex[t]) {  // the cone test is the whole certificate at the apex (f = 0, every direction bound)
                        if (g[t][2] / mu < fabs(g[t][0]) + fabs(g[t][1]) - prm.tol_d * gscale) {
                            act[t] = (g[t][0] < 0.0 ? 2 : 1) | (g[t][1] < 0.0 ? 8 : 4);
                            changed = 1;
                        }
                        continue;
                    }
                    // (act = 0: no multipliers, the residual is g itself)
                    const LegKkt kk = leg_kkt(act[t], g[t], mu, -prm.tol_d * gscale);
                    if (kk.drop >= 0) {
                        act[t] &= ~(1 << kk.drop);
                        changed = 1;
                    }
                    sres = fmax(sres, kk.res);
                }
                LQ_STAMP(9);  // polish verification
                if (!__any(changed)) {
                    // the active set is settled: it is the optimum's only if the trajectory is the forces' own and the
                    // gradient vanishes on every free direction; otherwise this attempt cannot verify (another round
                    // would repeat it bit for bit) and the retry ladder takes over
                    const double sr = wave_max(sres);
#ifdef LMPC_KKT_DIAG
                    if (lane == 0 && qp < LMPC_KKT_DIAG_QPS) {
                        lmpc_kkt_diag[qp][0] = sr / gscale;
                        lmpc_kkt_diag[qp][1] = lmpc_kkt_dyn;
                        lmpc_kkt_diag[qp][2] = gscale;
                        lmpc_kkt_diag[qp][3] = (double)prounds;
                    }
#endif
#ifndef LMPC_KKT_OFF
                    if (sr <= prm.tol_d * gscale && dyn_ok)
#endif
                    {
                        done = true;
                        break;
                    }
                    if (LQ_RP && !dyn_ok && !rp_off) {
                        rp_off = true;  // the same active set again, every polish stage in full inputs
                        continue;
                    }
                    rd = prm.max_rounds - 1;
                }
                if (++rd >= prm.max_rounds) {
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
        qstatus = LMPC_QP_MAX_ITER;  // no verified active set: the (feasible) interior-point iterate
#pragma unroll
        for (int t = 0; t < LS; ++t)
#pragma unroll
            for (int m = 0; m < 3; ++m) u[t][m] = f[t][m];
    }
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
        if constexpr (TERRAIN) {
            const ldouble* Rj = tf + 9 * lsj[t];
#pragma unroll
            for (int p = 0; p < 3; ++p) fo[p] = Rj[3 * p] * u[t][0] + Rj[3 * p + 1] * u[t][1] + Rj[3 * p + 2] * u[t][2];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) gout[3 * ls + p] = (anybad || !st[t]) ? 0.0 : fo[p];
    }
    if (lane == 0) {
        if (status) status[qp] = anybad ? LMPC_QP_NAN : qstatus;
        if (iters) iters[qp] = ipm_it | (prounds << 16);
    }
    LQ_STAMP(10);
    LQ_STAMP_FLUSH(qp);
}

}  // namespace lmpc

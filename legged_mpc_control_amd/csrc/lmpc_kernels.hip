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

namespace lmpc {

#define LMPC_SYNC() __syncthreads()

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of QP 0..STAMP_QPS-1,
// written to a buffer no other code reads.  Never compiled into the product library.
#ifdef LMPC_STAMPS
constexpr int STAMP_QPS = 4096;
__device__ unsigned long long lmpc_stamps[STAMP_QPS][8];
#define STAMP_DECL unsigned long long _st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _st_t0 = __builtin_readcyclecounter();
#define STAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _st_acc[i] += _t - _st_t0; _st_t0 = _t; } while (0)
#define STAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < STAMP_QPS) for (int _i = 0; _i < 8; ++_i) lmpc_stamps[qp][_i] = _st_acc[_i]; } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH(qp) do {} while (0)
#endif
// Explicit LDS address space: every shared access compiles to ds_read/ds_write
// (a generic pointer would fall back to flat_load/flat_store).
typedef __attribute__((address_space(3))) double ldouble;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
// sum over the 4 lanes of a stage (lanes 4q..4q+3 = legs of one stage)
__device__ __forceinline__ double quad_sum(double v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    return v;
}

__device__ __forceinline__ int pk(int r, int c) { return r * (r + 1) / 2 + c; }  // packed lower, c <= r

// inverse of pk: packed index -> (r, c)
__device__ __forceinline__ void unpk(int e, int& r, int& c) {
    r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    if (r * (r + 1) / 2 > e) --r;
    if ((r + 1) * (r + 2) / 2 <= e) ++r;
    c = e - r * (r + 1) / 2;
}

// ---- friction pyramid, flat ground (ConvexQPSolver.cpp:131-172) ------------
// rows: c0 -fx-mu fz <= 0 | c1 fx-mu fz <= 0 | c2 -fy-mu fz <= 0 | c3 fy-mu fz <= 0 | c4 fz <= fzmax
__device__ __forceinline__ void cons_resid(const double f[3], double mu, double fzmax, double o[5]) {
    o[0] = -f[0] - mu * f[2];
    o[1] = f[0] - mu * f[2];
    o[2] = -f[1] - mu * f[2];
    o[3] = f[1] - mu * f[2];
    o[4] = f[2] - fzmax;
}
__device__ __forceinline__ void cons_rowvec(int i, double mu, double c[3]) {
    c[0] = (i == 0) ? -1.0 : (i == 1) ? 1.0 : 0.0;
    c[1] = (i == 2) ? -1.0 : (i == 3) ? 1.0 : 0.0;
    c[2] = (i == 4) ? 1.0 : -mu;
}
__device__ __forceinline__ void cons_tw(const double w[5], double mu, double o[3]) {
    o[0] = -w[0] + w[1];
    o[1] = -w[2] + w[3];
    o[2] = -mu * (w[0] + w[1] + w[2] + w[3]) + w[4];
}

// M(yaw) = [c s 0; -s c 0; 0 0 1]  (ang_vel_to_rpy_rate, ConvexQPSolver.cpp:220-222)
__device__ __forceinline__ double Myaw(double c, double s, int i, int j) {
    if (i == 2) return j == 2 ? 1.0 : 0.0;
    if (j == 2) return 0.0;
    if (i == 0) return j == 0 ? c : s;
    return j == 0 ? -s : c;
}

// ---- LDS layout (doubles) --------------------------------------------------
// per-stage slot
constexpr int SO_RR = 0;     // 4 x 3x3 input Hessian blocks T'RtT
constexpr int SO_BT = 36;    // 6 x 12 Bt = G0 T
constexpr int SO_DV = 108;   // 6   d_k[6:12] = G0 up - g dt e5
constexpr int SO_RRV = 114;  // 12  input linear term rr (later: y)
constexpr int SO_KZ = 126;   // 6 x 12 K Z
constexpr int SO_VV = 198;   // 12  v = P_{k+1} d_k
constexpr int SO_CST = 210;  // 12  q_k - Z' psi
constexpr int SO_PSI = 222;  // 6   V' L^-1 rr
constexpr int SO_RHO = 228;  // 12  L^-1 rr (later: t)
constexpr int SO_S2 = 240;   // 6   (v + p_{k+1})[6:12]
constexpr int SO_N6 = 246;   // 6   K s2 + psi (later: q2)
constexpr int SO_XS = 252;   // 12  x_k
constexpr int SO_LAM = 264;  // 12  lambda_{k+1}
constexpr int SK = 276;
// global scratch per stage
constexpr int GO_LINV = 0;   // 78 packed L^-1
constexpr int GO_V = 78;     // 12 x 6 V = L^-1 Bt'
constexpr int GO_K = 150;    // 21 packed K
constexpr int GO_P2 = 171;   // 6 x 12 rows 6..11 of P_{k+1}
constexpr int GS = 243;

struct Smem {
    ldouble* G0;   // 72
    ldouble* hdr;  // 40: x0(12) R(9) feet(12)
    ldouble* cs;   // 2H
    ldouble* xr;   // 12H
    ldouble* xH;   // 12
    ldouble* P;    // 144
    ldouble* APA;  // 144
    ldouble* C;    // 72   P22 Bt
    ldouble* Z;    // 72   P2 A
    ldouble* G;    // 144  Guu -> L
    ldouble* RV;   // 12 x 18  [Bt' | I] -> [V | L^-1]
    ldouble* LP;   // 27   panel
    ldouble* XB;   // 54   panel rhs rows
    ldouble* K;    // 36
    ldouble* pa;   // 12
    ldouble* pb;   // 12
    ldouble* st;   // H * SK
};

__device__ __forceinline__ Smem carve(double* sm, int H) {
    Smem s;
    ldouble* p = (ldouble*)sm;
    s.G0 = p; p += 72;
    s.hdr = p; p += 40;
    s.cs = p; p += 2 * H;
    s.xr = p; p += 12 * H;
    s.xH = p; p += 12;
    s.P = p; p += 144;
    s.APA = p; p += 144;
    s.C = p; p += 72;
    s.Z = p; p += 72;
    s.G = p; p += 144;
    s.RV = p; p += 216;
    s.LP = p; p += 28;
    s.XB = p; p += 54;
    s.K = p; p += 36;
    s.pa = p; p += 12;
    s.pb = p; p += 12;
    s.st = p;  // offset 1058 + 14H doubles (even: 16-B aligned)
    return s;
}

// (P N)[r][c] with N the nilpotent part of A = I + dt N
template <class Ptr>
__device__ __forceinline__ double PNel(Ptr P, int r, int c, double ck, double sk) {
    if (c >= 6 && c < 9) {
        return P[r * 12 + 0] * Myaw(ck, sk, 0, c - 6) + P[r * 12 + 1] * Myaw(ck, sk, 1, c - 6) +
               P[r * 12 + 2] * Myaw(ck, sk, 2, c - 6);
    }
    if (c >= 9) return P[r * 12 + c - 6];
    return 0.0;
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
// Riccati factorisation (backward, matrix part)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void riccati_factor(const DevParams& prm, const Smem& S, double* __restrict__ gs, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    for (int e = lane; e < 144; e += 64) S.P[e] = (e % 13 == 0) ? prm.q[e / 13] : 0.0;
    LMPC_SYNC();
    for (int k = H - 1; k >= 0; --k) {
        const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
        ldouble* sl = S.st + k * SK;
        double* g = gs + k * GS;
        const ldouble* Bt = sl + SO_BT;
        // ---- level A: C = P22 Bt, Z = P2 A (+P2 -> global), v = P d, APA = A'PA ----
        for (int e = lane; e < 72 + 72 + 12 + 78; e += 64) {
            if (e < 72) {
                const int m = e / 12, c = e % 12;
                double v = 0.0;
#pragma unroll
                for (int n = 0; n < 6; ++n) v += S.P[(6 + m) * 12 + 6 + n] * Bt[n * 12 + c];
                S.C[e] = v;
            } else if (e < 144) {
                const int e2 = e - 72, m = e2 / 12, c = e2 % 12;
                const double p = S.P[(6 + m) * 12 + c];
                S.Z[e2] = p + dt * PNel(S.P, 6 + m, c, ck, sk);
                g[GO_P2 + e2] = p;
            } else if (e < 156) {
                const int r = e - 144;
                double v = 0.0;
#pragma unroll
                for (int n = 0; n < 6; ++n) v += S.P[r * 12 + 6 + n] * sl[SO_DV + n];
                sl[SO_VV + r] = v;
            } else {
                // lower-triangle entry (r, c) of A'PA = P + dt(PN + N'P) + dt^2 N'PN
                int r, c;
                unpk(e - 156, r, c);
                double v = S.P[r * 12 + c] + dt * (PNel(S.P, r, c, ck, sk) + PNel(S.P, c, r, ck, sk));
                double npn = 0.0;
                if (r >= 6 && r < 9) {
#pragma unroll
                    for (int i = 0; i < 3; ++i) npn += Myaw(ck, sk, i, r - 6) * PNel(S.P, i, c, ck, sk);
                } else if (r >= 9) {
                    npn = PNel(S.P, r - 6, c, ck, sk);
                }
                v += dt * dt * npn;
                S.APA[r * 12 + c] = v;
                S.APA[c * 12 + r] = v;
            }
        }
        LMPC_SYNC();
        // ---- level B: Guu = blockdiag(Rr) + Bt' C (lower) ----
        for (int e = lane; e < 78; e += 64) {
            int r, c;
            unpk(e, r, c);
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) v += Bt[m * 12 + r] * S.C[m * 12 + c];
            if (r / 3 == c / 3) v += sl[SO_RR + (r / 3) * 9 + (r % 3) * 3 + (c % 3)];
            S.G[r * 12 + c] = v;
        }
        LMPC_SYNC();
        // ---- levels C: block Cholesky by legs, RHS [Bt' | I] eliminated alongside ----
        for (int a = 0; a < 4; ++a) {
            const int o = 3 * a;
            const double g00 = S.G[o * 12 + o], g10 = S.G[(o + 1) * 12 + o], g11 = S.G[(o + 1) * 12 + o + 1];
            const double g20 = S.G[(o + 2) * 12 + o], g21 = S.G[(o + 2) * 12 + o + 1], g22 = S.G[(o + 2) * 12 + o + 2];
            const double l00 = sqrt(g00), i00 = 1.0 / l00;
            const double l10 = g10 * i00, l20 = g20 * i00;
            const double l11 = sqrt(g11 - l10 * l10), i11 = 1.0 / l11;
            const double l21 = (g21 - l20 * l10) * i11;
            const double l22 = sqrt(g22 - l20 * l20 - l21 * l21), i22 = 1.0 / l22;
            // Lai = L_aa^-1 (lower)
            const double m10 = -l10 * i00 * i11;
            const double m21 = -l21 * i11 * i22;
            const double m20 = -(l20 * i00 + l21 * m10) * i22;
            const double Lai[3][3] = {{i00, 0.0, 0.0}, {m10, i11, 0.0}, {m20, m21, i22}};
            const int npan = 9 * (3 - a);
            // panel: L_ba = G_ba L_aa^-T (b > a), X_a = L_aa^-1 RHS_a
            for (int e = lane; e < npan + 54; e += 64) {
                if (e < npan) {
                    const int bb = a + 1 + e / 9, i = (e % 9) / 3, j = e % 3;
                    // L_ba[i][j] = sum_{q<=j} G_ba[i][q] Lai[j][q]  (Lai lower: zero above the diagonal)
                    const double w0 = (j == 0) ? Lai[0][0] : (j == 1) ? Lai[1][0] : Lai[2][0];
                    const double w1 = (j == 0) ? 0.0 : (j == 1) ? Lai[1][1] : Lai[2][1];
                    const double w2 = (j == 2) ? Lai[2][2] : 0.0;
                    const int gr = (3 * bb + i) * 12 + o;
                    S.LP[e] = S.G[gr] * w0 + S.G[gr + 1] * w1 + S.G[gr + 2] * w2;
                } else {
                    const int e2 = e - npan, i = e2 / 18, c = e2 % 18;
                    double rhs[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        const int row = o + q;
                        rhs[q] = (a == 0) ? ((c < 6) ? Bt[c * 12 + row] : (c - 6 == row ? 1.0 : 0.0)) : S.RV[row * 18 + c];
                    }
                    const double w0 = (i == 0) ? Lai[0][0] : (i == 1) ? Lai[1][0] : Lai[2][0];
                    const double w1 = (i == 0) ? 0.0 : (i == 1) ? Lai[1][1] : Lai[2][1];
                    const double w2 = (i == 2) ? Lai[2][2] : 0.0;
                    S.XB[e2] = w0 * rhs[0] + w1 * rhs[1] + w2 * rhs[2];
                }
            }
            LMPC_SYNC();
            // trailing update of G (lower blocks b >= c > a) and RHS rows b > a
            const int nb = 3 - a;
            const int ntr = 9 * nb * (nb + 1) / 2;
            const int nrv = 54 * nb;
            for (int e = lane; e < ntr + nrv; e += 64) {
                if (e < ntr) {
                    int blk = e / 9, b2 = a + 1, c2 = a + 1;
                    while (blk > 0) {
                        if (c2 < b2) ++c2;
                        else { ++b2; c2 = a + 1; }
                        --blk;
                    }
                    const int i = (e % 9) / 3, j = e % 3;
                    const ldouble* Lb = S.LP + (b2 - a - 1) * 9;
                    const ldouble* Lc = S.LP + (c2 - a - 1) * 9;
                    double v = S.G[(3 * b2 + i) * 12 + 3 * c2 + j];
#pragma unroll
                    for (int q = 0; q < 3; ++q) v -= Lb[i * 3 + q] * Lc[j * 3 + q];
                    S.G[(3 * b2 + i) * 12 + 3 * c2 + j] = v;
                } else {
                    const int e2 = e - ntr, b2 = a + 1 + e2 / 54, i = (e2 % 54) / 18, c = e2 % 18;
                    const int row = 3 * b2 + i;
                    const ldouble* Lb = S.LP + (b2 - a - 1) * 9;
                    double v = (a == 0) ? ((c < 6) ? Bt[c * 12 + row] : (c - 6 == row ? 1.0 : 0.0)) : S.RV[row * 18 + c];
#pragma unroll
                    for (int q = 0; q < 3; ++q) v -= Lb[i * 3 + q] * S.XB[q * 18 + c];
                    S.RV[row * 18 + c] = v;
                }
            }
            // commit X_a -> RV rows o..o+2 (final rows of [V | L^-1]); rows > o+2 only touched above
            for (int e = lane; e < 54; e += 64) S.RV[(o + e / 18) * 18 + e % 18] = S.XB[e];
            LMPC_SYNC();
        }
        // ---- level D: K = V'V ; store L^-1, V, K to the global scratch ----
        for (int e = lane; e < 21 + 78 + 72; e += 64) {
            if (e < 21) {
                int m, n;
                unpk(e, m, n);
                double v = 0.0;
#pragma unroll
                for (int r = 0; r < 12; ++r) v += S.RV[r * 18 + m] * S.RV[r * 18 + n];
                S.K[m * 6 + n] = v;
                S.K[n * 6 + m] = v;
                g[GO_K + e] = v;
            } else if (e < 99) {
                int r, c;
                unpk(e - 21, r, c);
                g[GO_LINV + e - 21] = S.RV[r * 18 + 6 + c];
            } else {
                const int e2 = e - 99;
                g[GO_V + e2] = S.RV[(e2 / 6) * 18 + e2 % 6];
            }
        }
        LMPC_SYNC();
        // ---- level E: KZ = K Z ----
        for (int e = lane; e < 72; e += 64) {
            const int m = e / 12, c = e % 12;
            double v = 0.0;
#pragma unroll
            for (int n = 0; n < 6; ++n) v += S.K[m * 6 + n] * S.Z[n * 12 + c];
            sl[SO_KZ + e] = v;
        }
        LMPC_SYNC();
        // ---- level F: P_k = Q + A'PA - Z'(KZ) ----
        if (k > 0) {
            for (int e = lane; e < 78; e += 64) {
                int r, c;
                unpk(e, r, c);
                double v = S.APA[r * 12 + c] + (r == c ? prm.q[r] : 0.0);
#pragma unroll
                for (int m = 0; m < 6; ++m) v -= S.Z[m * 12 + r] * sl[SO_KZ + m * 12 + c];
                S.P[r * 12 + c] = v;
                S.P[c * 12 + r] = v;
            }
            LMPC_SYNC();
        }
    }
}

// ---------------------------------------------------------------------------
// Vector pass: pre-pass, backward/forward affine recursions, post-pass.
// Reads SO_RRV (rr) per stage; leaves y (12 per stage) in SO_RRV and x_k in SO_XS / xH.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void riccati_solve(const DevParams& prm, const Smem& S, const double* __restrict__ gs, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    // pre 1: rho = L^-1 rr
    for (int e = lane; e < 12 * H; e += 64) {
        const int k = e / 12, r = e % 12;
        const double* Li = gs + k * GS + GO_LINV + pk(r, 0);
        const ldouble* rr = S.st + k * SK + SO_RRV;
        double v = 0.0;
        for (int c = 0; c <= r; ++c) v += Li[c] * rr[c];
        S.st[k * SK + SO_RHO + r] = v;
    }
    LMPC_SYNC();
    // pre 2: psi = V' rho
    for (int e = lane; e < 6 * H; e += 64) {
        const int k = e / 6, m = e % 6;
        const double* V = gs + k * GS + GO_V;
        const ldouble* rho = S.st + k * SK + SO_RHO;
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 12; ++r) v += V[r * 6 + m] * rho[r];
        S.st[k * SK + SO_PSI + m] = v;
    }
    LMPC_SYNC();
    // pre 3: cst_k = q_k - A_k' P2' psi   (k >= 1)
    for (int e = lane; e < 12 * H; e += 64) {
        const int k = e / 12, r = e % 12;
        if (k == 0) continue;
        const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
        const double* P2 = gs + k * GS + GO_P2;
        const ldouble* psi = S.st + k * SK + SO_PSI;
        double w[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) v += P2[m * 12 + c] * psi[m];
            w[c] = v;
        }
        S.st[k * SK + SO_CST + r] = -prm.q[r] * S.xr[(k - 1) * 12 + r] - Atw_el(w, r, ck, sk, dt);
    }
    if (lane < 12) S.pa[lane] = -prm.q[lane] * S.xr[(H - 1) * 12 + lane];
    LMPC_SYNC();
    // backward: s = v_k + p_{k+1};  p_k = A's - (KZ)' s2 + cst_k
    ldouble* pcur = S.pa;
    ldouble* pnxt = S.pb;
    for (int k = H - 1; k >= 0; --k) {
        const ldouble* sl = S.st + k * SK;
        if (lane < 12 && k > 0) {
            const int r = lane;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            double sv[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) sv[i] = sl[SO_VV + i] + pcur[i];
            double v = Atw_el(sv, r, ck, sk, dt);
#pragma unroll
            for (int m = 0; m < 6; ++m) v -= sl[SO_KZ + m * 12 + r] * sv[6 + m];
            pnxt[r] = v + sl[SO_CST + r];
        } else if (lane >= 16 && lane < 22) {
            const int m = lane - 16;
            S.st[k * SK + SO_S2 + m] = sl[SO_VV + 6 + m] + pcur[6 + m];
        }
        LMPC_SYNC();
        ldouble* t = pcur;
        pcur = pnxt;
        pnxt = t;
    }
    // n6 = K s2 + psi
    for (int e = lane; e < 6 * H; e += 64) {
        const int k = e / 6, m = e % 6;
        const double* Kp = gs + k * GS + GO_K;
        const ldouble* s2 = S.st + k * SK + SO_S2;
        double v = S.st[k * SK + SO_PSI + m];
#pragma unroll
        for (int n = 0; n < 6; ++n) v += Kp[m >= n ? pk(m, n) : pk(n, m)] * s2[n];
        S.st[k * SK + SO_N6 + m] = v;
    }
    if (lane < 12) S.st[SO_XS + lane] = S.hdr[lane];
    LMPC_SYNC();
    // forward: x_{k+1} = A x - [0; KZ x + n6 - dv]
    for (int k = 0; k < H; ++k) {
        const ldouble* sl = S.st + k * SK;
        ldouble* xo = (k + 1 < H) ? S.st + (k + 1) * SK + SO_XS : S.xH;
        if (lane < 12) {
            const int r = lane;
            const ldouble* x = sl + SO_XS;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            double v = Ax_el(x, r, ck, sk, dt);
            if (r >= 6) {
                double kz = 0.0;
#pragma unroll
                for (int c = 0; c < 12; ++c) kz += sl[SO_KZ + (r - 6) * 12 + c] * x[c];
                v += -kz - sl[SO_N6 + r - 6] + sl[SO_DV + r - 6];
            }
            xo[r] = v;
        }
        LMPC_SYNC();
    }
    // post 1: q2 = P2 (A x_k) + s2   -> SO_N6
    for (int e = lane; e < 6 * H; e += 64) {
        const int k = e / 6, m = e % 6;
        const double* P2 = gs + k * GS + GO_P2;
        const ldouble* x = S.st + k * SK + SO_XS;
        const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
        double v = S.st[k * SK + SO_S2 + m];
#pragma unroll
        for (int c = 0; c < 12; ++c) v += P2[m * 12 + c] * Ax_el(x, c, ck, sk, dt);
        S.st[k * SK + SO_N6 + m] = v;
    }
    LMPC_SYNC();
    // post 2: t = V q2 + rho  -> SO_RHO
    for (int e = lane; e < 12 * H; e += 64) {
        const int k = e / 12, r = e % 12;
        const double* V = gs + k * GS + GO_V;
        double v = S.st[k * SK + SO_RHO + r];
#pragma unroll
        for (int m = 0; m < 6; ++m) v += V[r * 6 + m] * S.st[k * SK + SO_N6 + m];
        S.st[k * SK + SO_RHO + r] = v;
    }
    LMPC_SYNC();
    // post 3: y = -L^-T t  -> SO_RRV
    for (int e = lane; e < 12 * H; e += 64) {
        const int k = e / 12, c = e % 12;
        const double* Li = gs + k * GS + GO_LINV;
        const ldouble* t = S.st + k * SK + SO_RHO;
        double v = 0.0;
        for (int r = c; r < 12; ++r) v += Li[pk(r, c)] * t[r];
        S.st[k * SK + SO_RRV + c] = -v;
    }
    LMPC_SYNC();
}

// Adjoint: lambda_{k+1} for every stage (SO_LAM) from the trajectory in SO_XS / xH.
__device__ __forceinline__ void adjoint(const DevParams& prm, const Smem& S, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    if (lane < 12) S.st[(H - 1) * SK + SO_LAM + lane] = prm.q[lane] * (S.xH[lane] - S.xr[(H - 1) * 12 + lane]);
    LMPC_SYNC();
    for (int k = H - 1; k >= 1; --k) {
        if (lane < 12) {
            const int r = lane;
            const ldouble* lam = S.st + k * SK + SO_LAM;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            S.st[(k - 1) * SK + SO_LAM + r] =
                prm.q[r] * (S.st[k * SK + SO_XS + r] - S.xr[(k - 1) * 12 + r]) + Atw_el(lam, r, ck, sk, dt);
        }
        LMPC_SYNC();
    }
}

// Null-space parametrisation of one leg-step for active set `act` (bit i = row ci):
// f = up + T y, T columns orthonormal.  Returns true at the pyramid apex (f = 0).
__device__ bool leg_basis(int act, double mu, double fzmax, double T[9], double up[3]) {
#pragma unroll
    for (int i = 0; i < 9; ++i) T[i] = 0.0;
    up[0] = up[1] = up[2] = 0.0;
    if ((act & 3) == 3 || (act & 12) == 12) return true;
    double rows[3][3], bs[3];
    int nr = 0;
    for (int i = 0; i < 5; ++i) {
        if (!((act >> i) & 1) || nr >= 3) continue;
        cons_rowvec(i, mu, rows[nr]);
        bs[nr] = (i == 4) ? fzmax : 0.0;
        ++nr;
    }
    double qv[3][3];
    for (int a = 0; a < nr; ++a) {
        double v[3] = {rows[a][0], rows[a][1], rows[a][2]};
        for (int b = 0; b < a; ++b) {
            const double d = qv[b][0] * v[0] + qv[b][1] * v[1] + qv[b][2] * v[2];
            v[0] -= d * qv[b][0];
            v[1] -= d * qv[b][1];
            v[2] -= d * qv[b][2];
        }
        const double n = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        qv[a][0] = v[0] * n;
        qv[a][1] = v[1] * n;
        qv[a][2] = v[2] * n;
    }
    {
        double beta[3] = {0.0, 0.0, 0.0};
        for (int a = 0; a < nr; ++a) {
            double s = bs[a];
            for (int b = 0; b < a; ++b)
                s -= (rows[a][0] * qv[b][0] + rows[a][1] * qv[b][1] + rows[a][2] * qv[b][2]) * beta[b];
            const double diag = rows[a][0] * qv[a][0] + rows[a][1] * qv[a][1] + rows[a][2] * qv[a][2];
            beta[a] = s / diag;
        }
        for (int a = 0; a < nr; ++a)
            for (int i = 0; i < 3; ++i) up[i] += beta[a] * qv[a][i];
    }
    if (nr == 0) {
        T[0] = T[4] = T[8] = 1.0;
    } else if (nr == 1) {
        const double* n = qv[0];
        double e[3] = {0.0, 0.0, 0.0};
        if (fabs(n[0]) < 0.9) e[0] = 1.0;
        else e[1] = 1.0;
        const double d = n[0] * e[0] + n[1] * e[1] + n[2] * e[2];
        double t1[3] = {e[0] - d * n[0], e[1] - d * n[1], e[2] - d * n[2]};
        const double in = 1.0 / sqrt(t1[0] * t1[0] + t1[1] * t1[1] + t1[2] * t1[2]);
        t1[0] *= in;
        t1[1] *= in;
        t1[2] *= in;
        const double t2[3] = {n[1] * t1[2] - n[2] * t1[1], n[2] * t1[0] - n[0] * t1[2], n[0] * t1[1] - n[1] * t1[0]};
        for (int i = 0; i < 3; ++i) {
            T[i * 3 + 0] = t1[i];
            T[i * 3 + 1] = t2[i];
        }
    } else if (nr == 2) {
        double t[3] = {qv[0][1] * qv[1][2] - qv[0][2] * qv[1][1], qv[0][2] * qv[1][0] - qv[0][0] * qv[1][2],
                       qv[0][0] * qv[1][1] - qv[0][1] * qv[1][0]};
        const double in = 1.0 / sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        for (int i = 0; i < 3; ++i) T[i * 3 + 0] = t[i] * in;
    }
    return false;
}

// Per-leg-step stage data: Rr = T'RtT (fixed components -> identity), Bt = G0_j T, dv (quad-reduced).
// Rt is the symmetric input Hessian block [xx xy xz yy yz zz].  Must be called by ALL lanes.
template <int LS>
__device__ __forceinline__ void leg_stage_prep(const DevParams& prm, const Smem& S, const bool (&valid)[LS],
                                               const int (&lsk)[LS], const int (&lsj)[LS], const double (&Rt)[LS][6],
                                               const double (&T)[LS][9], const double (&up)[LS][3]) {
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        double du[6] = {0, 0, 0, 0, 0, 0};
        if (valid[t]) {
            const int k = lsk[t], j = lsj[t];
            ldouble* sl = S.st + k * SK;
            const double R3[9] = {Rt[t][0], Rt[t][1], Rt[t][2], Rt[t][1], Rt[t][3], Rt[t][4], Rt[t][2], Rt[t][4], Rt[t][5]};
            bool fixed[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) fixed[a] = (T[t][a] == 0.0 && T[t][3 + a] == 0.0 && T[t][6 + a] == 0.0);
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
                    sl[SO_RR + j * 9 + a * 3 + b] = v;
                }
#pragma unroll
            for (int m = 0; m < 6; ++m) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double v = 0.0;
#pragma unroll
                    for (int p = 0; p < 3; ++p) v += S.G0[m * 12 + 3 * j + p] * T[t][p * 3 + a];
                    sl[SO_BT + m * 12 + 3 * j + a] = v;
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
            ldouble* sl = S.st + lsk[t] * SK;
#pragma unroll
            for (int m = 0; m < 6; ++m) sl[SO_DV + m] = du[m] - (m == 5 ? prm.grav * prm.dt : 0.0);
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
// ---------------------------------------------------------------------------
template <int LS>
__global__ void __launch_bounds__(64) lmpc_qp_kernel(const DevParams prm, const double* __restrict__ rec,
                                                     const uint8_t* __restrict__ contact, int batch,
                                                     double* __restrict__ grf, int32_t* __restrict__ status,
                                                     int32_t* __restrict__ iters, double* __restrict__ scratch) {
    extern __shared__ __attribute__((aligned(16))) double lmpc_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    const int RL = 33 + 12 * H;
    const Smem S = carve(lmpc_smem, H);
    double* gs = scratch + (size_t)qp * GS * H;
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;
    STAMP_DECL

    // ---- load the record (coalesced, one pass) ----
    const double* rin = rec + (size_t)qp * RL;
    for (int i = lane; i < RL; i += 64) {
        const double v = rin[i];
        if (i < 33) S.hdr[i] = v;
        else S.xr[i - 33] = v;
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
        S.G0[e] = v;
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
        f[t][2] = st[t] ? 0.5 * fzmax : 0.0;
        double o[5];
        cons_resid(f[t], mu, fzmax, o);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            s[t][i] = st[t] ? -o[i] : 1.0;
            z[t][i] = 1.0;
        }
        u[t][0] = u[t][1] = u[t][2] = 0.0;
    }
    const double nst = wave_sum((double)nst_loc);
    STAMP(0);  // prologue
    int qstatus = LMPC_QP_CONVERGED;
    int ipm_it = 0, prounds = 0;
    bool done = false;
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
        double dsa[LS][5], dza[LS][5];
        double mu_c = 0.0, smu = 0.0;
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
                    // active set from the interior point: z > s, lift-off legs -> apex
#pragma unroll
                    for (int t = 0; t < LS; ++t) {
                        act[t] = 0;
                        if (!st[t]) continue;
#pragma unroll
                        for (int i = 0; i < 5; ++i)
                            if (z[t][i] > s[t][i]) act[t] |= 1 << i;
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
                                W[i] = z[t][i] / s[t][i];
                                wv[i] = W[i] * (s[t][i] - (i == 4 ? fzmax : 0.0));
                            }
                        }
                        const double sx = W[0] + W[1], sy = W[2] + W[3];
                        const int j = lsj[t];
                        Rt[t][0] = prm.r[3 * j + 0] + sx;
                        Rt[t][1] = 0.0;
                        Rt[t][2] = mu * (W[0] - W[1]);
                        Rt[t][3] = prm.r[3 * j + 1] + sy;
                        Rt[t][4] = mu * (W[2] - W[3]);
                        Rt[t][5] = prm.r[3 * j + 2] + mu * mu * (sx + sy) + W[4];
                        cons_tw(wv, mu, rt[t]);
#pragma unroll
                        for (int i = 0; i < 9; ++i) T[t][i] = (st[t] && (i % 4 == 0)) ? 1.0 : 0.0;
                        up[t][0] = up[t][1] = up[t][2] = 0.0;
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
                    Rt[t][0] = prm.r[3 * j];
                    Rt[t][1] = Rt[t][2] = 0.0;
                    Rt[t][3] = prm.r[3 * j + 1];
                    Rt[t][4] = 0.0;
                    Rt[t][5] = prm.r[3 * j + 2];
                    rt[t][0] = rt[t][1] = rt[t][2] = 0.0;
                }
            }
            if (mode != CORR) leg_stage_prep<LS>(prm, S, valid, lsk, lsj, Rt, T, up);
            leg_rhs<LS>(S, valid, lsk, lsj, Rt, rt, T, up);
            LMPC_SYNC();
            STAMP(1);  // leg-step work (IPM/polish bookkeeping, stage prep)
            if (mode != CORR) riccati_factor(prm, S, gs, lane);
            STAMP(2);  // factorisation
            riccati_solve(prm, S, gs, lane);
            STAMP(3);  // vector pass
            leg_u<LS>(S, valid, lsk, lsj, T, up, u);
            if (mode == PRED) {
                double amax = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) dsa[t][i] = dza[t][i] = 0.0;
                    if (!st[t]) continue;
                    double o[5];
                    cons_resid(u[t], mu, fzmax, o);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        dsa[t][i] = -o[i] - s[t][i];
                        dza[t][i] = -z[t][i] - (z[t][i] / s[t][i]) * dsa[t][i];
                        if (dsa[t][i] < 0.0) amax = fmin(amax, -s[t][i] / dsa[t][i]);
                        if (dza[t][i] < 0.0) amax = fmin(amax, -z[t][i] / dza[t][i]);
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
                        wv[i] = (z[t][i] / s[t][i]) * (s[t][i] - (i == 4 ? fzmax : 0.0)) +
                                (smu - dsa[t][i] * dza[t][i]) / s[t][i];
                    cons_tw(wv, mu, rt[t]);
                }
                mode = CORR;
            } else if (mode == CORR) {
                double ds[LS][5], dz[LS][5];
                double amax = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) ds[t][i] = dz[t][i] = 0.0;
                    if (!st[t]) continue;
                    double o[5];
                    cons_resid(u[t], mu, fzmax, o);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        ds[t][i] = -o[i] - s[t][i];
                        dz[t][i] = (smu - z[t][i] * s[t][i] - dsa[t][i] * dza[t][i] - z[t][i] * ds[t][i]) / s[t][i];
                        if (ds[t][i] < 0.0) amax = fmin(amax, -s[t][i] / ds[t][i]);
                        if (dz[t][i] < 0.0) amax = fmin(amax, -z[t][i] / dz[t][i]);
                    }
                }
                const double alpha = fmin(1.0, 0.99 * wave_min(amax));
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
#pragma unroll
                    for (int m = 0; m < 3; ++m) f[t][m] += alpha * (u[t][m] - f[t][m]);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        s[t][i] += alpha * ds[t][i];
                        z[t][i] += alpha * dz[t][i];
                    }
                }
                ++ipm_it;
                mode = PRED;
            } else {
                // ---- polish verification: primal feasibility + multiplier signs ----
                STAMP(1);
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
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        double v = prm.r[3 * j + p] * u[t][p];
#pragma unroll
                        for (int m = 0; m < 6; ++m) v += S.G0[m * 12 + 3 * j + p] * lam[6 + m];
                        g[t][p] = v;
                        gloc = fmax(gloc, fabs(v));
                    }
                }
                const double gscale = wave_max(gloc);
                int changed = 0;
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
                    if (apex[t]) {
                        if (g[t][2] / mu < fabs(g[t][0]) + fabs(g[t][1]) - prm.tol_d * gscale) {
                            act[t] = (g[t][0] < 0.0 ? 2 : 1) | (g[t][1] < 0.0 ? 8 : 4);
                            changed = 1;
                        }
                        continue;
                    }
                    if (act[t] == 0) continue;
                    // multipliers: C_S' z = -g, C_S full row rank (<= 3 rows)
                    int idx[3], nr = 0;
                    for (int i = 0; i < 5 && nr < 3; ++i)
                        if ((act[t] >> i) & 1) idx[nr++] = i;
                    double Cs[3][3], Gm[3][3], rhs[3];
                    for (int a = 0; a < nr; ++a) {
                        cons_rowvec(idx[a], mu, Cs[a]);
                        rhs[a] = -(Cs[a][0] * g[t][0] + Cs[a][1] * g[t][1] + Cs[a][2] * g[t][2]);
                    }
                    for (int a = 0; a < nr; ++a)
                        for (int b2 = 0; b2 < nr; ++b2)
                            Gm[a][b2] = Cs[a][0] * Cs[b2][0] + Cs[a][1] * Cs[b2][1] + Cs[a][2] * Cs[b2][2];
                    for (int a = 0; a < nr; ++a) {
                        for (int b2 = a + 1; b2 < nr; ++b2) {
                            const double fct = Gm[b2][a] / Gm[a][a];
                            for (int c2 = a; c2 < nr; ++c2) Gm[b2][c2] -= fct * Gm[a][c2];
                            rhs[b2] -= fct * rhs[a];
                        }
                    }
                    double zz[3];
                    for (int a = nr - 1; a >= 0; --a) {
                        double v = rhs[a];
                        for (int b2 = a + 1; b2 < nr; ++b2) v -= Gm[a][b2] * zz[b2];
                        zz[a] = v / Gm[a][a];
                    }
                    int amin = -1;
                    double zmin = -prm.tol_d * gscale;
                    for (int a = 0; a < nr; ++a)
                        if (zz[a] < zmin) {
                            zmin = zz[a];
                            amin = a;
                        }
                    if (amin >= 0) {
                        act[t] &= ~(1 << idx[amin]);
                        changed = 1;
                    }
                }
                if (!__any(changed)) {
                    done = true;
                    break;
                }
                if (++rd >= prm.max_rounds) {
                    // retry: tighter interior point, then a fresh polish
                    if (++att >= prm.max_attempts) break;
                    tol *= 1e-3;
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
#pragma unroll
        for (int p = 0; p < 3; ++p) gout[3 * ls + p] = (anybad || !st[t]) ? 0.0 : u[t][p];
    }
    STAMP(5);  // epilogue
    STAMP_FLUSH(qp);
    if (lane == 0) {
        if (status) status[qp] = anybad ? LMPC_QP_NAN : qstatus;
        if (iters) iters[qp] = ipm_it | (prounds << 16);
    }
}

template __global__ void lmpc_qp_kernel<1>(const DevParams, const double*, const uint8_t*, int, double*, int32_t*,
                                           int32_t*, double*);
template __global__ void lmpc_qp_kernel<2>(const DevParams, const double*, const uint8_t*, int, double*, int32_t*,
                                           int32_t*, double*);

// Host-side launcher (called from lmpc_capi.cpp).
hipError_t launch_qp(const DevParams& prm, const double* rec, const uint8_t* contact, int batch, double* grf,
                     int32_t* status, int32_t* iters, double* scratch, hipStream_t stream) {
    const size_t lds = lds_bytes(prm.H);
    const dim3 grid(batch), block(64);
    if (4 * prm.H <= 64) {
        (void)hipFuncSetAttribute((const void*)lmpc_qp_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lmpc_qp_kernel<1>, grid, block, lds, stream, prm, rec, contact, batch, grf, status, iters,
                           scratch);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_qp_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lmpc_qp_kernel<2>, grid, block, lds, stream, prm, rec, contact, batch, grf, status, iters,
                           scratch);
    }
    return hipGetLastError();
}

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_stamps(unsigned long long* out, int nqp) {
    if (nqp > STAMP_QPS) nqp = STAMP_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_stamps), (size_t)nqp * 8 * sizeof(unsigned long long)) == hipSuccess ? nqp : -1;
}
#endif

}  // namespace lmpc

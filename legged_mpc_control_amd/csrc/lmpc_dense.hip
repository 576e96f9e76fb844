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
//   diagonal tile   16x16 block Cholesky by leg blocks (3x3 pivots, VALU, one column per lane,
//                   [M_bb | I] -> U_bb^-1) -- the only serial part;
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

namespace lmpc {

constexpr int DN_TILE = 256;  // doubles per 16x16 tile

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of QP 0..4095 (tools/dense_check.py).
#ifdef LMPC_STAMPS
__device__ unsigned long long lmpc_dense_stamps[4096][8];
#define DSTAMP_DECL unsigned long long _ds_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _ds_t0 = __builtin_readcyclecounter();
#define DSTAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _ds_acc[i] += _t - _ds_t0; _ds_t0 = _t; } while (0)
#define DSTAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < 4096) for (int _i = 0; _i < 8; ++_i) lmpc_dense_stamps[qp][_i] = _ds_acc[_i]; } while (0)
#define DS_PARAMS , unsigned long long (&_ds_acc)[8], unsigned long long& _ds_t0
#define DS_ARGS , _ds_acc, _ds_t0
#else
#define DS_PARAMS
#define DS_ARGS
#define DSTAMP_DECL
#define DSTAMP(i) do {} while (0)
#define DSTAMP_FLUSH(qp) do {} while (0)
#endif

// packed index of the upper tile (r, c), r <= c < 4
__device__ __forceinline__ constexpr int tix(int r, int c) { return r * 4 - r * (r - 1) / 2 + (c - r); }
// index of the off-diagonal tile (a, b), a < b < 4
__device__ __forceinline__ constexpr int uix(int a, int b) { return a == 0 ? b - 1 : a == 1 ? b + 1 : 5; }
// element (r, c) of a tile in accumulator order (lane (r&3)*16 + c, register r>>2)
__device__ __forceinline__ int toff(int r, int c) { return (r >> 2) * 64 + (r & 3) * 16 + c; }
// variable of leg-step b, component a
__device__ __forceinline__ int vidx(int b, int a) { return 16 * (b / 5) + 3 * (b % 5) + a; }
// packed symmetric 3x3 [xx xy xz yy yz zz]
__device__ __forceinline__ int sym3(int p, int q) {
    const int lo = p < q ? p : q, hi = p < q ? q : p;
    return lo == 0 ? hi : lo == 1 ? 2 + hi : 5;
}

// acc += X' Y on 16x16 tiles (4 MFMAs); sub: acc -= X' Y
__device__ __forceinline__ d4 tprod(const d4& X, const d4& Y, d4 acc) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc = MFMA64(X[kk], Y[kk], acc);
    return acc;
}
__device__ __forceinline__ d4 tprod_sub(const d4& X, const d4& Y, d4 acc) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc = MFMA64(-X[kk], Y[kk], acc);
    return acc;
}

typedef __attribute__((address_space(3))) int lint;

// sum over the 16 lanes of each DPP row (every lane gets its row's total)
__device__ __forceinline__ double row_sum(double v) {
    v += dpp_f64<DPP_QP_1032>(v);
    v += dpp_f64<DPP_QP_2301>(v);
    v += dpp_f64<DPP_ROR4>(v);
    v += dpp_f64<DPP_ROR8>(v);
    return v;
}

struct DSmem {
    ldouble* hdr;   // 40: x0(12) R(9) feet(12)
    ldouble* G0;    // 72: B rows 6-11 (terrain: G0 blkdiag(R_j))
    ldouble* rb;    // 24: per-leg input Hessian block, packed symmetric
    ldouble* tf;    // 36: terrain frames R_j (row-major)
    ldouble* cs;    // 2H
    ldouble* xr;    // 12H
    ldouble* em;    // 12H: Q (c_{m+1} - xref_m)
    ldouble* Ht;    // 10 tiles: upper tiles of H
    ldouble* gv;    // 64: condensed gradient
    ldouble* vec;   // 64: right-hand side in / solution out
    ldouble* vec2;  // 64: matvec operand / result
    ldouble* blk;   // 180: per-leg-step 3x3 block (D in the IPM, T in the polish)
    ldouble* act;   // 20: 1 = leg-step coupled (T != 0)
    ldouble* lup;   // 60: polish particular solution up per leg-step (kept out of registers)
    ldouble* lua;   // 60: predictor step u_aff per leg-step
    ldouble* scr;   // union: P~ columns 6-11 (72H) during condensation | el(272) PNL(96) L^-1(272)
    lint* lsm;      // 20: stance leg-step b -> 4k + j
    lint* fb;       // H+1: first stance leg-step of step k
};
constexpr int DN_EL = 16 * 17;                // staging of one 16x16 tile, column stride 17
constexpr int DN_SCR_MIN = DN_EL + 96 + DN_EL;  // el | PNL | L^-1

__device__ __forceinline__ DSmem dcarve(double* sm, int H) {
    DSmem s;
    ldouble* p = (ldouble*)sm;
    s.hdr = p; p += 40;
    s.G0 = p; p += 72;
    s.rb = p; p += 24;
    s.tf = p; p += 36;
    s.Ht = p; p += 10 * DN_TILE;
    s.gv = p; p += 64;
    s.vec = p; p += 64;
    s.vec2 = p; p += 64;
    s.blk = p; p += 180;
    s.act = p; p += 20;
    s.lup = p; p += 60;
    s.lua = p; p += 60;
    s.cs = p; p += 2 * H;
    s.xr = p; p += 12 * H;
    s.em = p; p += 12 * H;
    s.scr = p; p += (72 * H > DN_SCR_MIN ? 72 * H : DN_SCR_MIN);
    lint* ip = (lint*)p;
    s.lsm = ip;
    s.fb = ip + 20;
    return s;
}

// ---------------------------------------------------------------------------
// Condensation: em, g, P~, H (see the header comment).  All lanes; lane v = variable v.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dense_condense(const DevParams& prm, const DSmem& S, int H, int nls, int lane) {
    const double dt = prm.dt;
    // ---- free response and adjoint (every lane redundantly: no exchange needed) ----
    {
        double x[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) x[r] = S.hdr[r];
        for (int m = 0; m < H; ++m) {
            const double ck = S.cs[2 * m], sk = S.cs[2 * m + 1];
            const double x6 = x[6], x7 = x[7], x8 = x[8];
            x[0] += dt * (ck * x6 + sk * x7);
            x[1] += dt * (-sk * x6 + ck * x7);
            x[2] += dt * x8;
            x[3] += dt * x[9];
            x[4] += dt * x[10];
            x[5] += dt * x[11];
            x[11] -= prm.grav * dt;
            if (lane < 12) {
                double xl = x[0];
#pragma unroll
                for (int r = 1; r < 12; ++r) xl = (lane == r) ? x[r] : xl;
                S.em[12 * m + lane] = prm.q[lane] * (xl - S.xr[12 * m + lane]);
            }
        }
    }
    // variable of this lane
    const int vt = lane >> 4, vw = lane & 15;
    const int vb = 5 * vt + vw / 3, va = vw % 3;
    const bool vvalid = vw < 15 && vb < nls;
    LMPC_SYNC();
    int vk = 0, vj = 0;
    if (vvalid) {
        const int id = S.lsm[vb];
        vk = id >> 2;
        vj = id & 3;
    }
    const int vc = 3 * vj + va;
    {
        double mu[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) mu[r] = 0.0;
        double gval = 0.0;
        for (int m = H; m >= 1; --m) {
            if (m < H) {  // mu <- A_m' mu
                const double ck = S.cs[2 * m], sk = S.cs[2 * m + 1];
                const double m0 = mu[0], m1 = mu[1], m2 = mu[2];
                mu[6] += dt * (ck * m0 - sk * m1);
                mu[7] += dt * (sk * m0 + ck * m1);
                mu[8] += dt * m2;
                mu[9] += dt * mu[3];
                mu[10] += dt * mu[4];
                mu[11] += dt * mu[5];
            }
#pragma unroll
            for (int r = 0; r < 12; ++r) mu[r] += S.em[12 * (m - 1) + r];
            if (vvalid && vk + 1 == m) {
                double gs = 0.0;
#pragma unroll
                for (int q = 0; q < 6; ++q) gs += S.G0[q * 12 + vc] * mu[6 + q];
                gval = gs;
            }
        }
        S.gv[lane] = gval;
    }
    // ---- P~ recursion on the matrix cores; store P~_m[:, 6:12] for m = 1..H ----
    {
        const int lc = lane & 15, lr = lane >> 4;
        d4 P;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = lr + 4 * i;
            P[i] = (r == lc && r < 12) ? prm.q[r < 12 ? r : 0] : 0.0;
        }
        const d4 Qd = P;
        double nc[2], ns[2], n1[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int r = 4 * kk + lr, c = lc;
            nc[kk] = ns[kk] = n1[kk] = 0.0;
            if (r < 3 && c >= 6 && c < 9) {
                const int j = c - 6;
                if (r == 0) { nc[kk] = (j == 0) ? dt : 0.0; ns[kk] = (j == 1) ? dt : 0.0; }
                if (r == 1) { ns[kk] = (j == 0) ? -dt : 0.0; nc[kk] = (j == 1) ? dt : 0.0; }
                if (r == 2) n1[kk] = (j == 2) ? dt : 0.0;
            }
            if (r >= 3 && r < 6 && c == r + 6) n1[kk] = dt;
        }
        for (int m = H; m >= 1; --m) {
            if (m < H) {
                const double ck = S.cs[2 * m], sk = S.cs[2 * m + 1];
                double nh[2];
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) nh[kk] = fma(nc[kk], ck, fma(ns[kk], sk, n1[kk]));
                d4 PA = P;
                PA = MFMA64(P[0], nh[0], PA);
                PA = MFMA64(P[1], nh[1], PA);
                d4 Pn = Qd + PA;
                Pn = MFMA64(nh[0], PA[0], Pn);
                Pn = MFMA64(nh[1], PA[1], Pn);
                P = Pn;
            }
            if (lc >= 6 && lc < 12) {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int r = lr + 4 * i;
                    S.scr[72 * (m - 1) + 6 * r + (lc - 6)] = P[i];
                }
            }
        }
    }
    // ---- H: zero tiles, identity on padding / unused slots, then one column per lane ----
#pragma unroll 4
    for (int e = lane; e < 10 * DN_TILE; e += 64) S.Ht[e] = 0.0;
    LMPC_SYNC();
    {
        // identity on the diagonal of padding and unused variables (lane v = variable v)
        if (!vvalid) S.Ht[tix(vt, vt) * DN_TILE + toff(vw, vw)] = 1.0;
    }
    if (vvalid) {
        double L[12];
        const ldouble* Pt = S.scr + 72 * vk;  // P~_{k+1}
        double gc[6];
#pragma unroll
        for (int q = 0; q < 6; ++q) gc[q] = S.G0[q * 12 + vc];
#pragma unroll
        for (int r = 0; r < 12; ++r) {
            double acc = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q) acc = fma(Pt[6 * r + q], gc[q], acc);
            L[r] = acc;
        }
        const int v = lane;
        for (int i = vk; i >= 0; --i) {
            if (i < vk) {  // L <- A_{i+1}' L
                const double ck = S.cs[2 * (i + 1)], sk = S.cs[2 * (i + 1) + 1];
                const double l0 = L[0], l1 = L[1], l2 = L[2];
                L[6] += dt * (ck * l0 - sk * l1);
                L[7] += dt * (sk * l0 + ck * l1);
                L[8] += dt * l2;
                L[9] += dt * L[3];
                L[10] += dt * L[4];
                L[11] += dt * L[5];
            }
            const int b0 = S.fb[i], b1 = S.fb[i + 1];
            for (int bp = b0; bp < b1; ++bp) {
                const int jp = S.lsm[bp] & 3;
#pragma unroll
                for (int ap = 0; ap < 3; ++ap) {
                    const int cp = 3 * jp + ap;
                    double val = 0.0;
#pragma unroll
                    for (int q = 0; q < 6; ++q) val = fma(S.G0[q * 12 + cp], L[6 + q], val);
                    if (bp == vb) val += S.rb[6 * vj + sym3(ap, va)];
                    const int vp = vidx(bp, ap);
                    const int tp = vp >> 4;
                    if (tp <= vt) S.Ht[tix(tp, vt) * DN_TILE + toff(vp & 15, vw)] = val;
                    if (tp == vt && i < vk) S.Ht[tix(vt, vt) * DN_TILE + toff(vw, vp & 15)] = val;
                }
            }
        }
    }
    LMPC_SYNC();
}

// ---------------------------------------------------------------------------
// Diagonal tile: U_bb^-1 (Ui, = L^-T) and its transpose (UiT, = L^-1) of M_bb = L L'.
// Block Cholesky by leg blocks (3x3 pivots) on [M_bb | I], one column per lane (lanes 0-31),
// decoupled identity blocks (unused / padding / apex legs) skipped.  amask: coupled blocks (bits 0-4).
// ---------------------------------------------------------------------------
struct DiagInv {
    d4 ui, uit;
};
// Outlined (one call site): the elimination gets the caller-saved registers to itself instead of
// competing with the factor tiles and the leg state that are live around it.
__device__ __attribute__((noinline)) DiagInv diag_inverse(ldouble* scr, d4 M, int amask, int lane) {
    // column-major staging with an odd column stride (17 doubles): a wave's 16 columns fall on
    // distinct LDS banks (a stride of 16 puts them on two banks: 8-way conflicts)
    ldouble* el = scr;
    ldouble* PNL = scr + DN_EL;
    ldouble* li = scr + DN_EL + 96;
    const int lc = lane & 15, lr = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) el[lc * 17 + lr + 4 * i] = M[i];
    LMPC_SYNC();
    double a[16];
    {
        const ldouble* src = el + 17 * (lane < 16 ? lane : 0);
        const double keep = (lane < 16) ? 1.0 : 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = fma(src[r], keep, (r == lane - 16) ? 1.0 : 0.0);
    }
    if (amask) {
        const int b0 = __builtin_ctz(amask);
        if (lane >= 3 * b0 && lane < 3 * b0 + 3) {
#pragma unroll
            for (int r = 0; r < 16; ++r) PNL[(lane - 3 * b0) * 16 + r] = a[r];
        }
    }
    int par = 0;
#pragma unroll
    for (int blk = 0; blk < 5; ++blk) {
        if (!((amask >> blk) & 1)) continue;
        const int o = 3 * blk;
        const ldouble* pnl = PNL + par * 48;
        LMPC_SYNC();
        const double i00 = rsq_nr(pnl[o]);
        const double l10 = pnl[o + 1] * i00, l20 = pnl[o + 2] * i00;
        const double i11 = rsq_nr(pnl[16 + o + 1] - l10 * l10);
        const double l21 = (pnl[16 + o + 2] - l20 * l10) * i11;
        const double i22 = rsq_nr(pnl[32 + o + 2] - l20 * l20 - l21 * l21);
        const double z0 = i00 * a[o];
        const double z1 = (a[o + 1] - l10 * z0) * i11;
        const double z2 = (a[o + 2] - l20 * z0 - l21 * z1) * i22;
        const int rest = amask >> (blk + 1);
        if (blk < 4 && rest) {
            const double y2 = z2 * i22;
            const double y1 = (z1 - l21 * y2) * i11;
            const double y0 = (z0 - l10 * y1 - l20 * y2) * i00;
            const int nb = blk + 1 + __builtin_ctz(rest);
#pragma unroll
            for (int r = o + 3; r < o + 6; ++r) a[r] -= pnl[r] * y0 + pnl[16 + r] * y1 + pnl[32 + r] * y2;
            const bool pub = lane >= 3 * nb && lane < 3 * nb + 3;
            ldouble* nx = PNL + (par ^ 1) * 48 + (pub ? (lane - 3 * nb) * 16 : 0);
            if (pub && nb == blk + 1) {
#pragma unroll
                for (int r = o + 3; r < o + 6; ++r) nx[r] = a[r];
            }
#pragma unroll
            for (int r = o + 6; r < 15; ++r) a[r] -= pnl[r] * y0 + pnl[16 + r] * y1 + pnl[32 + r] * y2;
            if (pub) {
#pragma unroll
                for (int r = o + 6; r < 15; ++r) nx[r] = a[r];
            }
        }
        a[o] = z0;
        a[o + 1] = z1;
        a[o + 2] = z2;
        par ^= 1;
    }
    // lanes 16+c hold column c of L^-1: stage it (stride 17), then read both tile orientations
    if (lane >= 16 && lane < 32) {
        const int c = lane - 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) li[c * 17 + r] = a[r];
    }
    LMPC_SYNC();
    DiagInv out;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        out.uit[i] = li[lc * 17 + r];  // (r, c) = L^-1[r][c]
        out.ui[i] = li[r * 17 + lc];   // (r, c) = L^-1[c][r]
    }
    return out;
}

// coupled-block mask of tile t (bits 0-4: leg-steps 5t..5t+4 valid, and with use_act also coupled)
__device__ __forceinline__ int tile_mask(const DSmem& S, int t, int nls, bool use_act) {
    int m = 0;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int b = 5 * t + s;
        if (b < nls && (!use_act || S.act[b < 20 ? b : 0] != 0.0)) m |= 1 << s;
    }
    return __builtin_amdgcn_readfirstlane(m);
}

// lane-wise y = H x for the variables (lane v = variable v), H from its upper tiles in LDS.
// Lane v walks the columns starting at its own index, so a wave's reads spread over the banks.
__device__ __forceinline__ double h_matvec(const DSmem& S, const ldouble* x, int NT, int lane) {
    const int tv = lane >> 4, wv = lane & 15;
    const int n = 16 * NT;
    double acc = 0.0;
    if (tv < NT) {
        int w = lane;
        for (int it = 0; it < n; ++it) {
            w = (w + 1 == n) ? 0 : w + 1;
            const int tw = w >> 4, ww = w & 15;
            const int idx = (tv <= tw) ? tix(tv, tw) * DN_TILE + toff(wv, ww) : tix(tw, tv) * DN_TILE + toff(ww, wv);
            acc = fma(S.Ht[idx], x[w], acc);
        }
    }
    return acc;
}

// ---------------------------------------------------------------------------
// The dense-path kernel.  One wave per QP; QPs with more than 20 stance leg-steps are left to the
// Riccati kernel (lmpc_qp_kernel), which skips the ones handled here.
// ---------------------------------------------------------------------------
template <bool TERRAIN>
__global__ void __launch_bounds__(64) lmpc_dense_kernel(const DevParams prm, const double* __restrict__ rec,
                                                        const uint8_t* __restrict__ contact,
                                                        const double* __restrict__ normals, int batch,
                                                        double* __restrict__ grf, int32_t* __restrict__ status,
                                                        int32_t* __restrict__ iters) {
    extern __shared__ __attribute__((aligned(16))) double dn_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    // ---- stance leg-steps: ballot over lane i = 4k + j ----
    const bool stl = lane < 4 * H && contact[(size_t)qp * 4 * H + lane] != 0;
    const unsigned long long smask = __ballot(stl);
    const int nls = __popcll(smask);
    if (nls > DENSE_MAX_LS || nls == 0) return;  // Riccati kernel (it also owns the all-swing QPs)
    const int RL = 33 + 12 * H;
    const DSmem S = dcarve(dn_smem, H);
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;
    DSTAMP_DECL

    // ---- record, leg-step map ----
    const double* rin = rec + (size_t)qp * RL;
    for (int i = lane; i < RL; i += 64) {
        const double v = rin[i];
        if (i < 33) S.hdr[i] = v;
        else S.xr[i - 33] = v;
    }
    const int rank = __builtin_amdgcn_mbcnt_hi((unsigned)(smask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)smask, 0));
    if (stl) S.lsm[rank] = lane;
    if (lane <= H) {
        // first stance leg-step of step `lane` = stance leg-steps with 4k + j < 4 lane
        const unsigned long long below = (lane >= 16) ? smask : (smask & ((1ull << (4 * lane)) - 1ull));
        S.fb[lane] = __popcll(below);
    }
    if (TERRAIN && lane < 4) {
        const double* nin = normals + (size_t)qp * 12 + 3 * lane;
        const double n0 = nin[0], n1 = nin[1], n2 = nin[2];
        const double nn = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
        const double nx = n0 / nn, ny = n1 / nn, c = n2 / nn;
        const double h = 1.0 / (1.0 + c);
        const double R[9] = {1.0 - nx * nx * h, -nx * ny * h, nx, -nx * ny * h, 1.0 - ny * ny * h, ny, -nx, -ny, c};
#pragma unroll
        for (int e = 0; e < 9; ++e) S.tf[9 * lane + e] = R[e];
    }
    LMPC_SYNC();
    double iw[9];
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
    for (int e = lane; e < 72; e += 64) {
        const int r = e / 12, c = e % 12, j = c / 3, cc = c % 3;
        double w[3];
        if (r < 3) {
            const ldouble* ft = S.hdr + LMPC_REC_FEET + 3 * j;
            w[0] = dt * (iw[r * 3 + 1] * ft[2] - iw[r * 3 + 2] * ft[1]);
            w[1] = dt * (-iw[r * 3 + 0] * ft[2] + iw[r * 3 + 2] * ft[0]);
            w[2] = dt * (iw[r * 3 + 0] * ft[1] - iw[r * 3 + 1] * ft[0]);
        } else {
            w[0] = w[1] = w[2] = 0.0;
            w[r - 3] = dt / prm.mass;
        }
        double v = w[cc];
        if constexpr (TERRAIN) {
            const ldouble* Rj = S.tf + 9 * j;
            v = w[0] * Rj[cc] + w[1] * Rj[3 + cc] + w[2] * Rj[6 + cc];
        }
        S.G0[e] = v;
    }
    if (lane < 4) {
        const double r0 = prm.r[3 * lane], r1 = prm.r[3 * lane + 1], r2 = prm.r[3 * lane + 2];
        if constexpr (TERRAIN) {
            const ldouble* R = S.tf + 9 * lane;
            int e = 0;
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = a; b < 3; ++b)
                    S.rb[6 * lane + e++] = r0 * R[a] * R[b] + r1 * R[3 + a] * R[3 + b] + r2 * R[6 + a] * R[6 + b];
        } else {
            S.rb[6 * lane + 0] = r0;
            S.rb[6 * lane + 1] = 0.0;
            S.rb[6 * lane + 2] = 0.0;
            S.rb[6 * lane + 3] = r1;
            S.rb[6 * lane + 4] = 0.0;
            S.rb[6 * lane + 5] = r2;
        }
    }
    S.vec[lane] = 0.0;
    S.vec2[lane] = 0.0;
    LMPC_SYNC();

    DSTAMP(0);  // prologue
    dense_condense(prm, S, H, nls, lane);
    // Always four tiles: leg-steps beyond nls are identity padding (exact, and it keeps every tile
    // index static, so register liveness is exact across the predictor / corrector solves).
    constexpr int NT = 4;
    DSTAMP(1);  // condensation

    // ---- leg-step state: lane b = stance leg-step b ----
    const bool st = lane < nls;
    int lk = 0, lj = 0;
    if (st) {
        const int id = S.lsm[lane];
        lk = id >> 2;
        lj = id & 3;
    }
    double f[3], s[5], z[5];
    {
        const double cnt = st ? (double)(S.fb[lk + 1] - S.fb[lk]) : 1.0;
        f[0] = f[1] = 0.0;
        f[2] = st ? fmin(0.5 * fzmax, prm.mass * prm.grav / cnt) : 0.0;
        double o[5];
        cons_resid(f, mu, fzmax, o);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            s[i] = st ? -o[i] : 1.0;
            z[i] = 1.0 / s[i];
        }
    }
    double u[3] = {0.0, 0.0, 0.0}, rt[3] = {0.0, 0.0, 0.0};
    int qstatus = LMPC_QP_CONVERGED, ipm_it = 0, prounds = 0;
    bool done = false;
    enum { PRED = 0, CORR = 1, POLISH = 2 };
    const double mc = 5.0 * nls;
    double tol = prm.tol_mu;
    int att = 0, rd = 0, it_end = prm.max_iter, mode = PRED, act = 0;
    bool apex = false;
    double mu_c = 0.0, smu = 0.0;
    // factor tiles (register resident through the corrector): U's off-diagonal tiles in Tl, U_bb^-1, U_bb^-T
    d4 Tl[10], Ui[4], UiT[4];
    const int lc = lane & 15, lr = lane >> 4;
    for (;;) {
        if (mode == PRED) {
            double loc = 0.0;
            if (st) {
#pragma unroll
                for (int i = 0; i < 5; ++i) loc += s[i] * z[i];
            }
            mu_c = wave_sum(loc) / mc;
            if (mu_c < tol || ipm_it >= it_end) {
                act = 0;
                if (st) {
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        if (z[i] > s[i]) act |= 1 << i;
                    const double fm = fmax(fabs(f[0]), fmax(fabs(f[1]), fabs(f[2])));
                    if (fm < 1e-6 * fzmax) act = 15;
                }
                mode = POLISH;
                rd = 0;
            } else {
                double W[5] = {0, 0, 0, 0, 0}, wv[5] = {0, 0, 0, 0, 0};
                if (st) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        W[i] = z[i] * rcp_nr(s[i]);
                        wv[i] = W[i] * (s[i] - (i == 4 ? fzmax : 0.0));
                    }
                }
                const double sx = W[0] + W[1], sy = W[2] + W[3];
                if (st) {  // D = C'WC (R is inside H)
                    ldouble* bk = S.blk + 9 * lane;
                    const double dxz = mu * (W[0] - W[1]), dyz = mu * (W[2] - W[3]), dzz = mu * mu * (sx + sy) + W[4];
                    bk[0] = sx;  bk[1] = 0.0; bk[2] = dxz;
                    bk[3] = 0.0; bk[4] = sy;  bk[5] = dyz;
                    bk[6] = dxz; bk[7] = dyz; bk[8] = dzz;
                }
                cons_tw(wv, mu, rt);
            }
        }
        if (mode == POLISH) {
            ++prounds;
            apex = false;
            double T[9], up[3];
            if (st) apex = leg_basis(act, mu, fzmax, T, up);
            S.vec2[lane] = 0.0;  // padding / unused variables of the up vector
            LMPC_SYNC();
            if (st) {
#pragma unroll
                for (int p = 0; p < 3; ++p) S.lup[3 * lane + p] = up[p];
                ldouble* bk = S.blk + 9 * lane;
#pragma unroll
                for (int e = 0; e < 9; ++e) bk[e] = T[e];
                bool coupled = false;
#pragma unroll
                for (int e = 0; e < 9; ++e) coupled |= T[e] != 0.0;
                S.act[lane] = coupled ? 1.0 : 0.0;
#pragma unroll
                for (int p = 0; p < 3; ++p) S.vec2[vidx(lane, p)] = up[p];
            }
        }
        // ---- right-hand side (and, except in the corrector, the Newton matrix) ----
        if (mode != POLISH) {
            if (st) {
#pragma unroll
                for (int a = 0; a < 3; ++a) S.vec[vidx(lane, a)] = -(S.gv[vidx(lane, a)] + rt[a]);
            }
            LMPC_SYNC();
        } else {
            LMPC_SYNC();
            // rhs = -T'(H up + g)
            const double hv = h_matvec(S, S.vec2, NT, lane) + S.gv[lane];
            LMPC_SYNC();
            S.vec2[lane] = hv;
            LMPC_SYNC();
            if (st) {
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    double v = 0.0;
#pragma unroll
                    for (int p = 0; p < 3; ++p) v += S.blk[9 * lane + p * 3 + a] * S.vec2[vidx(lane, p)];
                    S.vec[vidx(lane, a)] = -v;
                }
            }
            LMPC_SYNC();
        }
        DSTAMP(2);  // leg-step work + right-hand side (+ polish matvec)
        if (mode != CORR) {
            // ---- M tiles ----
            if (mode == PRED) {
#pragma unroll
                for (int t = 0; t < 10; ++t) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Tl[t][i] = S.Ht[t * DN_TILE + i * 64 + lane];
                }
                // + D on the diagonal leg blocks
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = lr + 4 * i;
                        const int bb = 5 * t + r / 3;
                        const bool inb = r < 15 && lc < 15 && (r / 3) == (lc / 3) && bb < nls;
                        const double d = S.blk[inb ? 9 * bb + 3 * (r % 3) + (lc % 3) : 0];
                        Tl[tix(t, t)][i] += inb ? d : 0.0;
                    }
                }
            } else {
                // polish: T^ tiles (block diagonal; identity on unused / padding slots)
                d4 Th[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = lr + 4 * i;
                        const int bb = 5 * t + r / 3;
                        const bool inb = r < 15 && lc < 15 && (r / 3) == (lc / 3) && bb < nls;
                        const double tv = S.blk[inb ? 9 * bb + 3 * (r % 3) + (lc % 3) : 0];
                        Th[t][i] = inb ? tv : (r == lc ? 1.0 : 0.0);
                    }
                }
                // Tl(tr, tc) = T^_tr' H_tr,tc T^_tc  (two X'Y products per tile)
#pragma unroll
                for (int tr = 0; tr < 4; ++tr) {
#pragma unroll
                    for (int tc = tr; tc < 4; ++tc) {
                        if (tc >= NT) continue;
                        d4 Hrc;
#pragma unroll
                        for (int i = 0; i < 4; ++i) Hrc[i] = S.Ht[tix(tr, tc) * DN_TILE + i * 64 + lane];
                        const d4 zero = {0.0, 0.0, 0.0, 0.0};
                        const d4 Yt = tprod(Hrc, Th[tr], zero);  // (T_r' H_rc)'
                        Tl[tix(tr, tc)] = tprod(Yt, Th[tc], zero);
                    }
                }
                // + identity on fixed components (zero T columns) of the diagonal leg blocks
#pragma unroll
                for (int t = 0; t < 4; ++t) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = lr + 4 * i;
                        const int bb = 5 * t + r / 3;
                        const bool dg = r == lc && r < 15 && bb < nls;
                        const ldouble* bk = S.blk + 9 * (dg ? bb : 0);
                        const int a = r % 3;
                        const bool fixed = bk[a] == 0.0 && bk[3 + a] == 0.0 && bk[6 + a] == 0.0;
                        Tl[tix(t, t)][i] += (dg && fixed) ? 1.0 : 0.0;
                    }
                }
            }
            if (mode == POLISH) DSTAMP(7);  // M tiles (polish)
            else DSTAMP(3);                  // M tiles (interior point)
            // ---- tiled Cholesky M = U'U ----
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= NT) continue;
                DSTAMP(4);
                {
                    const DiagInv di = diag_inverse(S.scr, Tl[tix(b, b)], tile_mask(S, b, nls, mode == POLISH), lane);
                    Ui[b] = di.ui;
                    UiT[b] = di.uit;
                }
                DSTAMP(6);  // diagonal tiles
#pragma unroll
                for (int c = b + 1; c < 4; ++c) {
                    if (c >= NT) continue;
                    const d4 zero = {0.0, 0.0, 0.0, 0.0};
                    const d4 Mbc = Tl[tix(b, c)];
                    Tl[tix(b, c)] = tprod(Ui[b], Mbc, zero);  // U_bc = U_bb^-T M_bc
                }
#pragma unroll
                for (int c = b + 1; c < 4; ++c) {
#pragma unroll
                    for (int d = c; d < 4; ++d) {
                        if (d >= NT) continue;
                        Tl[tix(c, d)] = tprod_sub(Tl[tix(b, c)], Tl[tix(b, d)], Tl[tix(c, d)]);
                    }
                }
            }
        }
        DSTAMP(4);  // factorisation
        // ---- solve: U'y = r, U x = y (vectors replicated across the accumulator columns) ----
        {
            d4 y[4], x[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
#pragma unroll
                for (int i = 0; i < 4; ++i) y[b][i] = S.vec[16 * b + lr + 4 * i];
            }
            const d4 zero = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= NT) continue;
                d4 acc = y[b];
#pragma unroll
                for (int a = 0; a < b; ++a) acc = tprod_sub(Tl[tix(a, b)], y[a], acc);
                y[b] = tprod(Ui[b], acc, zero);
            }
            // backward: t = y_b - sum_c U_bc x_c on the VALU (x_c column-replicated: lane l holds
            // x_c[l&15]; one DPP row sum per register), then x_b = U_bb^-1 t on the matrix cores
            double xcol[4];
#pragma unroll
            for (int b = 3; b >= 0; --b) {
                if (b >= NT) continue;
                d4 acc = y[b];
                if (b + 1 < NT) {
                    double part[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int c = b + 1; c < 4; ++c) {
                        if (c >= NT) continue;
#pragma unroll
                        for (int i = 0; i < 4; ++i) part[i] = fma(Tl[tix(b, c)][i], xcol[c], part[i]);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] -= row_sum(part[i]);
                }
                x[b] = tprod(UiT[b], acc, zero);
                if (b > 0) {  // column-replicated copy for the tiles above
                    if (lc == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) S.vec2[16 * b + lr + 4 * i] = x[b][i];
                    }
                    LMPC_SYNC();
                    xcol[b] = S.vec2[16 * b + lc];
                }
            }
            LMPC_SYNC();
            if (lc == 0) {
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    if (b >= NT) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) S.vec[16 * b + lr + 4 * i] = x[b][i];
                }
            }
            LMPC_SYNC();
        }
        DSTAMP(5);  // solve
        // ---- leg-step solution ----
        u[0] = u[1] = u[2] = 0.0;
        if (st) {
            double y3[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) y3[a] = S.vec[vidx(lane, a)];
            if (mode == POLISH) {
                const ldouble* Tb = S.blk + 9 * lane;
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    u[p] = S.lup[3 * lane + p] + Tb[p * 3] * y3[0] + Tb[p * 3 + 1] * y3[1] + Tb[p * 3 + 2] * y3[2];
            } else {
#pragma unroll
                for (int p = 0; p < 3; ++p) u[p] = y3[p];
            }
        }
        if (mode == PRED) {
            double amax = 1.0;
            double dsa[5], dza[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) dsa[i] = dza[i] = 0.0;
            if (st) {
#pragma unroll
                for (int m = 0; m < 3; ++m) S.lua[3 * lane + m] = u[m];
            }
            if (st) {
                double o[5];
                cons_resid(u, mu, fzmax, o);
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    dsa[i] = -o[i] - s[i];
                    dza[i] = -z[i] - z[i] * rcp_nr(s[i]) * dsa[i];
                    if (dsa[i] < 0.0) amax = fmin(amax, -s[i] * __builtin_amdgcn_rcp(dsa[i]));
                    if (dza[i] < 0.0) amax = fmin(amax, -z[i] * __builtin_amdgcn_rcp(dza[i]));
                }
            }
            const double aa = wave_min(amax);
            double loc = 0.0;
            if (st) {
#pragma unroll
                for (int i = 0; i < 5; ++i) loc += (s[i] + aa * dsa[i]) * (z[i] + aa * dza[i]);
            }
            const double ratio = (wave_sum(loc) / mc) / mu_c;
            smu = ratio * ratio * ratio * mu_c;
            if (st) {
                double wv[5];
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    wv[i] = (z[i] * (s[i] - (i == 4 ? fzmax : 0.0)) + smu - dsa[i] * dza[i]) * rcp_nr(s[i]);
                cons_tw(wv, mu, rt);
            }
            mode = CORR;
        } else if (mode == CORR) {
            double ds[5], dz[5];
            double amax = 1.0;
#pragma unroll
            for (int i = 0; i < 5; ++i) ds[i] = dz[i] = 0.0;
            if (st) {
                double o[5], oa[5], ua[3];
#pragma unroll
                for (int m = 0; m < 3; ++m) ua[m] = S.lua[3 * lane + m];
                cons_resid(u, mu, fzmax, o);
                cons_resid(ua, mu, fzmax, oa);
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const double is = rcp_nr(s[i]);
                    const double dsa = -oa[i] - s[i];
                    const double dza = -z[i] - z[i] * is * dsa;
                    ds[i] = -o[i] - s[i];
                    dz[i] = (smu - z[i] * s[i] - dsa * dza - z[i] * ds[i]) * is;
                    if (ds[i] < 0.0) amax = fmin(amax, -s[i] * __builtin_amdgcn_rcp(ds[i]));
                    if (dz[i] < 0.0) amax = fmin(amax, -z[i] * __builtin_amdgcn_rcp(dz[i]));
                }
            }
            const double alpha = fmin(1.0, 0.99 * wave_min(amax));
            if (st) {
#pragma unroll
                for (int m = 0; m < 3; ++m) f[m] += alpha * (u[m] - f[m]);
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    s[i] += alpha * ds[i];
                    z[i] += alpha * dz[i];
                }
            }
            ++ipm_it;
            mode = PRED;
        } else {
            // ---- polish verification: gradient H u + g, primal feasibility, multiplier signs ----
            S.vec2[lane] = 0.0;
            LMPC_SYNC();
            if (st) {
#pragma unroll
                for (int p = 0; p < 3; ++p) S.vec2[vidx(lane, p)] = u[p];
            }
            LMPC_SYNC();
            const double gl = h_matvec(S, S.vec2, NT, lane) + S.gv[lane];
            LMPC_SYNC();
            S.vec2[lane] = gl;
            LMPC_SYNC();
            double g[3] = {0.0, 0.0, 0.0};
            double gloc = 1.0;
            if (st) {
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    g[p] = S.vec2[vidx(lane, p)];
                    gloc = fmax(gloc, fabs(g[p]));
                }
            }
            const double gscale = wave_max(gloc);
            int changed = 0;
            if (st) {
                double o[5];
                cons_resid(u, mu, fzmax, o);
                int imax = -1;
                double vmax = prm.tol_p * fzmax;
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    if (!((act >> i) & 1) && o[i] > vmax) {
                        vmax = o[i];
                        imax = i;
                    }
                if (imax >= 0) {
                    act |= 1 << imax;
                    changed = 1;
                } else if (apex) {
                    if (g[2] / mu < fabs(g[0]) + fabs(g[1]) - prm.tol_d * gscale) {
                        act = (g[0] < 0.0 ? 2 : 1) | (g[1] < 0.0 ? 8 : 4);
                        changed = 1;
                    }
                } else if (act != 0) {
                    int idx[3], nr = 0;
                    for (int i = 0; i < 5 && nr < 3; ++i)
                        if ((act >> i) & 1) idx[nr++] = i;
                    double Cs[3][3], Gm[3][3], rhs[3];
                    for (int a = 0; a < nr; ++a) {
                        cons_rowvec(idx[a], mu, Cs[a]);
                        rhs[a] = -(Cs[a][0] * g[0] + Cs[a][1] * g[1] + Cs[a][2] * g[2]);
                    }
                    for (int a = 0; a < nr; ++a)
                        for (int b2 = 0; b2 < nr; ++b2)
                            Gm[a][b2] = Cs[a][0] * Cs[b2][0] + Cs[a][1] * Cs[b2][1] + Cs[a][2] * Cs[b2][2];
                    for (int a = 0; a < nr; ++a)
                        for (int b2 = a + 1; b2 < nr; ++b2) {
                            const double fct = Gm[b2][a] / Gm[a][a];
                            for (int c2 = a; c2 < nr; ++c2) Gm[b2][c2] -= fct * Gm[a][c2];
                            rhs[b2] -= fct * rhs[a];
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
                        act &= ~(1 << idx[amin]);
                        changed = 1;
                    }
                }
            }
            if (!__any(changed)) {
                done = true;
                break;
            }
            if (++rd >= prm.max_rounds) {
                if (++att >= prm.max_attempts) break;
                tol *= 1e-3;
                it_end += prm.max_iter;
                mode = PRED;
            }
        }
    }
    if (!done) {
        qstatus = LMPC_QP_MAX_ITER;
#pragma unroll
        for (int m = 0; m < 3; ++m) u[m] = f[m];
    }
    // ---- output: stance forces through LDS to the lane of leg-step 4k + j ----
    const int bad = st && (u[0] != u[0] || u[1] != u[1] || u[2] != u[2]);
    const bool anybad = __any(bad);
    LMPC_SYNC();
    if (st) {
        double fo[3] = {u[0], u[1], u[2]};
        if constexpr (TERRAIN) {
            const ldouble* Rj = S.tf + 9 * lj;
#pragma unroll
            for (int p = 0; p < 3; ++p) fo[p] = Rj[3 * p] * u[0] + Rj[3 * p + 1] * u[1] + Rj[3 * p + 2] * u[2];
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) S.vec[3 * lane + p] = fo[p];
    }
    LMPC_SYNC();
    double* gout = grf + (size_t)qp * 12 * H;
    if (lane < 4 * H) {
#pragma unroll
        for (int p = 0; p < 3; ++p) gout[3 * lane + p] = (anybad || !stl) ? 0.0 : S.vec[3 * (stl ? rank : 0) + p];
    }
    if (lane == 0) {
        if (status) status[qp] = anybad ? LMPC_QP_NAN : qstatus;
        if (iters) iters[qp] = ipm_it | (prounds << 16);
    }
    DSTAMP(2);
    DSTAMP_FLUSH(qp);
}

template __global__ void lmpc_dense_kernel<false>(const DevParams, const double*, const uint8_t*, const double*, int,
                                                  double*, int32_t*, int32_t*);
template __global__ void lmpc_dense_kernel<true>(const DevParams, const double*, const uint8_t*, const double*, int,
                                                 double*, int32_t*, int32_t*);

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_dense_stamps(unsigned long long* out, int nqp) {
    if (nqp > 4096) nqp = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_dense_stamps), (size_t)nqp * 8 * sizeof(unsigned long long)) ==
                   hipSuccess ? nqp : -1;
}
#endif

size_t dense_lds_bytes(int H) {
    const int scr = 72 * H > DN_SCR_MIN ? 72 * H : DN_SCR_MIN;
    const int doubles = 40 + 72 + 24 + 36 + 10 * DN_TILE + 64 * 3 + 180 + 20 + 120 + 2 * H + 12 * H + 12 * H + scr;
    return (size_t)doubles * sizeof(double) + (20 + 33) * sizeof(int);
}

hipError_t launch_dense(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                        int batch, double* grf, int32_t* status, int32_t* iters, hipStream_t stream) {
    const size_t lds = dense_lds_bytes(prm.H);
    const dim3 grid(batch), block(LMPC_WAVE);
    if (normals) {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_kernel<true>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_dense_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_dense_kernel<false>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters);
    }
    return hipGetLastError();
}

}  // namespace lmpc

// lmpc_dense_common.h -- the condensed dense path's shared device code (gfx950), used by both
// dense-path kernels: lmpc_dense.hip (interior point + active-set polish on the condensed QP) and
// lmpc_gi.hip (dual active-set / Goldfarb-Idnani on the condensed QP).
//
// Variables of the condensed QP are the stance forces only, laid out 5 leg-steps (15 variables + 1
// padding slot) per 16-wide tile, so every 3x3 leg block sits inside one tile and N <= 64 fits 4x4
// tiles.  The Hessian H is kept in LDS as its upper tiles in the MFMA accumulator layout
// (lane l, register i <-> row (l>>4)+4i, column l&15).  Padding / unused slots carry identity rows.
//
// Prologue (record load, I_w^-1, B = G0, yaw cos/sin, per-leg R blocks; ConvexQPSolver.cpp:198-228)
// and condensation (ConvexQPSolver.cpp:254-313 in condensed form):
//   free response  c_{m+1} = A_m c_m - g dt e11,  c_0 = x0
//   adjoint        mu_m = Q (c_m - xref_{m-1}) + A_m' mu_{m+1}          -> g_i = B' mu_{i+1}
//   cost-to-go     P~_H = Q,  P~_m = Q + A_m' P~_{m+1} A_m              (fp64 MFMA, 12x12)
//   Hessian        H[i][j] = B' (A_j ... A_{i+1})' P~_{j+1} B  (i <= j), + R on the diagonal blocks,
//                  one column per lane: L = P~_{j+1} B e_c, then L <- A_{i+1}' L down the steps.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

namespace lmpc {

constexpr int DN_TILE = 256;  // doubles per 16x16 tile
size_t dense_lds_bytes(int H);  // host: dynamic LDS of the dense-path carve (lmpc_dense.hip)

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

// row_sum of four registers at once (each lane gets all four row totals): a transposing butterfly -- after the
// xor-1 and xor-2 exchanges lane 4q + k holds the quad sum of p[k] only, two rotations finish the row, and a
// quad broadcast per register hands every total back -- 35 instructions instead of four row_sums' 48.
constexpr int DPP_QP_BC0 = 0x00, DPP_QP_BC1 = 0x55, DPP_QP_BC2 = 0xAA, DPP_QP_BC3 = 0xFF;  // quad_perm [k,k,k,k]
__device__ __forceinline__ void row_sum4(const double p[4], double out[4]) {
    const int lane = __lane_id();
    const bool odd = lane & 1, hi2 = lane & 2;
    const double sa = odd ? p[0] : p[1], sb = odd ? p[2] : p[3];
    const double ka = odd ? p[1] : p[0], kb = odd ? p[3] : p[2];
    const double s0 = ka + dpp_f64<DPP_QP_1032>(sa);  // p[lane & 1] over the pair
    const double s1 = kb + dpp_f64<DPP_QP_1032>(sb);  // p[2 + (lane & 1)] over the pair
    const double sc = hi2 ? s0 : s1, kc = hi2 ? s1 : s0;
    double t = kc + dpp_f64<DPP_QP_2301>(sc);          // p[lane & 3] over the quad
    t += dpp_f64<DPP_ROR4>(t);
    t += dpp_f64<DPP_ROR8>(t);                          // ... over the row
    out[0] = dpp_f64<DPP_QP_BC0>(t);
    out[1] = dpp_f64<DPP_QP_BC1>(t);
    out[2] = dpp_f64<DPP_QP_BC2>(t);
    out[3] = dpp_f64<DPP_QP_BC3>(t);
}

// v + v(lane ^ W), W = 16 or 32: v_permlane{16,32}_swap of each dword with a copy of itself returns the lane's own
// and its partner's value in its two outputs (which one is which depends on the half), so their sum needs no select.
// The copy is opaque: with the same value in both operands hipcc (ROCm 7.2) merged the swaps of different
// registers into one (tools/ubench/permlane_probe.hip).
__device__ __forceinline__ unsigned opaque_u32(unsigned v) {
    asm volatile("" : "+v"(v));
    return v;
}
template <int W>
__device__ __forceinline__ double xor_pair_sum(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    unsigned l0, l1, h0, h1;
    if constexpr (W == 32) {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, opaque_u32(lo), false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, opaque_u32(hi), false, false);
        l0 = l[0]; l1 = l[1]; h0 = h[0]; h1 = h[1];
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, opaque_u32(lo), false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, opaque_u32(hi), false, false);
        l0 = l[0]; l1 = l[1]; h0 = h[0]; h1 = h[1];
    }
    const double d0 = __builtin_bit_cast(double, ((unsigned long long)h0 << 32) | l0);
    const double d1 = __builtin_bit_cast(double, ((unsigned long long)h1 << 32) | l1);
    return d0 + d1;
}
// sum over the four row groups (lanes c, 16+c, 32+c, 48+c); bitwise the same in all four (fp addition commutes)
__device__ __forceinline__ double group_sum4(double v) { return xor_pair_sum<16>(xor_pair_sum<32>(v)); }

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
    ldouble* lua;   // 64: predictor step u_aff per leg-step (interior point) | the last factorised polish round's
                    //     solution y0 by variable (polish, range-space rounds: lmpc_dense_kernel.h)
    ldouble* lhg;   // 64: H up + g of the last factorised polish round (range-space rounds' new directions)
    ldouble* scr;   // union: P~ columns 6-11 (72H) during condensation | diag_inverse: T, W staging (256) W' (272) | h_matvec (48)
                    //        | range-space rounds: h_matvec (48), entries (48..120), solves and column vectors (128..512)
    lint* lsm;      // 20: stance leg-step b -> 4k + j
    lint* fb;       // H+1: first stance leg-step of step k
};
constexpr int DN_EL = 16 * 17;               // staging of one 16x16 tile, column stride 17
constexpr int DN_SCR_MIN = 256 + DN_EL;  // diag_inverse: staging of T and W (128 each) | W'

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
    s.lua = p; p += 64;
    s.cs = p; p += 2 * H;
    s.xr = p; p += 12 * H;
    s.em = p; p += 12 * H;
    s.lhg = p; p += 64;
    s.scr = p; p += (72 * H > DN_SCR_MIN ? 72 * H : DN_SCR_MIN);
    lint* ip = (lint*)p;
    s.lsm = ip;
    s.fb = ip + 20;
    return s;
}

// ---------------------------------------------------------------------------
// Condensation: em, g, P~, H (see the header comment).  All lanes; lane v = variable v.
// ---------------------------------------------------------------------------
#ifdef LMPC_STAMPS
// Diagnostic build only: cycles of the condensation's sub-phases per QP (tools/dense_check.py stamps).
__device__ unsigned long long lmpc_condense_stamps[4096][5];
#define CSTAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); \
    if (lane == 0 && blockIdx.x < 4096) lmpc_condense_stamps[blockIdx.x][i] = _t - _cs_t0; _cs_t0 = _t; } while (0)
#define CSTAMP_DECL unsigned long long _cs_t0 = __builtin_readcyclecounter();
#else
#define CSTAMP(i) do {} while (0)
#define CSTAMP_DECL
#endif
// 1: the H-column pass keeps G0's rows 0-2 in registers on flat ground (round 5: H columns 21.3 k -> 17.1 k cycles
// per QP, config 2 -0.7 %, profiles/r05/border/ab_hoist_g0.log); 0: LDS loads in the loop (the compiler cannot hoist
// them past the H stores, which may alias).  Loading the step's yaw terms one iteration ahead here and in the free
// response changed neither phase's cycles and was not kept.
#ifndef LMPC_COND_HOIST_G0
#define LMPC_COND_HOIST_G0 1
#endif
template <bool TERRAIN>
__device__ __forceinline__ void dense_condense(const DevParams& prm, const DSmem& S, int H, int nls,
                                               unsigned long long smask, int lane) {
    const double dt = prm.dt;
    CSTAMP_DECL
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
    CSTAMP(0);  // free response
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
    // this variable's column of B (rows 6-11: G0) and its leg's input-Hessian row, loaded once up front (inside the
    // step loops they were loads under divergent branches, each waiting for its own LDS round trip)
    double gc[6], rbl[3];
#pragma unroll
    for (int q = 0; q < 6; ++q) gc[q] = S.G0[q * 12 + vc];
#pragma unroll
    for (int ap = 0; ap < 3; ++ap) rbl[ap] = S.rb[6 * vj + sym3(ap, va)];
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
                for (int q = 0; q < 6; ++q) gs += gc[q] * mu[6 + q];
                gval = gs;
            }
        }
        S.gv[lane] = gval;
    }
    CSTAMP(1);  // adjoint + gradient
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
    CSTAMP(2);  // P~ recursion
    // ---- H: zero tiles, identity on padding / unused slots, then one column per lane ----
#pragma unroll 4
    for (int e = lane; e < 10 * DN_TILE; e += 64) S.Ht[e] = 0.0;
    LMPC_SYNC();
    {
        // identity on the diagonal of padding and unused variables (lane v = variable v)
        if (!vvalid) S.Ht[tix(vt, vt) * DN_TILE + toff(vw, vw)] = 1.0;
    }
    CSTAMP(3);  // H zero + identity
    {
        // Column v of H (this lane's variable: leg-step vb at step vk, leg vj, component va):
        //   L_i = (A_vk ... A_{i+1})' P~_{vk+1} B e_v for i = vk..0, and H[v'][v] = G0_j'^T L_i[6:12] for the stance
        //   variables v' of step i (+ R on the own 3x3 block).  The step loop is uniform (lanes with vk < i idle):
        //   the stance legs of step i come from the ballot (smask: bit 4k+j) in scalar registers, so no LDS load
        //   (first leg-step of the step, leg of the leg-step) sits ahead of the G0 loads.
        const double dtm = dt / prm.mass;
        double L[12];
        {
            const ldouble* Pt = S.scr + 72 * vk;  // P~_{k+1}
#pragma unroll
            for (int r = 0; r < 12; ++r) {
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < 6; ++q) acc = fma(Pt[6 * r + q], gc[q], acc);
                L[r] = acc;
            }
        }
        const int vkk = vvalid ? vk : -1;  // padding / unused lanes take part in no step
#if LMPC_COND_HOIST_G0
        // flat ground: rows 0-2 of G0 in registers (loop-invariant; in the loop they are LDS loads the compiler cannot
        // hoist past the H stores, which may alias)
        double g0r[3][12];
        if constexpr (!TERRAIN) {
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
                for (int c = 0; c < 12; ++c) g0r[q][c] = S.G0[q * 12 + c];
        }
#endif
        for (int i = H - 1; i >= 0; --i) {
            if (i < vkk) {  // L <- A_{i+1}' L
                const double ck = S.cs[2 * (i + 1)], sk = S.cs[2 * (i + 1) + 1];
                const double l0 = L[0], l1 = L[1], l2 = L[2];
                L[6] += dt * (ck * l0 - sk * l1);
                L[7] += dt * (sk * l0 + ck * l1);
                L[8] += dt * l2;
                L[9] += dt * L[3];
                L[10] += dt * L[4];
                L[11] += dt * L[5];
            }
            const unsigned legs = (unsigned)(smask >> (4 * i)) & 15u;
            int bp = __popcll(smask & ((1ull << (4 * i)) - 1ull));  // first stance leg-step of step i
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
                if (!((legs >> jp) & 1u)) continue;  // uniform
                if (i <= vkk) {
                    const int vb0 = 16 * (bp / 5) + 3 * (bp % 5);  // first variable of leg-step bp
                    const int tp = vb0 >> 4;
#pragma unroll
                    for (int ap = 0; ap < 3; ++ap) {
                        const int cp = 3 * jp + ap;
                        double val = 0.0;
                        if constexpr (TERRAIN) {
#pragma unroll
                            for (int q = 0; q < 6; ++q) val = fma(S.G0[q * 12 + cp], L[6 + q], val);
                        } else {  // flat ground: rows 3-5 of G0 are dt/m I (dense_prologue) -- the same sum, bit for bit
#if LMPC_COND_HOIST_G0
#pragma unroll
                            for (int q = 0; q < 3; ++q) val = fma(g0r[q][cp], L[6 + q], val);
#else
#pragma unroll
                            for (int q = 0; q < 3; ++q) val = fma(S.G0[q * 12 + cp], L[6 + q], val);
#endif
                            val = fma(dtm, L[9 + ap], val);
                        }
                        if (bp == vb) val += rbl[ap];
                        const int vp = vb0 + ap;
                        if (tp <= vt) S.Ht[tix(tp, vt) * DN_TILE + toff(vp & 15, vw)] = val;
                        if (tp == vt && i < vkk) S.Ht[tix(vt, vt) * DN_TILE + toff(vw, vp & 15)] = val;
                    }
                }
                ++bp;
            }
        }
    }
    LMPC_SYNC();
    CSTAMP(4);  // H columns
}

// ---------------------------------------------------------------------------
// Diagonal tile: U_bb^-1 (Ui, = L^-T) and its transpose (UiT, = L^-1) of M_bb = L L'.
// Block Cholesky by leg blocks (3x3 pivots), decoupled identity blocks (unused / padding / apex legs)
// skipped.  amask: coupled blocks (bits 0-4).
//
// The tile T and W = L^-1 (from I) stay in the MFMA accumulator layout (lane 16g + c, register i <->
// element (4i + g, c)).  Per pivot block P = T[o..o+2][o..o+2] (o = 3 blk):
//   the registers holding the three pivot rows of T and W go through LDS once (one write -> read round trip;
//   every lane stores, so the reads have static offsets);
//   every lane factors P = L_p L_p' itself (3 rsq + Newton);
//   lane 16k + m forms L_C[m][k] = (L_p^-1 T[o..o+2][m])_k for the rows m below the pivot (T symmetric)
//   and (L_p^-1 W[o..o+2][c])_k -- the MFMA A and B operands;
//   trailing update T -= L_C L_C' and W -= L_C (L_p^-1 W_p): one v_mfma_f64_16x16x4f64 each (rank 3 of 4);
//   the pivot rows of W become L_p^-1 W_p (Gauss-Jordan on [L | I]: W = L_n^-1 ... L_1^-1 = L^-1).
// Per pivot: 2 MFMAs, one LDS round trip, ~40 VALU -- the row-by-row elimination it replaces (one column
// per lane, three broadcast LDS reads per row and pivot) issued ~5x the LDS reads.
// ---------------------------------------------------------------------------
struct DiagInv {
    d4 ui, uit;
};
// 1: the 3x3 pivot's reciprocals one after another instead of from the leading minors (diagnostic A/B)
#ifndef LMPC_DIAG_SEQ_RSQ
#define LMPC_DIAG_SEQ_RSQ 0
#endif
// Inlined at its call sites (round 3): outlined, the call cost the caller ~1.7 k cycles per tile in argument /
// result moves and in the caller-saved registers it had to park around the call (5.6 k cycles per tile in the
// kernel vs 3.9 k alone, tools/ubench/diag_parts.hip); inlined, config 2 runs 2 % faster (0.2304 -> 0.2259 ms,
// tools/ab_bench.sh, two alternating runs each; bit-identical results).  -DLMPC_DIAG_OUTLINE (diagnostic builds
// only) restores the call.
#ifdef LMPC_DIAG_OUTLINE
#define LMPC_DIAG_ATTR noinline
#else
#define LMPC_DIAG_ATTR always_inline
#endif
static __device__ __attribute__((LMPC_DIAG_ATTR)) DiagInv diag_inverse(ldouble* scr, d4 M, int amask, int lane) {
    amask = __builtin_amdgcn_readfirstlane(amask);  // uniform (tile_mask), but arguments arrive in VGPRs
    // staging of the registers that hold the pivot rows (i0, i1): every lane stores its value unconditionally, so
    // row r of register i sits at 16 (r & 3) + c (+64 for i1) -- static read offsets, no per-lane address select
    ldouble* sT = scr;        // 128: T
    ldouble* sW = scr + 128;  // 128: W
    ldouble* tr = scr + 256;  // 16 x 17: transpose staging of W
    const int c = lane & 15, g = lane >> 4;
    d4 T = M, W;
#pragma unroll
    for (int i = 0; i < 4; ++i) W[i] = (4 * i + g == c) ? 1.0 : 0.0;
#pragma unroll
    for (int blk = 0; blk < 5; ++blk) {
        if (!((amask >> blk) & 1)) continue;
        const int o = 3 * blk;
        // rows o..o+2 live in registers i0 = o>>2 and i1 = (o+2)>>2 (static); this lane's row of register i is 4i+g
        const int i0 = o >> 2, i1 = (o + 2) >> 2;
        const int ra = 4 * i0 + g - o, rb = 4 * i1 + g - o;
        const bool ina = ra >= 0 && ra < 3, inb = i1 != i0 && rb >= 0 && rb < 3;
        // staging offset of pivot row o+a (static)
        auto so = [&](int a) { return ((o + a) >> 2 == i0 ? 0 : 64) + 16 * ((o + a) & 3); };
        LMPC_SYNC();
        // publish the registers of T first: the T chain of this pivot waits only for the previous T update
        sT[lane] = T[i0];
        if (i1 != i0) sT[64 + lane] = T[i1];
        LMPC_SYNC();
        const double p00 = sT[so(0) + o], p10 = sT[so(1) + o], p11 = sT[so(1) + o + 1];
        const double p20 = sT[so(2) + o], p21 = sT[so(2) + o + 1], p22 = sT[so(2) + o + 2];
        const double t0 = sT[so(0) + c], t1 = sT[so(1) + c], t2 = sT[so(2) + c];  // T[o+a][c] = T[c][o+a]
        // then those of W, read while the pivot is factored; W's pivot rows are cleared so the MFMA below writes
        // L_p^-1 W_p into them
        sW[lane] = W[i0];
        if (i1 != i0) sW[64 + lane] = W[i1];
        W[i0] = ina ? 0.0 : W[i0];
        if (i1 != i0) W[i1] = inb ? 0.0 : W[i1];
        LMPC_SYNC();
        const double w0 = sW[so(0) + c], w1 = sW[so(1) + c], w2 = sW[so(2) + c];  // W[o+a][c]
        // P = L_p L_p' with the three pivot reciprocals from the leading minors, so their rsq chains run side by
        // side instead of one after the other: d1 = m11 / p00, d2 = det / m11 (m11 = p00 p11 - p10^2), hence
        // 1/sqrt(d1) = sqrt(p00) rsq(m11) and 1/sqrt(d2) = sqrt(m11) rsq(det)
#if LMPC_DIAG_SEQ_RSQ
        // the pivots one after another (12 fewer fp64 instructions, two more rsq latencies on the chain)
        const double i00 = rsq_nr(p00);
        const double l10 = p10 * i00, l20 = p20 * i00;
        const double i11 = rsq_nr(fma(-l10, l10, p11));
        const double l21 = fma(-l20, l10, p21) * i11;
        const double i22 = rsq_nr(fma(-l21, l21, fma(-l20, l20, p22)));
#else
        const double m11 = fma(p00, p11, -p10 * p10);
        const double c00 = fma(p11, p22, -p21 * p21), c01 = fma(p10, p22, -p21 * p20), c02 = fma(p10, p21, -p11 * p20);
        const double det = fma(p00, c00, fma(-p10, c01, p20 * c02));
        const double i00 = rsq_nr(p00), r1 = rsq_nr(m11), r2 = rsq_nr(det);
        const double l10 = p10 * i00, l20 = p20 * i00;
        const double i11 = (p00 * i00) * r1;
        const double l21 = fma(-l20, l10, p21) * i11;
        const double i22 = (m11 * r1) * r2;
#endif
        // row c of L_C (zero in and above the pivot rows)
        const double x0 = t0 * i00;
        const double x1 = fma(-l10, x0, t1) * i11;
        const double x2 = fma(-l21, x1, fma(-l20, x0, t2)) * i22;
        const double xs = g == 0 ? x0 : g == 1 ? x1 : x2;
        const double av = (c > o + 2 && g < 3) ? xs : 0.0;
        // column c of L_p^-1 W_p
        const double v0 = w0 * i00;
        const double v1 = fma(-l10, v0, w1) * i11;
        const double v2 = fma(-l21, v1, fma(-l20, v0, w2)) * i22;
        const double vs = g == 0 ? v0 : g == 1 ? v1 : v2;
        const double bv = g < 3 ? vs : 0.0;
        // W's A operand: -L_C below the pivot, the unit rows of the pivot block (W_new pivot rows = L_p^-1 W_p)
        const bool cp = c >= o && c <= o + 2;
        const double aw = cp ? (g == c - o ? 1.0 : 0.0) : -av;
        T = MFMA64(-av, av, T);
        W = MFMA64(aw, bv, W);
    }
    // W = L^-1 (lower triangular): uit = W; ui = W' through LDS (column stride 17: distinct banks)
#pragma unroll
    for (int i = 0; i < 4; ++i) tr[c * 17 + 4 * i + g] = W[i];
    LMPC_SYNC();
    DiagInv out;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out.uit[i] = W[i];
        out.ui[i] = tr[(4 * i + g) * 17 + c];
    }
    return out;
}


// coupled-block mask of tile t (bits 0-4: leg-steps 5t..5t+4 valid, and with use_act also coupled)
__device__ __forceinline__ int tile_mask(const DSmem& S, int t, int nls, bool use_act) {
    int m = 0;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int b = 5 * t + s;
        const double a = S.act[b < 20 ? b : 0];  // loaded unconditionally: no branch waits on it
        m |= ((b < nls) & (!use_act | (a != 0.0))) << s;
    }
    return __builtin_amdgcn_readfirstlane(m);
}

// lane-wise y = H x for the variables (lane v = variable v; x in LDS by variable), H from its upper tiles in LDS,
// as VALU tile products in the accumulator layout (lane 16g + c, register i <-> tile element (4i + g, c)):
//   y_t gets T_rt' x_r for r <= t (the stored tile and the diagonal one): lane 16g + c sums T_rt[4i+g][c] x_r[4i+g]
//       over its rows, then over the four row groups -> column-indexed (group_sum4);
//   y_t gets T_tc x_c for c > t: lane 16g + c sums T_tc[4i+g][c] x_c[c] per register, then over its 16-lane row
//       (row_sum) -> row-indexed, handed to lane order through tmp (64 doubles of LDS).
// All loads are independent (one batch); until round 2 every lane walked its row of H with 64 dependent steps.
__device__ __forceinline__ double h_matvec(const DSmem& S, const ldouble* x, ldouble* tmp, int lane) {
    const int lc = lane & 15, lr = lane >> 4;
    double xr[4][4], xc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int i = 0; i < 4; ++i) xr[b][i] = x[16 * b + 4 * i + lr];
        xc[b] = x[16 * b + lc];
    }
    double pc[4] = {0.0, 0.0, 0.0, 0.0};
    double pr[3][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int c = r; c < 4; ++c) {
            const int k = tix(r, c);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const double h = S.Ht[k * DN_TILE + i * 64 + lane];
                pc[c] = fma(h, xr[r][i], pc[c]);
                if (c > r) pr[r][i] = fma(h, xc[c], pr[r][i]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double rs[4];
        row_sum4(pr[r], rs);
        if (lc == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) tmp[16 * r + 4 * i + lr] = rs[i];
        }
    }
    double yc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) yc[c] = group_sum4(pc[c]);
    LMPC_SYNC();
    const double ys = lr == 0 ? yc[0] : lr == 1 ? yc[1] : lr == 2 ? yc[2] : yc[3];
    return ys + (lr < 3 ? tmp[lane < 48 ? lane : 0] : 0.0);
}

// ---------------------------------------------------------------------------
// Prologue: record -> LDS, stance leg-step map (lsm, fb), terrain frames, I_w^-1, G0 = B rows 6-11,
// yaw cos/sin of every step, per-leg input Hessian blocks.  smask = ballot of stance leg-steps
// (lane 4k + j).  Returns this lane's rank among the stance leg-steps (valid when stl).
// ---------------------------------------------------------------------------
template <bool TERRAIN>
__device__ __forceinline__ int dense_prologue(const DevParams& prm, const DSmem& S, const double* __restrict__ rec,
                                              const double* __restrict__ normals, int qp, int H,
                                              unsigned long long smask, bool stl, int lane) {
    const int RL = 33 + 12 * H;
    const double dt = prm.dt;
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

    return rank;
}

}  // namespace lmpc

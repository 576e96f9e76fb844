// lmpc_dense_kernel.h -- the condensed dense path's per-QP solve (dense_body), shared by the dense kernel
// (lmpc_dense.hip) and the fused dense + Riccati kernel (lmpc_lq.hip).  The algorithm is described at the top of
// lmpc_dense.hip.  The diagnostic hooks (DSTAMP*, LMPC_KKT_DIAG) are those of lmpc_dense.hip, which defines them
// before including this header; elsewhere they compile to nothing.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"
#include "lmpc_dense_common.h"

#ifndef DSTAMP
#define DS_PARAMS
#define DS_ARGS
#define DSTAMP_DECL
#define DSTAMP(i) do {} while (0)
#define DSTAMP_FLUSH(qp) do {} while (0)
#endif

// Range-space (Schur complement) polish rounds after a factorised one (dense_body): 1 on, 0 every round refactors;
// LMPC_SCHUR_KMAX added face rows at most per update
#ifndef LMPC_POLISH_SCHUR
#define LMPC_POLISH_SCHUR 1
#endif
#ifndef LMPC_SCHUR_KMAX
#define LMPC_SCHUR_KMAX 6
#endif

namespace lmpc {

// ---------------------------------------------------------------------------
// The dense-path solve of QP blockIdx.x, one wave.  Returns false for a QP it leaves to the Riccati kernel (more
// than 20 stance leg-steps, none, or no verified optimum: done_out[qp] = 0, nothing written), true otherwise.
// lmpc_dense_kernel (lmpc_dense.hip) runs it alone; lmpc_dense_lq_kernel (lmpc_lq.hip) runs the Riccati solve
// after it in the same wave where it returns false (one launch instead of two at one QP per SIMD).
// ---------------------------------------------------------------------------
template <bool TERRAIN>
__device__ __forceinline__ bool dense_body(const DevParams prm, const double* __restrict__ rec,
                                           const uint8_t* __restrict__ contact, const double* __restrict__ normals,
                                           int batch, double* __restrict__ grf, int32_t* __restrict__ status,
                                           int32_t* __restrict__ iters, uint8_t* __restrict__ done_out) {
    extern __shared__ __attribute__((aligned(16))) double dn_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return true;
    const int lane = threadIdx.x;
    const int H = prm.H;
    // ---- stance leg-steps: ballot over lane i = 4k + j ----
    const bool stl = lane < 4 * H && contact[(size_t)qp * 4 * H + lane] != 0;
    const unsigned long long smask = __ballot(stl);
    const int nls = __popcll(smask);
    if (nls > DENSE_MAX_LS || nls == 0) return false;  // Riccati kernel (it also owns the all-swing QPs)
    const DSmem S = dcarve(dn_smem, H);
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;
    DSTAMP_DECL

    const int rank = dense_prologue<TERRAIN>(prm, S, rec, normals, qp, H, smask, stl, lane);
    DSTAMP(0);  // prologue
    dense_condense<TERRAIN>(prm, S, H, nls, smask, lane);
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
    double f[3], s[5], z[5], is[5];  // is = 1/s, refreshed whenever s changes (used 4x per iteration)
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
            is[i] = z[i];
        }
    }
    double u[3] = {0.0, 0.0, 0.0}, rt[3] = {0.0, 0.0, 0.0};
    int qstatus = LMPC_QP_CONVERGED, ipm_it = 0, prounds = 0;
    bool done = false;
    enum { PRED = 0, CORR = 1, POLISH = 2 };
    const double mc = 5.0 * nls, imc = 1.0 / mc;  // complementarity pairs
    double tol = prm.tol_mu;
    // first attempt: at most dense_polish_iter interior-point iterations before the polish (the polish verifies
    // the optimum exactly; a failed polish resumes the interior point with a tighter tolerance below)
    int att = 0, rd = 0, it_end = min(prm.max_iter, prm.dense_polish_iter), mode = PRED, act = 0;
    // polish rounds after a polish round: diagonal tiles before the first leg-step whose active set changed keep their
    // factors (their M tiles, and every panel and update feeding them, are bitwise those of the previous round)
    int keep_tiles = 0;
    bool apex = false;
    // Range-space polish rounds (LMPC_POLISH_SCHUR): a round whose active set only adds faces to the set of the last
    // factorised round (bact, per leg-step lane) is that round's equality QP with k more rows A y = d on its
    // coordinates y, so y = y0 - M^-1 A' (A M^-1 A')^-1 (A y0 - d) from the factorisation in hand: k + 1 solves and
    // a k x k Cholesky instead of T'HT, its tiled Cholesky and one solve (tools/polish_schur_proto.py: 113 of 143
    // later rounds qualify on config 2).  The verification below is the same either way.
    int bact = 0;
    bool have_base = false, schur = false;
    int nsch = 0;
    double mu_c = 0.0, smu = 0.0, sz = 0.0;  // sz = sum of s'z at the iterate (mu_c = sz / mc)
    // factor tiles (register resident through the corrector): U's off-diagonal tiles in Tl, U_bb^-1, U_bb^-T
    d4 Tl[10], Ui[4], UiT[4];
    const int lc = lane & 15, lr = lane >> 4;
    // Diagonal-tile elements inside a 3x3 leg block: lane 16 lr + lc holds rows lr + 4i of column lc, and at most one
    // of them (register lblk_reg, -1 if none) lies in lc's block (rows 3 lblk_q .. 3 lblk_q + 2); lblk_off is its
    // offset in the leg-step's 9-entry block of S.blk
    int lblk_reg = -1, lblk_q = 0, lblk_off = 0, ldg_reg = -1;  // ldg_reg: the register holding element (lc, lc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = lr + 4 * i;
        if (r < 15 && lc < 15 && r / 3 == lc / 3) {
            lblk_reg = i;
            lblk_q = r / 3;
            lblk_off = 3 * (r % 3) + lc % 3;
            if (r == lc) ldg_reg = i;
        }
    }
    for (;;) {
        if (mode == PRED) {
            if (ipm_it >= prm.dense_iter_cap) break;  // test hook: hand the QP to the Riccati kernel
            double loc = 0.0;
            if (st) {
#pragma unroll
                for (int i = 0; i < 5; ++i) loc += s[i] * z[i];
            }
            DSTAMP(2);
            sz = wave_sum(loc);
            mu_c = sz * imc;
            DSTAMP(12);  // complementarity mean (wave reduction)
            if (mu_c < tol || ipm_it >= it_end) {
                act = 0;
                if (st) {
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        if (z[i] > LMPC_ACT_RATIO * s[i]) act |= 1 << i;
                    const double fm = fmax(fabs(f[0]), fmax(fabs(f[1]), fabs(f[2])));
                    if (fm < 1e-6 * fzmax) act = 15;
                }
                mode = POLISH;
                rd = 0;
                keep_tiles = 0;
                have_base = false;
            } else {
                double W[5] = {0, 0, 0, 0, 0}, wv[5] = {0, 0, 0, 0, 0};
                if (st) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        W[i] = z[i] * is[i];
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
            DSTAMP(13);  // Newton-matrix blocks D and weights
        }
        double Tn[9], upn[3];  // this polish round's leg basis (leg_basis of act)
        if (mode == POLISH) {
            ++prounds;
            apex = false;
            double (&T)[9] = Tn;
            if (st) apex = leg_basis(act, mu, fzmax, T, upn);
            schur = false;
#if LMPC_POLISH_SCHUR
            if (have_base) {
                // qualifies where every leg-step keeps its factorised faces and adds at most two, each removing one
                // free direction of the factorised basis (independent of the faces it joins), none at the apex
                const int add = st ? (act & ~bact) : 0;
                const int k = __popc(add);
                bool ok = !st || (act & bact) == bact;  // a dropped face (any leg-step) needs a factorisation
                if (st && add) {
                    const ldouble* Tb = S.blk + 9 * lane;
                    int nb = 0, nn = 0;
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        nb += (Tb[q] != 0.0 || Tb[3 + q] != 0.0 || Tb[6 + q] != 0.0) ? 1 : 0;
                        nn += (T[q] != 0.0 || T[3 + q] != 0.0 || T[6 + q] != 0.0) ? 1 : 0;
                    }
                    ok = ok && !apex && k <= 2 && nn == nb - k;
                }
                const unsigned long long b1 = __ballot(k >= 1), b2 = __ballot(k >= 2);
                nsch = __popcll(b1) + __popcll(b2);
                schur = __all(ok) && nsch >= 1 && nsch <= LMPC_SCHUR_KMAX;
            }
            // a factorised round: tiles ahead of the first leg-step whose faces differ from the last factorised
            // round's keep their factors
            if (!schur) {
                const unsigned long long dif = __ballot(have_base && act != bact);
                keep_tiles = have_base && dif ? (__ffsll((long long)dif) - 1) / 5 : 0;
            }
#endif
        }
        if (mode == POLISH && !schur) {
            S.vec2[lane] = 0.0;  // padding / unused variables of the up vector
            LMPC_SYNC();
            if (st) {
                const double (&T)[9] = Tn;
                const double (&up)[3] = upn;
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
        if (schur) {
        } else if (mode != POLISH) {
            if (st) {
#pragma unroll
                for (int a = 0; a < 3; ++a) S.vec[vidx(lane, a)] = -(S.gv[vidx(lane, a)] + rt[a]);
            }
            LMPC_SYNC();
        } else {
            LMPC_SYNC();
            // rhs = -T'(H up + g)
            const double hv = h_matvec(S, S.vec2, S.scr, lane) + S.gv[lane];
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
        if (mode == POLISH) DSTAMP(11);  // polish set-up + right-hand side (matvec)
        else DSTAMP(2);                  // interior point: leg-step work + right-hand side
        if (mode != CORR && !schur) {
            // ---- M tiles ----
            if (mode == PRED) {
#pragma unroll
                for (int t = 0; t < 10; ++t) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Tl[t][i] = S.Ht[t * DN_TILE + i * 64 + lane];
                }
                // + D on the diagonal leg blocks: one load per tile (lblk_reg below)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int bb = 5 * t + lblk_q;
                    const bool inb = lblk_reg >= 0 && bb < nls;
                    const double d = S.blk[inb ? 9 * bb + lblk_off : 0];
#pragma unroll
                    for (int i = 0; i < 4; ++i) Tl[tix(t, t)][i] += (inb && i == lblk_reg) ? d : 0.0;
                }
            } else {
                // polish: T^ tiles (block diagonal; identity on unused / padding slots)
                d4 Th[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int bb = 5 * t + lblk_q;
                    const bool inb = lblk_reg >= 0 && bb < nls;
                    const double tv = S.blk[inb ? 9 * bb + lblk_off : 0];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        Th[t][i] = (inb && i == lblk_reg) ? tv : (lr + 4 * i == lc ? 1.0 : 0.0);
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
                // + identity on fixed components (zero T columns) of the diagonal leg blocks: the lane's own diagonal
                // element (register ldg_reg, if it holds one) -- one test per tile
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int bb = 5 * t + lblk_q;
                    const bool dg = ldg_reg >= 0 && bb < nls;
                    const ldouble* bk = S.blk + 9 * (dg ? bb : 0);
                    const int a = lc % 3;
                    // all three loads, then bitwise ands (a short-circuit && waited on each load in turn)
                    const double b0 = bk[a], b1 = bk[3 + a], b2 = bk[6 + a];
                    const bool fixed = dg & (b0 == 0.0) & (b1 == 0.0) & (b2 == 0.0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) Tl[tix(t, t)][i] += (fixed && i == ldg_reg) ? 1.0 : 0.0;
                }
            }
            if (mode == POLISH) DSTAMP(7);  // M tiles (polish)
            else DSTAMP(3);                  // M tiles (interior point)
            // ---- tiled Cholesky M = U'U ----
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= NT) continue;
                DSTAMP(4);
                if (b >= keep_tiles) {
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
        // ---- solve: U'y = r, U x = y (vectors replicated across the accumulator columns), S.vec in place ----
        auto solve_vec = [&]() {
            // forward: y_b = U_bb^-T (r_b - sum_{a<b} U_ab' y_a), all on the VALU (a matrix-core product would use
            // 1 of its 16 columns).  The bracket is column-indexed: lane 16g + c sums U_ab[4i+g][c] y_a[4i+g] over
            // its rows, then over the four row groups -> t[c]; y_b = UiT_b (r_b - t) row by row (the four
            // registers' row sums at once, row_sum4) comes out replicated across the columns, the layout the
            // next bracket reads.
            d4 y[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= NT) continue;
                double acc = S.vec[16 * b + lc];
                if (b > 0) {
                    double part = 0.0;
#pragma unroll
                    for (int a = 0; a < b; ++a) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) part = fma(Tl[tix(a, b)][i], y[a][i], part);
                    }
                    acc -= group_sum4(part);
                }
                double pp[4], rs[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) pp[i] = UiT[b][i] * acc;
                row_sum4(pp, rs);
#pragma unroll
                for (int i = 0; i < 4; ++i) y[b][i] = rs[i];
            }
            // backward: t = y_b - sum_c U_bc x_c on the VALU (x_c column-replicated: lane l holds
            // x_c[l&15]; the four registers' row sums at once), then x_b = U_bb^-1 t = UiT_b' t also on the VALU
            // (lane 16g + c sums UiT_b[4i+g][c] t[4i+g], then over the row groups): x_b comes out
            // column-replicated, which is the layout the tiles above read -- no LDS exchange
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
                    double rs[4];
                    row_sum4(part, rs);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] -= rs[i];
                }
                double p = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) p = fma(UiT[b][i], acc[i], p);
                xcol[b] = group_sum4(p);
            }
            if (lr == 0) {
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    if (b >= NT) continue;
                    S.vec[16 * b + lc] = xcol[b];
                }
            }
            LMPC_SYNC();
        };
        if (!schur) {
            solve_vec();
#if LMPC_POLISH_SCHUR
            if (mode == POLISH) {  // this factorised round's solution and faces: the base of range-space rounds
                S.lua[lane] = S.vec[lane];
                bact = act;
                have_base = true;
            }
#endif
        }
#if LMPC_POLISH_SCHUR
        else {
            // ---- range-space round: y = y0 - W lambda, W = M^-1 A', (A W) lambda = A y0 - d ----
            // rows of the added faces on the factorised coordinates (this lane's leg-step: T, up of the base)
            const int add = st ? (act & ~bact) : 0;
            const unsigned long long b1 = __ballot(__popc(add) >= 1), b2 = __ballot(__popc(add) >= 2);
            const unsigned long long below = (1ull << lane) - 1ull;
            const int r0 = __popcll(b1 & below) + __popcll(b2 & below);
            ldouble* rows = S.scr + 64;                  // LMPC_SCHUR_KMAX x [a0 a1 a2 d]
            ldouble* rleg = rows + 4 * LMPC_SCHUR_KMAX;  // leg-step of each row
            ldouble* Wc = S.scr + 96;                    // M^-1 a_j by variable, 64 doubles each
            if (add) {
                const ldouble* Tb = S.blk + 9 * lane;
                const ldouble* ub = S.lup + 3 * lane;
                int r = r0;
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    if (!((add >> i) & 1)) continue;
                    double c[3];
                    cons_rowvec(i, mu, c);
#pragma unroll
                    for (int q = 0; q < 3; ++q) rows[4 * r + q] = fma(c[0], Tb[q], fma(c[1], Tb[3 + q], c[2] * Tb[6 + q]));
                    rows[4 * r + 3] = (i == 4 ? fzmax : 0.0) - fma(c[0], ub[0], fma(c[1], ub[1], c[2] * ub[2]));
                    rleg[r] = (double)lane;
                    ++r;
                }
            }
            LMPC_SYNC();
            for (int j = 0; j < nsch; ++j) {  // wave-uniform
                const int bj = (int)rleg[j];
                S.vec[lane] = 0.0;
                LMPC_SYNC();
                if (lane < 3) S.vec[vidx(bj, lane)] = rows[4 * j + lane];
                LMPC_SYNC();
                solve_vec();
                Wc[64 * j + lane] = S.vec[lane];
            }
            LMPC_SYNC();
            // A W and A y0 - d on every lane, then its Cholesky (rows beyond nsch: identity)
            constexpr int KM = LMPC_SCHUR_KMAX;
            double Am[KM][KM], e[KM];
#pragma unroll
            for (int i = 0; i < KM; ++i) {
                const bool iv = i < nsch;
                const int bi = iv ? (int)rleg[i] : 0;
                double a[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) a[q] = iv ? rows[4 * i + q] : 0.0;
                double ev = iv ? -rows[4 * i + 3] : 0.0;
#pragma unroll
                for (int q = 0; q < 3; ++q) ev = fma(a[q], S.lua[vidx(bi, q)], ev);
                e[i] = ev;
#pragma unroll
                for (int j = 0; j < KM; ++j) {
                    double v = (!iv || j >= nsch) ? (i == j ? 1.0 : 0.0) : 0.0;
                    if (iv && j < nsch) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) v = fma(a[q], Wc[64 * j + vidx(bi, q)], v);
                    }
                    Am[i][j] = v;
                }
            }
            bool bad = false;
#pragma unroll
            for (int c = 0; c < KM; ++c) {
                double d = Am[c][c];
#pragma unroll
                for (int b = 0; b < c; ++b) d = fma(-Am[c][b], Am[c][b], d);
                bad |= !(d > 1e-14 * Am[c][c]);
                const double inv = rsq_nr(d > 0.0 ? d : 1.0);
                Am[c][c] = inv;  // the reciprocal of the pivot
#pragma unroll
                for (int r = c + 1; r < KM; ++r) {
                    double v = Am[r][c];
#pragma unroll
                    for (int b = 0; b < c; ++b) v = fma(-Am[r][b], Am[c][b], v);
                    Am[r][c] = v * inv;
                }
            }
            double lam[KM];
#pragma unroll
            for (int r = 0; r < KM; ++r) {  // L w = e
                double v = e[r];
#pragma unroll
                for (int b = 0; b < r; ++b) v = fma(-Am[r][b], lam[b], v);
                lam[r] = v * Am[r][r];
            }
#pragma unroll
            for (int r = KM - 1; r >= 0; --r) {  // L' lam = w
                double v = lam[r];
#pragma unroll
                for (int b = r + 1; b < KM; ++b) v = fma(-Am[b][r], lam[b], v);
                lam[r] = v * Am[r][r];
            }
            double yv = S.lua[lane];
#pragma unroll
            for (int j = 0; j < KM; ++j)
                if (j < nsch) yv = fma(-Wc[64 * j + lane], lam[j], yv);
            // a rank-deficient update (rounding): keep y0; the round will not verify and the next one refactors
            S.vec[lane] = bad ? S.lua[lane] : yv;
            if (bad) have_base = false;
            LMPC_SYNC();
        }
#endif
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
                    dza[i] = -z[i] - z[i] * is[i] * dsa[i];
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
            const double ratio = wave_sum(loc) / sz;  // = mu_aff / mu (the 1/mc factors cancel)
            smu = ratio * ratio * ratio * mu_c;
            if (st) {
                double wv[5];
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    wv[i] = (z[i] * (s[i] - (i == 4 ? fzmax : 0.0)) + smu - dsa[i] * dza[i]) * is[i];
                cons_tw(wv, mu, rt);
            }
            mode = CORR;
            DSTAMP(8);  // predictor step length + corrector terms
        } else if (mode == CORR) {
            double ds[5], dz[5];
            double amax = 1.0, dmax = 1.0;  // primal (s) and dual (z) distances to the boundary
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
                    const double dsa = -oa[i] - s[i];
                    const double dza = -z[i] - z[i] * is[i] * dsa;
                    ds[i] = -o[i] - s[i];
                    dz[i] = (smu - z[i] * s[i] - dsa * dza - z[i] * ds[i]) * is[i];
                    if (ds[i] < 0.0) amax = fmin(amax, -s[i] * __builtin_amdgcn_rcp(ds[i]));
                    if (dz[i] < 0.0) dmax = fmin(dmax, -z[i] * __builtin_amdgcn_rcp(dz[i]));
                }
            }
#if LMPC_SPLIT_STEP
            const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(amax));
            const double alpd = fmin(1.0, LMPC_STEP_FRAC * wave_min(dmax));
#else
            const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(fmin(amax, dmax))), alpd = alpha;
#endif
            if (st) {
#pragma unroll
                for (int m = 0; m < 3; ++m) f[m] += alpha * (u[m] - f[m]);
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    s[i] += alpha * ds[i];
                    z[i] += alpd * dz[i];
                    is[i] = rcp_nr(s[i]);
                }
            }
            ++ipm_it;
            mode = PRED;
            DSTAMP(9);  // corrector step + iterate update
        } else {
            // ---- polish verification: gradient H u + g, primal feasibility, multiplier signs ----
            S.vec2[lane] = 0.0;
            LMPC_SYNC();
            if (st) {
#pragma unroll
                for (int p = 0; p < 3; ++p) S.vec2[vidx(lane, p)] = u[p];
            }
            LMPC_SYNC();
            const double gl = h_matvec(S, S.vec2, S.scr, lane) + S.gv[lane];
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
            double sres = 0.0;  // stationarity residual on the leg-step's free directions (lmpc_kernel_common.h)
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
                } else if (apex) {  // the cone test is the whole certificate at the apex
                    if (g[2] / mu < fabs(g[0]) + fabs(g[1]) - prm.tol_d * gscale) {
                        act = (g[0] < 0.0 ? 2 : 1) | (g[1] < 0.0 ? 8 : 4);
                        changed = 1;
                    }
                } else {  // (act = 0: no multipliers, the residual is g itself)
                    const LegKkt kk = leg_kkt(act, g, mu, -prm.tol_d * gscale);
                    if (kk.drop >= 0) {
                        act &= ~(1 << kk.drop);
                        changed = 1;
                    }
                    sres = kk.res;
                }
            }
            DSTAMP(10);  // polish verification
            const unsigned long long chg = __ballot(changed);
            if (!chg) {
                // a settled active set is the optimum's only if H u + g vanishes on every free direction; otherwise
                // this attempt cannot verify (another round would repeat it) and the retry ladder takes over
                const double sr = wave_max(sres);
#ifdef LMPC_KKT_DIAG
                if (lane == 0 && qp < LMPC_KKT_DIAG_QPS) {
                    lmpc_kkt_diag_dense[qp][0] = sr / gscale;
                    lmpc_kkt_diag_dense[qp][1] = 0.0;
                    lmpc_kkt_diag_dense[qp][2] = gscale;
                    lmpc_kkt_diag_dense[qp][3] = 1.0;
                }
#endif
#ifndef LMPC_KKT_OFF
                if (sr <= prm.tol_d * gscale)
#endif
                {
                    done = true;
                    break;
                }
                rd = prm.max_rounds - 1;
            }
            keep_tiles = chg ? (__ffsll((long long)chg) - 1) / 5 : 0;  // tile of the first changed leg-step
            if (++rd >= prm.max_rounds) {
                keep_tiles = 0;
                schur = false;  // the interior point resumes: its own right-hand sides and factorisations
                if (++att >= prm.max_attempts) break;
                tol = retry_tol(tol, att);
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
    const int bad = st && (u[0] != u[0] || u[1] != u[1] || u[2] != u[2]);
    const bool anybad = __any(bad);
    // A QP without a verified optimum (iteration caps, non-finite iterate) is left to the Riccati kernel of the
    // same launch, as lmpc_gi_kernel does: flag 0, nothing written.  Flag 1: solved here.
    if (done_out) {
        const bool keep = done && !anybad;
        if (lane == 0) done_out[qp] = keep ? 1 : 0;
        if (!keep) {
            DSTAMP_FLUSH(qp);
            return false;
        }
    }
    // ---- output: stance forces through LDS to the lane of leg-step 4k + j ----
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
    return true;
}

}  // namespace lmpc

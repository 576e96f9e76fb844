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
// ... including rounds that drop factorised faces (new columns: the bordered system); 0: only rounds that add faces
// cost rule in half-units of one solve: 2 per entry, LMPC_SCHUR_CW2 more per column (its matvec), LMPC_SCHUR_SLOPE2
// per diagonal tile a refactorisation would keep, at most LMPC_SCHUR_LIM2
#ifndef LMPC_SCHUR_CW2
#define LMPC_SCHUR_CW2 0
#endif
#ifndef LMPC_SCHUR_SLOPE2
#define LMPC_SCHUR_SLOPE2 4
#endif
#ifndef LMPC_SCHUR_LIM2
#define LMPC_SCHUR_LIM2 10
#endif
// interior-point start: z = LMPC_DENSE_Z0 / s (complementarity LMPC_DENSE_Z0 per pair)
#ifndef LMPC_DENSE_Z0
#define LMPC_DENSE_Z0 1.0
#endif
#ifndef LMPC_POLISH_BORDER
#define LMPC_POLISH_BORDER 1
#endif
// Gondzio centrality correctors per interior-point iteration (0: none, the product; diagnostic A/B)
#ifndef LMPC_GONDZIO
#define LMPC_GONDZIO 0
#endif
#ifndef LMPC_GZ_SKIP
#define LMPC_GZ_SKIP 0.9
#endif
#ifndef LMPC_GZ_DA
#define LMPC_GZ_DA 0.2
#endif
#ifndef LMPC_GZ_GAMMA
#define LMPC_GZ_GAMMA 0.1
#endif
#ifndef LMPC_GZ_BMIN
#define LMPC_GZ_BMIN 0.1
#endif
#ifndef LMPC_GZ_BMAX
#define LMPC_GZ_BMAX 10.0
#endif
// one step of iterative refinement of a verified range-space round whose stationarity residual is above
// LMPC_REFINE_SR of the gradient scale, certified again (round 6); 0: the update as is.  Over 8192 config-2 QPs
// (tools/refine_diag.py, profiles/r06/refine/) 1857 end on a range-space round; their residuals are <= 6.2e-13 of
// gscale except one at 3.4e-12 -- the QP whose forces sat 1.8e-9 from the optimum (the others' corrections <= 3e-10).
// Refining every such QP cost config 2 +3.4 %; this trigger refines that one.
#ifndef LMPC_POLISH_REFINE
#define LMPC_POLISH_REFINE 1
#endif
#ifndef LMPC_REFINE_SR
#ifdef LMPC_REFINE_DIAG
#define LMPC_REFINE_SR 0.0
#else
#define LMPC_REFINE_SR 1e-12
#endif
#endif

namespace lmpc {

// range-space rounds' scratch (S.scr): h_matvec 0..47, entries U / uleg / utyp / Cb 48..119, the round's s 120..125
// (for its refinement) and K's smallest pivot ratio 126, W = M^-1 V and the columns' V from 128
static_assert(48 + 4 * LMPC_SCHUR_KMAX + 2 * LMPC_SCHUR_KMAX + LMPC_SCHUR_KMAX * LMPC_SCHUR_KMAX <= 120 &&
                  120 + LMPC_SCHUR_KMAX + 1 <= 128, "range-space scratch layout");
constexpr int DN_SCHUR_SV = 120;

// nonzero columns of a leg basis (leg_basis puts them first)
template <typename P>
__device__ __forceinline__ int ncols3(const P* T) {
    int n = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) n += (T[q] != 0.0 || T[3 + q] != 0.0 || T[6 + q] != 0.0) ? 1 : 0;
    return n;
}
// sum over the wave of k in 0..7, and its exclusive prefix (lanes in `below`)
__device__ __forceinline__ int wave_count3(int k) {
    return __popcll(__ballot(k & 1)) + 2 * __popcll(__ballot(k & 2)) + 4 * __popcll(__ballot(k & 4));
}
__device__ __forceinline__ int wave_prefix3(int k, unsigned long long below) {
    return __popcll(__ballot(k & 1) & below) + 2 * __popcll(__ballot(k & 2) & below) +
           4 * __popcll(__ballot(k & 4) & below);
}

// One leg-step of a range-space polish round (dense_body): faces act against the factorised round's bact (basis
// Tb in LDS; Tn = leg_basis(act), nap its apex flag).  The kept faces cm = act & bact leave nc free directions,
// nb of them the factorised ones: kc = nc - nb new columns, kr rows (the added faces, each removing one free
// direction, or at a new apex the nc rows u = 0).  ok = false: the round refactorises.
struct SchurLeg {
    int kc, kr;
    bool ok;
};
__device__ __forceinline__ SchurLeg schur_leg(bool chg, int act, int bact, bool nap, const ldouble* Tb,
                                              const double Tn[9], double mu, double fzmax) {
    SchurLeg r{0, 0, true};
    if (!chg) return r;
    const bool bap = (bact & 3) == 3 || (bact & 12) == 12;
    if (bap && nap) return r;  // the force stays zero
    const int cm = act & bact;
    double Tc[9], uc[3];
    (void)leg_basis(cm, mu, fzmax, Tc, uc);
    const int nb = ncols3(Tb), nc = ncols3(Tc), nn = ncols3(Tn);
    r.kc = nc - nb;
    r.kr = nap ? nc : __popc(act & ~bact);
    // the factorised particular solution must lie in the kept space: no f_max face at an apex on either side
    r.ok = r.kc >= 0 && r.kc <= 3 && r.kr <= 3 && (!bap || !(cm & 16)) && (!nap || !((act | bact) & 16)) &&
           (nap || nn == nc - r.kr);
#if !LMPC_POLISH_BORDER
    r.ok = r.ok && r.kc == 0 && !nap && !bap;
#endif
    return r;
}

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
            is[i] = 1.0 / s[i];
            z[i] = LMPC_DENSE_Z0 * is[i];
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
    int nsch = 0, ncol = 0;  // range-space entries (columns + rows) and columns of the current round
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
#if LMPC_POLISH_SCHUR
    // K s = cv of a range-space round (S.scr: entries U / uleg / utyp / Cb, W = M^-1 V in Wc; every lane alike):
    // K = Cb - V'W, rows by their three entries, entries beyond nsch the identity; L D L' without pivoting (K is
    // quasi-definite: columns +, rows -).  Returns true (bad) when a pivot leaves its sign: rank-deficient in rounding.
    auto schur_ksolve = [&](const double (&cv)[LMPC_SCHUR_KMAX], double (&sv)[LMPC_SCHUR_KMAX], double& kmin) -> bool {
        constexpr int KM = LMPC_SCHUR_KMAX;
        const ldouble* U = S.scr + 48;
        const ldouble* uleg = U + 4 * KM;
        const ldouble* utyp = uleg + KM;
        const ldouble* Cb = utyp + KM;
        const ldouble* Wc = S.scr + 128;
        double Am[KM][KM], sg[KM];
        int rb_[KM];
        bool rw[KM];
#pragma unroll
        for (int i = 0; i < KM; ++i) {
            const bool iv = i < nsch;
            rw[i] = iv && utyp[iv ? i : 0] < 0.5;
            rb_[i] = iv ? (int)uleg[i] : 0;
            sg[i] = rw[i] ? -1.0 : 1.0;
        }
#pragma unroll
        for (int i = 0; i < KM; ++i) {
            const bool iv = i < nsch;
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                const bool jv = j < nsch;
                double v = (iv && jv) ? Cb[KM * i + j] : (i == j ? 1.0 : 0.0);
                if (iv && jv) {
                    if (rw[i]) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) v = fma(-U[4 * i + q], Wc[64 * j + vidx(rb_[i], q)], v);
                    } else if (rw[j]) {
#pragma unroll
                        for (int q = 0; q < 3; ++q) v = fma(-U[4 * j + q], Wc[64 * i + vidx(rb_[j], q)], v);
                    }
                }
                Am[i][j] = v;
            }
        }
        bool bad = false;
        double dd[KM];
#pragma unroll
        for (int c = 0; c < KM; ++c) {
            double d = Am[c][c];
#pragma unroll
            for (int b = 0; b < c; ++b) d = fma(-Am[c][b], Am[c][b] * dd[b], d);
            bad |= !(sg[c] * d > 1e-14 * fabs(Am[c][c]));
            if (c < nsch) kmin = fmin(kmin, fabs(d) / fabs(Am[c][c]));  // pivot over its diagonal: K's cancellation
            dd[c] = d;
            const double inv = rcp_nr(d != 0.0 ? d : 1.0);
#pragma unroll
            for (int r = c + 1; r < KM; ++r) {
                double v = Am[r][c];
#pragma unroll
                for (int b = 0; b < c; ++b) v = fma(-Am[r][b], Am[c][b] * dd[b], v);
                Am[r][c] = v * inv;
            }
        }
#pragma unroll
        for (int r = 0; r < KM; ++r) {  // L z = c
            double v = cv[r];
#pragma unroll
            for (int b = 0; b < r; ++b) v = fma(-Am[r][b], sv[b], v);
            sv[r] = v;
        }
#pragma unroll
        for (int r = 0; r < KM; ++r) sv[r] = sv[r] * rcp_nr(dd[r] != 0.0 ? dd[r] : 1.0);
#pragma unroll
        for (int r = KM - 1; r >= 0; --r) {  // L' s = D^-1 z
            double v = sv[r];
#pragma unroll
            for (int b = r + 1; b < KM; ++b) v = fma(-Am[b][r], sv[b], v);
            sv[r] = v;
        }
        return bad;
    };
    // a settled active set failed the certificate right after a range-space round: the same faces once more as a
    // factorised round before the retry ladder (the update's rounding, not the faces, may be what failed)
    bool force_fact = false, refact_done = false;
#endif
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
            if (have_base && !force_fact) {
                // Per changed leg-step: the faces it keeps (cm) span a space of nc free directions holding the
                // factorised basis's nb; the update adds kc = nc - nb of them as new columns (faces dropped) and kr
                // rows (faces added, or at a new apex the nc rows u = 0), each row removing one free direction.
                // Not at an apex with the f_max face (its particular solution is not in the kept space).
                const SchurLeg sl = schur_leg(st && act != bact, act, bact, apex, S.blk + 9 * lane, T, mu, fzmax);
                const int k = sl.kc + sl.kr;
                nsch = wave_count3(k);
                ncol = wave_count3(sl.kc);
                // against a refactorisation from the first changed tile kt on (cheaper the later kt)
                const unsigned long long dif = __ballot(st && act != bact);
                const int kt = dif ? (__ffsll((long long)dif) - 1) / 5 : 4;
                schur = __all(sl.ok) && nsch + ncol <= LMPC_SCHUR_KMAX &&
                        2 * nsch + LMPC_SCHUR_CW2 * ncol + LMPC_SCHUR_SLOPE2 * kt <= LMPC_SCHUR_LIM2;
            }
            // a factorised round: tiles ahead of the first leg-step whose faces differ from the last factorised
            // round's keep their factors
            if (!schur) {
                const unsigned long long dif = __ballot(have_base && act != bact);
                keep_tiles = have_base && dif ? (__ffsll((long long)dif) - 1) / 5 : 0;
                force_fact = false;
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
#if LMPC_POLISH_SCHUR
            S.lhg[lane] = hv;
#endif
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
        double du[3] = {0.0, 0.0, 0.0};  // range-space rounds: the new columns' part of this leg-step's force
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
            // ---- range-space round on the factorised coordinates y (u_b = up_b + T_b y_b) ----
            // Entries e < nsch, in leg-step order, a leg-step's columns before its rows:
            //   column: a new free direction t (unit, in u-space) with coefficient w: v_e = T'H e_t (base
            //           coordinates), c_e = -t'(H up + g)_b;
            //   row:    r'u_b = beta on the base coordinates: v_e = T_b'r (on leg-step b only), c_e = beta - r'up_b.
            // With W_e = M^-1 v_e and s = [w; lambda] the round's KKT system reduces to K s = c - V'y0,
            // K = Cb - V'W (Cb: t't'H blocks between columns, r't between a row and a column of the same leg-step):
            // quasi-definite (columns +, rows -), so LDL' needs no pivoting; y = y0 - W s, u_b += sum of t w.
            constexpr int KM = LMPC_SCHUR_KMAX;
            ldouble* U = S.scr + 48;       // KM x [x0 x1 x2 c]: t (column) or T_b'r (row), and c_e
            ldouble* uleg = U + 4 * KM;    // leg-step of each entry
            ldouble* utyp = uleg + KM;     // 0: row, 1 + j: column j
            ldouble* Cb = utyp + KM;       // KM x KM
            ldouble* Wc = S.scr + 128;     // M^-1 v_e by variable, 64 doubles each
            ldouble* Vc = Wc + 64 * nsch;  // the columns' v_e by variable (nsch + ncol <= KM)
            const SchurLeg sl = schur_leg(st && act != bact, act, bact, apex, S.blk + 9 * lane, Tn, mu, fzmax);
            const unsigned long long below = (1ull << lane) - 1ull;
            const int e0 = wave_prefix3(sl.kc + sl.kr, below), c0 = wave_prefix3(sl.kc, below);
            if (lane < KM * KM) Cb[lane] = 0.0;
            LMPC_SYNC();
            if (sl.kc + sl.kr) {
                const ldouble* Tb = S.blk + 9 * lane;
                const ldouble* ub = S.lup + 3 * lane;
                double Tc[9], uc[3];
                (void)leg_basis(act & bact, mu, fzmax, Tc, uc);
                // new directions: T_c's columns beyond span(T_b) (orthonormal)
                double tv[3][3];
                const int nb = ncols3(Tb);
                if (nb == 0) {
#pragma unroll
                    for (int j = 0; j < 3; ++j)
#pragma unroll
                        for (int p = 0; p < 3; ++p) tv[j][p] = Tc[3 * p + j];
                } else {
                    double best = -1.0, rb[3] = {0.0, 0.0, 0.0};
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        double r[3] = {Tc[q], Tc[3 + q], Tc[6 + q]};
#pragma unroll
                        for (int m = 0; m < 2; ++m) {  // T_b's columns (nb <= 2 where columns are added)
                            const double pr = Tb[m] * r[0] + Tb[3 + m] * r[1] + Tb[6 + m] * r[2];
#pragma unroll
                            for (int p = 0; p < 3; ++p) r[p] = fma(-pr, Tb[3 * p + m], r[p]);
                        }
                        const double n2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
                        if (n2 > best) {
                            best = n2;
                            rb[0] = r[0]; rb[1] = r[1]; rb[2] = r[2];
                        }
                    }
                    const double in = rsq_nr(best > 0.0 ? best : 1.0);
#pragma unroll
                    for (int p = 0; p < 3; ++p) tv[0][p] = rb[p] * in;
                    // second (nb = 1, nc = 3): orthogonal to T_b's column and the first
                    const double b0 = Tb[0], b1 = Tb[3], b2 = Tb[6];
                    tv[1][0] = b1 * tv[0][2] - b2 * tv[0][1];
                    tv[1][1] = b2 * tv[0][0] - b0 * tv[0][2];
                    tv[1][2] = b0 * tv[0][1] - b1 * tv[0][0];
                    tv[2][0] = tv[2][1] = tv[2][2] = 0.0;
                }
                // rows: added faces, or at a new apex T_c's columns (u_b = 0)
                double rv[3][3], rbv[3];
                if (apex) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) rv[j][p] = Tc[3 * p + j];
                        rbv[j] = 0.0;
                    }
                } else {
                    const ActiveRows ar = active_rows(act & ~bact);
                    cons_rowvec(ar.i0, mu, rv[0]);
                    cons_rowvec(ar.i1, mu, rv[1]);
                    cons_rowvec(ar.i2, mu, rv[2]);
                    rbv[0] = ar.i0 == 4 ? fzmax : 0.0;
                    rbv[1] = ar.i1 == 4 ? fzmax : 0.0;
                    rbv[2] = ar.i2 == 4 ? fzmax : 0.0;
                }
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    if (j >= sl.kc) continue;
                    const int e = e0 + j;
                    double c = 0.0;
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        U[4 * e + p] = tv[j][p];
                        c = fma(-tv[j][p], S.lhg[vidx(lane, p)], c);
                    }
                    U[4 * e + 3] = c;
                    uleg[e] = (double)lane;
                    utyp[e] = (double)(1 + c0 + j);
                }
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (i >= sl.kr) continue;
                    const int e = e0 + sl.kc + i;
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        U[4 * e + q] = fma(rv[i][0], Tb[q], fma(rv[i][1], Tb[3 + q], rv[i][2] * Tb[6 + q]));
                    U[4 * e + 3] = rbv[i] - fma(rv[i][0], ub[0], fma(rv[i][1], ub[1], rv[i][2] * ub[2]));
                    uleg[e] = (double)lane;
                    utyp[e] = 0.0;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        if (j >= sl.kc) continue;
                        const double a = rv[i][0] * tv[j][0] + rv[i][1] * tv[j][1] + rv[i][2] * tv[j][2];
                        Cb[KM * e + e0 + j] = a;
                        Cb[KM * (e0 + j) + e] = a;
                    }
                }
            }
            LMPC_SYNC();
            // columns: v = T'H e_t (one matvec each), and the t't'H block of Cb
            if (ncol) {
                const int w16 = lane & 15, bl = 5 * (lane >> 4) + w16 / 3, al = w16 % 3;
                const bool vl = w16 < 15 && bl < nls;
                for (int e = 0; e < nsch; ++e) {  // wave-uniform
                    const double ty = utyp[e];
                    if (ty < 0.5) continue;
                    const int be = (int)uleg[e];
                    S.vec2[lane] = 0.0;
                    LMPC_SYNC();
                    if (lane < 3) S.vec2[vidx(be, lane)] = U[4 * e + lane];
                    LMPC_SYNC();
                    const double h = h_matvec(S, S.vec2, S.scr, lane);
                    LMPC_SYNC();
                    S.vec2[lane] = h;
                    LMPC_SYNC();
                    double v = 0.0;
                    if (vl) {
#pragma unroll
                        for (int p = 0; p < 3; ++p) v = fma(S.blk[9 * bl + 3 * p + al], S.vec2[vidx(bl, p)], v);
                    }
                    Vc[64 * ((int)ty - 1) + lane] = v;
                    if (lane < nsch && utyp[lane] > 0.5) {
                        const int bj = (int)uleg[lane];
                        double c = 0.0;
#pragma unroll
                        for (int p = 0; p < 3; ++p) c = fma(U[4 * lane + p], S.vec2[vidx(bj, p)], c);
                        Cb[KM * lane + e] = c;
                    }
                    LMPC_SYNC();
                }
            }
            // W_e = M^-1 v_e
            for (int e = 0; e < nsch; ++e) {  // wave-uniform
                const double ty = utyp[e];
                if (ty > 0.5) {
                    S.vec[lane] = Vc[64 * ((int)ty - 1) + lane];
                } else {
                    S.vec[lane] = 0.0;
                    LMPC_SYNC();
                    if (lane < 3) S.vec[vidx((int)uleg[e], lane)] = U[4 * e + lane];
                }
                LMPC_SYNC();
                solve_vec();
                Wc[64 * e + lane] = S.vec[lane];
            }
            LMPC_SYNC();
            // column-column products and the columns' right-hand sides (wave sums over the variables)
            if (ncol) {
                const double y0l = S.lua[lane];
                for (int e = 0; e < nsch; ++e) {  // wave-uniform
                    const double ty = utyp[e];
                    if (ty < 0.5) continue;
                    const double vl = Vc[64 * ((int)ty - 1) + lane];
                    const double cy = wave_sum(vl * y0l);
                    if (lane == 0) U[4 * e + 3] -= cy;
                    for (int f = e; f < nsch; ++f) {
                        if (utyp[f] < 0.5) continue;
                        const double g = wave_sum(vl * Wc[64 * f + lane]);
                        if (lane == 0) {
                            Cb[KM * e + f] -= g;
                            if (f != e) Cb[KM * f + e] -= g;
                        }
                    }
                }
                LMPC_SYNC();
            }
            // K's right-hand side c - V'y0 on every lane (entries beyond nsch: 0; the columns' V'y0 is in U already)
            double cv[KM], sv[KM];
#pragma unroll
            for (int i = 0; i < KM; ++i) {
                const bool iv = i < nsch;
                const bool rwi = iv && utyp[iv ? i : 0] < 0.5;
                const int rbi = iv ? (int)uleg[i] : 0;
                double c = iv ? U[4 * i + 3] : 0.0;
                if (rwi) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) c = fma(-U[4 * i + q], S.lua[vidx(rbi, q)], c);
                }
                cv[i] = c;
            }
            double kmin = 1.0;
            const bool bad = schur_ksolve(cv, sv, kmin);
            double yv = S.lua[lane];
#pragma unroll
            for (int j = 0; j < KM; ++j)
                if (j < nsch) yv = fma(-Wc[64 * j + lane], sv[j], yv);
            if (ncol && !bad && st) {
#pragma unroll
                for (int j = 0; j < KM; ++j) {
                    if (j >= nsch || utyp[j] < 0.5 || (int)uleg[j] != lane) continue;
#pragma unroll
                    for (int p = 0; p < 3; ++p) du[p] = fma(U[4 * j + p], sv[j], du[p]);
                }
            }
#if LMPC_POLISH_REFINE
            if (lane == 0) {  // s of this round, for the refinement of a verified round (polish verification below)
#pragma unroll
                for (int j = 0; j < KM; ++j) S.scr[DN_SCHUR_SV + j] = sv[j];
                S.scr[DN_SCHUR_SV + KM] = kmin;
            }
#endif
            // a rank-deficient update (rounding): keep y0; the round will not verify and the next one refactorises
            // the same faces (a settled set that fails right after a range-space round, below)
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
                    u[p] = apex ? 0.0
                                : S.lup[3 * lane + p] + Tb[p * 3] * y3[0] + Tb[p * 3 + 1] * y3[1] + Tb[p * 3 + 2] * y3[2] +
                                      du[p];
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
#if LMPC_GONDZIO
            double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(amax));
            double alpd = fmin(1.0, LMPC_STEP_FRAC * wave_min(dmax));
#else
            const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(amax));
            const double alpd = fmin(1.0, LMPC_STEP_FRAC * wave_min(dmax));
#endif
#else
            const double alpha = fmin(1.0, LMPC_STEP_FRAC * wave_min(fmin(amax, dmax))), alpd = alpha;
#endif
#if LMPC_GONDZIO && LMPC_SPLIT_STEP
            // Gondzio's multiple centrality correctors (diagnostic A/B): while the step is short,
            // pull the complementarity products of the trial point at a longer step into [bmin, bmax] x sigma mu and
            // re-solve with the factorisation in hand; keep the new direction if its step is longer by gamma x delta
            for (int gk = 0; gk < LMPC_GONDZIO; ++gk) {
                const double am = fmin(alpha, alpd);
                if (am >= LMPC_GZ_SKIP) break;  // wave-uniform
                const double tp = fmin(1.0, alpha + LMPC_GZ_DA), td = fmin(1.0, alpd + LMPC_GZ_DA);
                const double lo = LMPC_GZ_BMIN * smu, hi = LMPC_GZ_BMAX * smu;
                double rg[5] = {0.0, 0.0, 0.0, 0.0, 0.0}, dsaz[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                double rtg[3] = {0.0, 0.0, 0.0};
                if (st) {
                    double oa[5], ua[3], wg[5];
#pragma unroll
                    for (int m = 0; m < 3; ++m) ua[m] = S.lua[3 * lane + m];
                    cons_resid(ua, mu, fzmax, oa);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        const double dsa = -oa[i] - s[i];
                        const double dza = -z[i] - z[i] * is[i] * dsa;
                        dsaz[i] = dsa * dza;
                        const double v = (s[i] + tp * ds[i]) * (z[i] + td * dz[i]);
                        const double r = v < lo ? lo - v : (v > hi ? fmax(hi - v, -hi) : 0.0);
                        rg[i] = r;
                        wg[i] = (z[i] * (s[i] - (i == 4 ? fzmax : 0.0)) + smu + r - dsaz[i]) * is[i];
                    }
                    cons_tw(wg, mu, rtg);
                }
                LMPC_SYNC();
                if (st) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) S.vec[vidx(lane, a)] = -(S.gv[vidx(lane, a)] + rtg[a]);
                }
                LMPC_SYNC();
                solve_vec();
                double ug[3] = {0.0, 0.0, 0.0}, dsg[5], dzg[5];
                double amg = 1.0, dmg = 1.0;
#pragma unroll
                for (int i = 0; i < 5; ++i) dsg[i] = dzg[i] = 0.0;
                if (st) {
                    double o[5];
#pragma unroll
                    for (int a = 0; a < 3; ++a) ug[a] = S.vec[vidx(lane, a)];
                    cons_resid(ug, mu, fzmax, o);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        dsg[i] = -o[i] - s[i];
                        dzg[i] = (smu + rg[i] - z[i] * s[i] - dsaz[i] - z[i] * dsg[i]) * is[i];
                        if (dsg[i] < 0.0) amg = fmin(amg, -s[i] * __builtin_amdgcn_rcp(dsg[i]));
                        if (dzg[i] < 0.0) dmg = fmin(dmg, -z[i] * __builtin_amdgcn_rcp(dzg[i]));
                    }
                }
                const double ag = fmin(1.0, LMPC_STEP_FRAC * wave_min(amg));
                const double adg = fmin(1.0, LMPC_STEP_FRAC * wave_min(dmg));
                if (!(fmin(ag, adg) >= am + LMPC_GZ_GAMMA * LMPC_GZ_DA)) break;
                alpha = ag;
                alpd = adg;
#pragma unroll
                for (int m = 0; m < 3; ++m) u[m] = ug[m];
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    ds[i] = dsg[i];
                    dz[i] = dzg[i];
                }
            }
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
#if LMPC_POLISH_SCHUR && LMPC_POLISH_REFINE
                    if (schur && sr > LMPC_REFINE_SR * gscale) {
                        // One step of iterative refinement of a verified range-space round.  The
                        // update solves the round's bordered system [M V; V' Cb] [y; s] = [r0; c] through K = Cb - V'W,
                        // W = M^-1 V; K's rounding, amplified by W, left config 2's forces up to ~2e-9 N from the optimum
                        // (~1e-10 N refactorised).  The residuals come from the gradient G = H u + g in hand (S.vec2):
                        //   base coordinates  rho_y = -T_b'G - (rows' a) lambda
                        //   a column entry    rho_e = -t'G - (r't) lambda;   a row entry  rho_e = c_e - a'y - (r't) w
                        // and the same factorisations give the correction: dy0 = M^-1 rho_y, K ds = rho_s - V'dy0,
                        // dy = dy0 - W ds, du_b = T_b dy_b + t dw.  The refined forces are certified again (feasibility
                        // of the free faces, stationarity / the apex cone test); if they fail, the verified ones stand.
                        constexpr int KM = LMPC_SCHUR_KMAX;
                        const ldouble* U = S.scr + 48;
                        const ldouble* uleg = U + 4 * KM;
                        const ldouble* utyp = uleg + KM;
                        const ldouble* Cb = utyp + KM;
                        const ldouble* Wc = S.scr + 128;
                        const ldouble* Vc = Wc + 64 * nsch;
                        const ldouble* svs = S.scr + DN_SCHUR_SV;
                        double re = 0.0;  // entry residual (lane e)
                        if (lane < nsch) {
                            const int b = (int)uleg[lane];
                            const bool row = utyp[lane] < 0.5;
                            if (row) {
                                re = U[4 * lane + 3];
#pragma unroll
                                for (int q = 0; q < 3; ++q) re = fma(-U[4 * lane + q], S.vec[vidx(b, q)], re);
                            } else {
#pragma unroll
                                for (int p = 0; p < 3; ++p) re = fma(-U[4 * lane + p], S.vec2[vidx(b, p)], re);
                            }
#pragma unroll
                            for (int f = 0; f < KM; ++f)
                                if (f < nsch && (utyp[f] < 0.5) != row) re = fma(-Cb[KM * lane + f], svs[f], re);
                        }
                        // rho_y, lane = variable (16 t + 3 a + q <-> leg-step 5 t + a, component q)
                        const int vw = lane & 15, vb = 5 * (lane >> 4) + vw / 3, vq = vw % 3;
                        double ry = 0.0;
                        if (vw < 15 && vb < nls) {
                            const ldouble* Tb = S.blk + 9 * vb;
#pragma unroll
                            for (int p = 0; p < 3; ++p) ry = fma(-Tb[3 * p + vq], S.vec2[vidx(vb, p)], ry);
#pragma unroll
                            for (int e = 0; e < KM; ++e)
                                if (e < nsch && utyp[e] < 0.5 && (int)uleg[e] == vb) ry = fma(-U[4 * e + vq], svs[e], ry);
                        }
                        LMPC_SYNC();  // the reads of y above come first
                        S.vec[lane] = ry;
                        LMPC_SYNC();
                        solve_vec();  // dy0 = M^-1 rho_y (the base factorisation, untouched by range-space rounds)
                        const double dyl = S.vec[lane];
                        double rc = re;
                        if (lane < nsch && utyp[lane] < 0.5) {
                            const int b = (int)uleg[lane];
#pragma unroll
                            for (int q = 0; q < 3; ++q) rc = fma(-U[4 * lane + q], S.vec[vidx(b, q)], rc);
                        }
                        double cv[KM], dsv[KM];
#pragma unroll
                        for (int e = 0; e < KM; ++e) {
                            cv[e] = 0.0;
                            if (e < nsch) {  // wave-uniform
                                double c = readlane_f64(rc, e);
                                const double ty = utyp[e];
                                if (ty > 0.5) c -= wave_sum(Vc[64 * ((int)ty - 1) + lane] * dyl);
                                cv[e] = c;
                            }
                        }
                        double kmin2 = 1.0;
                        const bool bad2 = schur_ksolve(cv, dsv, kmin2);
                        double dy = dyl;
#pragma unroll
                        for (int j = 0; j < KM; ++j)
                            if (j < nsch) dy = fma(-Wc[64 * j + lane], dsv[j], dy);
                        LMPC_SYNC();
                        S.vec[lane] = dy;
                        LMPC_SYNC();
                        double ur[3] = {u[0], u[1], u[2]};
                        if (st && !apex) {
                            const ldouble* Tb = S.blk + 9 * lane;
                            double d3[3];
#pragma unroll
                            for (int a = 0; a < 3; ++a) d3[a] = S.vec[vidx(lane, a)];
#pragma unroll
                            for (int p = 0; p < 3; ++p) ur[p] += Tb[3 * p] * d3[0] + Tb[3 * p + 1] * d3[1] + Tb[3 * p + 2] * d3[2];
#pragma unroll
                            for (int j = 0; j < KM; ++j) {
                                if (j >= nsch || utyp[j] < 0.5 || (int)uleg[j] != lane) continue;
#pragma unroll
                                for (int p = 0; p < 3; ++p) ur[p] = fma(U[4 * j + p], dsv[j], ur[p]);
                            }
                        }
                        // certify the refined forces
                        S.vec2[lane] = 0.0;
                        LMPC_SYNC();
                        if (st) {
#pragma unroll
                            for (int p = 0; p < 3; ++p) S.vec2[vidx(lane, p)] = ur[p];
                        }
                        LMPC_SYNC();
                        const double gr = h_matvec(S, S.vec2, S.scr, lane) + S.gv[lane];
                        LMPC_SYNC();
                        S.vec2[lane] = gr;
                        LMPC_SYNC();
                        double g2[3] = {0.0, 0.0, 0.0}, gl2 = 1.0;
                        if (st) {
#pragma unroll
                            for (int p = 0; p < 3; ++p) {
                                g2[p] = S.vec2[vidx(lane, p)];
                                gl2 = fmax(gl2, fabs(g2[p]));
                            }
                        }
                        const double gs2 = wave_max(gl2);
                        bool ok = !bad2;
                        if (st) {
                            double o[5];
                            cons_resid(ur, mu, fzmax, o);
#pragma unroll
                            for (int i = 0; i < 5; ++i)
                                if (!((act >> i) & 1) && o[i] > prm.tol_p * fzmax) ok = false;
                            if (apex) {
                                ok = ok && !(g2[2] / mu < fabs(g2[0]) + fabs(g2[1]) - prm.tol_d * gs2);
                            } else {
                                const LegKkt kk = leg_kkt(act, g2, mu, -prm.tol_d * gs2);
                                ok = ok && kk.drop < 0 && kk.res <= prm.tol_d * gs2;
                            }
                        }
#ifdef LMPC_REFINE_DIAG
                        {
                            double dl = 0.0;
#pragma unroll
                            for (int p = 0; p < 3; ++p) dl = fmax(dl, fabs(ur[p] - u[p]));
                            dl = wave_max(dl);
                            const bool allok = __all(ok);
                            if (lane == 0 && qp < LMPC_KKT_DIAG_QPS) {
                                lmpc_refine_diag[qp][0] = sr / gscale;
                                lmpc_refine_diag[qp][1] = S.scr[DN_SCHUR_SV + KM];
                                lmpc_refine_diag[qp][2] = dl;
                                lmpc_refine_diag[qp][3] = allok ? 1.0 : 2.0;
                            }
                        }
#endif
                        if (__all(ok)) {
#pragma unroll
                            for (int p = 0; p < 3; ++p) u[p] = ur[p];
                        }
                    }
#endif
                    done = true;
                    break;
                }
#if LMPC_POLISH_SCHUR
                if (schur && !refact_done) {
                    force_fact = true;  //  the same faces once more, factorised, before the retry ladder
                    refact_done = true;
                } else
#endif
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

// lmpc_hoqp.hip -- batched hierarchical QP of the whole-body controller, one wavefront
// per instance, all levels in one launch.
//
// Reference: src/legged_ctrl/src/wbc_ctrl/HoQp.cpp (one qpOASES QProblem per priority level) and
// include/wbc_ctrl/task.h; caller wbc.cpp:93-99.  Per level l, with Z the null-space basis of every higher
// level's equalities (n x nd, identity at level 0) and x the higher levels' solution:
//   setup   G = A_l Z (m x nd) and the level gradient c = G'(A_l x - b_l)            (HoQp.cpp:94-107)
//           Hy = G'G + 1e-12 I                                                         (:73-92)
//           Z' = Z ker(G), ker from Eigen's FullPivLU (full pivoting, rank threshold
//           eps * min(m, nd) * max pivot, basis Q [-U11^-1 U12; I])                    (:147-156)
//           constraint rows in y: R = [D_stack Z; D_l Z], bounds h = f_stack - D_stack x + w_stack,
//           g = f_l - D_l x, the stacked rows current-first and the slacks current-last, as the
//           reference pairs them                                                      (:58, :109-145, :176-182)
//   solve   min 1/2 y'Hy y + c'y + 1/2 |v|^2  s.t. -v <= 0, D_stack Z y <= h, D_l Z y - v <= g   (:158-174)
//           by a Mehrotra interior point over (y, v) with v eliminated: per iteration
//           K = Hy + R' diag(w) R (w = z/s on frozen rows, w3 (1 + w1)/(1 + w1 + w3) on own rows) on the
//           matrix cores, its LDL' factor with a pivot floor (Hy is singular in double along ker G,
//           where 1e-12 is below the rounding of G'G: such a pivot freezes its coordinate), two solves;
//           afterwards v = max(0, D_l Z y - g) exactly for the final y
//   output  x += Z y (HoQp.h:41-45), w_l = v, and Z <- Z'.
// Layout: the instance records stay in HBM and are read by the level setup only; the level's constraint
// rows R and K live in LDS (one wave = one instance, ~40 KB at the WBC's n = 42); Z, Z' and Hy live in a
// per-instance global scratch, read once per level or once per iteration.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "lmpc_hoqp_device.h"
#include "lmpc_kernel_common.h"

namespace lmpc {
namespace {

constexpr double HQ_REG = 1e-12;        // HoQp.cpp:84
constexpr double HQ_PIV_FLOOR = 1e-13;  // relative to max(1, largest diagonal entry of K)
constexpr double HQ_PIV_BIG = 1e64;     // pivot of a frozen coordinate
constexpr double HQ_FRAC = 0.99;        // fraction of the step to the boundary

typedef __attribute__((address_space(3))) int lint;

}  // namespace

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of instance 0..4095 (tools/hoqp_stamps.py):
// 0 setup (G, c, Hy), 1 FullPivLU + basis, 2 constraint rows + bounds, 3 residuals, 4 K on the matrix cores,
// 5 Cholesky, 6 Newton systems + steps, 7 outputs.
#ifdef LMPC_STAMPS
__device__ unsigned long long lmpc_hoqp_stamps[4096][8];
#define HSTAMP_DECL unsigned long long _hs_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _hs_t0 = __builtin_readcyclecounter();
#define HSTAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _hs_acc[i] += _t - _hs_t0; _hs_t0 = _t; } while (0)
#define HSTAMP_FLUSH(b) do { if (threadIdx.x == 0 && (b) < 4096) for (int _i = 0; _i < 8; ++_i) { lmpc_hoqp_stamps[b][_i] = _hs_acc[_i]; lmpc_hoqp_substamps[b][_i] = _hq_acc[_i]; } } while (0)
// sub-phases of one interior-point iteration: 0 q, 1 R'q, 2 substitutions, 3 R dy + directions, 4 step length,
// 5 mu_aff + corrector targets, 6 update
__device__ unsigned long long lmpc_hoqp_substamps[4096][8];
#define HQSUB_DECL unsigned long long _hq_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _hq_t0 = 0;
#define HQSUB_START() do { _hq_t0 = __builtin_readcyclecounter(); } while (0)
#define HQSUB(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _hq_acc[i] += _t - _hq_t0; _hq_t0 = _t; } while (0)
#else
#define HQSUB_DECL
#define HQSUB_START() do {} while (0)
#define HQSUB(i) do {} while (0)
#define HSTAMP_DECL
#define HSTAMP(i) do {} while (0)
#define HSTAMP_FLUSH(b) do {} while (0)
#endif

// Diagnostic builds only (tools/build, -DHQ_INL_<helper>): that per-iteration helper inlined instead of outlined
// (A/B of the call overhead against register pressure, tools/hoqp_ab.sh).
#ifdef HQ_INL_chol_floor
#define HQ_ATTR_chol_floor always_inline
#else
#define HQ_ATTR_chol_floor noinline
#endif
#ifdef HQ_INL_chol_solve
#define HQ_ATTR_chol_solve always_inline
#else
#define HQ_ATTR_chol_solve noinline
#endif
#ifdef HQ_INL_row_dot
#define HQ_ATTR_row_dot always_inline
#else
#define HQ_ATTR_row_dot noinline
#endif
#ifdef HQ_INL_rt_dot
#define HQ_ATTR_rt_dot always_inline
#else
#define HQ_ATTR_rt_dot noinline
#endif
#ifdef HQ_INL_hy_dot
#define HQ_ATTR_hy_dot always_inline
#else
#define HQ_ATTR_hy_dot noinline
#endif
#ifdef HQ_INL_form_K
#define HQ_ATTR_form_K always_inline
#else
#define HQ_ATTR_form_K noinline
#endif
namespace {

struct HS {
    ldouble* R;    // rmax x ls: constraint rows in y (columns nd..np-1 zero)
    ldouble* KL;   // kmax x ls: G (setup, FullPivLU) then K and its Cholesky factor (lower)
    ldouble* y;    // np
    ldouble* dy;   // np
    ldouble* c;    // np: level gradient
    ldouble* x;    // np: x (n used)
    ldouble* dI;   // np: 1 / L_kk
    ldouble* vb;   // kmax: A x - b during setup
    ldouble* q;    // rmax: per-row operand of R' q
    ldouble* wh;   // rmax: per-row weight of K
    ldouble* t;    // rmax: spare per-row vector
    lint* rt;      // 64: FullPivLU row transpositions
    lint* ct;      // 64: column transpositions
    lint* qp;      // 64: column permutation Q
    lint* pv;      // 64: pivots above the rank threshold
};

__device__ __forceinline__ HS carve(ldouble* sm, const HoqpDev& P) {
    HS S;
    const int ls = hq_ls(P);
    S.R = sm;
    S.KL = S.R + (size_t)P.rmax * ls;
    S.y = S.KL + (size_t)P.kmax * ls;
    S.dy = S.y + P.np;
    S.c = S.dy + P.np;
    S.x = S.c + P.np;
    S.dI = S.x + P.np;
    S.vb = S.dI + P.np;
    S.q = S.vb + P.kmax;
    S.wh = S.q + P.rmax;
    S.t = S.wh + P.rmax;
    S.rt = (lint*)(S.t + P.rmax);
    S.ct = S.rt + 64;
    S.qp = S.ct + 64;
    S.pv = S.qp + 64;
    return S;
}

// level l's blocks inside one record
__device__ __forceinline__ const double* lev_a(const HoqpDev& P, const double* rec, int l) { return rec + P.off[l]; }
__device__ __forceinline__ const double* lev_b(const HoqpDev& P, const double* rec, int l) {
    return rec + P.off[l] + (int64_t)P.m[l] * P.n;
}
__device__ __forceinline__ const double* lev_d(const HoqpDev& P, const double* rec, int l) {
    return rec + P.off[l] + (int64_t)P.m[l] * (P.n + 1);
}
__device__ __forceinline__ const double* lev_f(const HoqpDev& P, const double* rec, int l) {
    return lev_d(P, rec, l) + (int64_t)P.s[l] * P.n;
}

// Row r of level l's constraint block: r < p = sum_{k<l} s_k are the higher levels' rows stacked
// current-first, [d_{l-1}; d_{l-2}; ...; d_0] (stacked_tasks_ = task_ + stacked_tasks_prev_, HoQp.cpp:58);
// r >= p is the level's own row r - p.  Returns the row and its f.
__device__ __forceinline__ const double* cons_row(const HoqpDev& P, const double* rec, int l, int p, int r,
                                                  double& f) {
    int lev = l, idx = r - p;
    if (r < p) {
        idx = r;
        for (int k = l - 1; k >= 0; --k) {
            if (idx < P.s[k]) {
                lev = k;
                break;
            }
            idx -= P.s[k];
        }
    }
    f = lev_f(P, rec, lev)[idx];
    return lev_d(P, rec, lev) + (int64_t)idx * P.n;
}

// C[rows][0..16 nt) = X Z on the matrix cores; X row r = xrow(r) (global, n entries), Z global n x np, of which
// only the nt column tiles that cover the level's nd coordinates are read (columns nd..16 nt - 1 zero; Z == nullptr:
// Z = I, generated, as long as no level above had equalities).  A[m][k] comes from lane 16k+m, B[k][n] from lane
// 16k+n, C element (4i+g, c) lands in register i of lane 16g+c.  Columns 16 nt.. of C are not written.
template <int NP, class RowFn>
__device__ __forceinline__ void gemm_xz(const HoqpDev& P, RowFn xrow, int rows, const gdouble* Z, int nt, ldouble* C,
                                        int ldc, int lane) {
    constexpr int KC = NP / 4, NT = NP / 16;  // k chunks of 4, column tiles
    const int kq = lane >> 4, mm = lane & 15;
    double bz[KC][NT];  // this lane's B operands for every chunk and live tile, loaded once for all row tiles
#pragma unroll
    for (int c = 0; c < KC; ++c) {
        const int k = 4 * c + kq;
#pragma unroll
        for (int J = 0; J < NT; ++J) {
            bz[c][J] = 0.0;
            if (J < nt && k < P.n) bz[c][J] = Z ? (double)Z[(int64_t)k * P.np + 16 * J + mm] : (k == 16 * J + mm ? 1.0 : 0.0);
        }
    }
    for (int I = 0; I * 16 < rows; ++I) {
        const double* xr = (16 * I + mm < rows) ? xrow(16 * I + mm) : nullptr;
        double a[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            const int k = 4 * c + kq;
            a[c] = (xr != nullptr && k < P.n) ? xr[k] : 0.0;
        }
        d4 acc[NT];
#pragma unroll
        for (int J = 0; J < NT; ++J) acc[J] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < KC; ++c)
#pragma unroll
            for (int J = 0; J < NT; ++J)
                if (J < nt) acc[J] = MFMA64(a[c], bz[c][J], acc[J]);
#pragma unroll
        for (int J = 0; J < NT; ++J)
            if (J < nt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 16 * I + 4 * i + kq;
                    if (row < rows) C[row * ldc + 16 * J + mm] = acc[J][i];
                }
            }
    }
}

// max that propagates NaN (fmax drops it): a non-finite input must reach the stop test
__device__ __forceinline__ double nan_max(double a, double b) { return (a > b || a != a) ? a : b; }
struct OpNanMax { __device__ static double f(double a, double b) { return nan_max(a, b); } };

// Outlined helpers receive their arguments in VGPRs and their structs through flat pointers: counts are made
// uniform again (scalar branches and loop bounds instead of exec masks), structs copied to locals once.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint64_t u = (uint64_t)v;
    return (int64_t)(((uint64_t)(uint32_t)uni((int)(u >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)u));
}
__device__ __forceinline__ HoqpDev uniform(const HoqpDev& p) {
    HoqpDev q = p;
    q.n = uni(p.n);
    q.np = uni(p.np);
    q.nt = uni(p.nt);
    q.L = uni(p.L);
#pragma unroll
    for (int i = 0; i < HQ_MAX_LEVELS; ++i) {
        q.m[i] = uni(p.m[i]);
        q.s[i] = uni(p.s[i]);
        q.off[i] = uni64(p.off[i]);
    }
    q.rec_len = uni64(p.rec_len);
    q.slack_len = uni(p.slack_len);
    q.rmax = uni(p.rmax);
    q.kmax = uni(p.kmax);
    q.max_iter = uni(p.max_iter);
    q.scratch_len = uni64(p.scratch_len);
    return q;
}

// Lower tiles (I >= J) of sum_r w_r M[r][.]' M[r][.] over rows 0..rows-1 of an LDS matrix (stride ld,
// columns 0..16 nt - 1), accumulated onto acc[tile(I,J)] (w == nullptr: unit weights).
__device__ __forceinline__ int tid(int I, int J) { return I * (I + 1) / 2 + J; }
// 16-wide tiles that cover the level's nd coordinates (at least one): columns nd..np-1 of G, R and Z are zero
__device__ __forceinline__ int nd_tiles(int nd) { return nd > 16 ? (nd + 15) >> 4 : 1; }
__device__ __forceinline__ void sym_tiles(const ldouble* M, int ld, int rows, const ldouble* w, int nt, d4 acc[10],
                                          int lane) {
    const int kq = lane >> 4, mm = lane & 15;
    for (int r0 = 0; r0 < rows; r0 += 4) {
        const int r = r0 + kq;
        const bool live = r < rows;
        const double wr = live ? (w ? w[r] : 1.0) : 0.0;
        double v[4];
#pragma unroll
        for (int I = 0; I < 4; ++I) v[I] = (live && I < nt) ? M[r * ld + 16 * I + mm] : 0.0;
#pragma unroll
        for (int I = 0; I < 4; ++I)
            if (I < nt) {
                const double a = wr * v[I];
#pragma unroll
                for (int J = 0; J <= I; ++J) acc[tid(I, J)] = MFMA64(a, v[J], acc[tid(I, J)]);
            }
    }
}

// LDL' factor of K (nd x nd) with a pivot floor, lane i = row i held in registers (kr[j] = K_ij, statically
// indexed: NP = np unrolls every loop).  Step k broadcasts the raw column K_jk (rows j > k) through LDS (S.dy
// as the buffer) before its pivot is known, so the LDS round trip overlaps the pivot's reciprocal chain; row
// i's multiplier K_ik / d_k is lane-local.  Row updates stop at the last 16-wide block that holds live
// columns.  The unit lower factor goes back to S.KL (lower part), dI[k] = 1 / d_k.
template <int NP>
__device__ __attribute__((HQ_ATTR_chol_floor)) void chol_floor(const HS& S_, int ls, int nd, int lane) {
    // local copy: members read through the reference (a flat pointer, which may alias LDS) would be reloaded
    // after every LDS store
    const HS S = S_;
    nd = uni(nd);
    ls = uni(ls);
    double kr[NP];
    const bool live = lane < nd;
    const int nt = nd_tiles(nd);
#pragma unroll
    for (int j = 0; j < NP; ++j) kr[j] = 0.0;
    if (live) {  // one exec region, loads unmasked: columns nd..16 nt - 1 of K are zero (zero columns of Z)
#pragma unroll
        for (int J = 0; J < NP / 16; ++J)
            if (J < nt) {
#pragma unroll
                for (int j = 16 * J; j < 16 * J + 16; ++j) kr[j] = S.KL[lane * ls + j];
            }
    }
    const double dmax = wave_max(live ? S.KL[lane * ls + lane] : 0.0);
    const double thr = HQ_PIV_FLOOR * fmax(1.0, dmax);
    ldouble* col = S.dy;
    double di = 0.0;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        if (k < nd) {
            if (lane < NP) col[lane] = lane > k ? kr[k] : 0.0;  // col = S.dy has np = NP entries
            LMPC_SYNC();
            double cj[NP];  // the whole column loaded ahead of the pivot chain (dead rows hold zeros)
#pragma unroll
            for (int j = k + 1; j < NP; ++j) cj[j] = col[j];
            const double pkk = readlane_f64(kr[k], k);
            const double piv = pkk > thr ? pkk : HQ_PIV_BIG;
            const double inv = rcp_nr(piv);
            const double l = kr[k] * inv;
            di = lane == k ? inv : di;
#pragma unroll
            for (int J = k / 16; J < NP / 16; ++J)
                if (J == 0 || J < nt) {  // nt >= 1: block 0 unconditional
#pragma unroll
                    for (int j = (16 * J > k + 1 ? 16 * J : k + 1); j < 16 * J + 16; ++j) kr[j] = fma(-l, cj[j], kr[j]);
                }
            LMPC_SYNC();
        }
    }
    // store the unit lower factor Lt (K = Lt D Lt'; its substitutions need no division per step) over the live
    // tiles with its diagonal, upper part and dead rows zeroed, so the solves load it without masks
    if (live) S.dI[lane] = di;
    LMPC_SYNC();
    if (lane < NP) {
#pragma unroll
        for (int J = 0; J < NP / 16; ++J)
            if (J < nt) {
#pragma unroll
                for (int j = 16 * J; j < 16 * J + 16; ++j) {
                    const double dj = S.dI[j];  // unconditional broadcast load, then a select
                    S.KL[lane * ls + j] = (live && j < lane) ? kr[j] * dj : 0.0;
                }
            }
    }
    LMPC_SYNC();
}

// K u = rhs with K = Lt D Lt' (Lt unit lower in S.KL, zero elsewhere over the live tiles; D^-1 in S.dI): rhs in
// lane i (i < nd); returns u in lane i, also stored to out[i].  Lt v = rhs, then Lt' u = D^-1 v.  The row and
// then the column of Lt a lane needs are loaded up front (NP statically indexed registers); a step of either
// substitution is one readlane broadcast and one fma, in blocks of 8 steps guarded by nd.  A lane's own entry
// needs no select: its coefficients from its own step on are zero, so its accumulator stops at its solution.
template <int NP>
__device__ __attribute__((HQ_ATTR_chol_solve)) double chol_solve(const HS& S_, int ls, int nd, double rhs, ldouble* out,
                                                       int lane) {
    const HS S = S_;
    nd = uni(nd);
    ls = uni(ls);
    const bool live = lane < nd;
    const int nt = nd_tiles(nd);
    double lr[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) lr[k] = 0.0;
    double di = 0.0;
    if (live) {  // row lane of Lt
        di = S.dI[lane];
#pragma unroll
        for (int J = 0; J < NP / 16; ++J)
            if (J < nt) {
#pragma unroll
                for (int k = 16 * J; k < 16 * J + 16; ++k) lr[k] = S.KL[lane * ls + k];
            }
    }
    double acc = live ? rhs : 0.0;
#pragma unroll
    for (int k0 = 0; k0 < NP; k0 += 8)
        if (k0 < nd) {
#pragma unroll
            for (int k = k0; k < k0 + 8; ++k) acc = fma(-lr[k], readlane_f64(acc, k), acc);  // Lt v = rhs
        }
    if (live) {  // column lane of Lt
#pragma unroll
        for (int J = 0; J < NP / 16; ++J)
            if (J < nt) {
#pragma unroll
                for (int k = 16 * J; k < 16 * J + 16; ++k) lr[k] = S.KL[k * ls + lane];
            }
    }
    acc *= di;
#pragma unroll
    for (int k1 = NP; k1 > 0; k1 -= 8)
        if (k1 - 8 < nd) {
#pragma unroll
            for (int k = k1 - 1; k >= k1 - 8; --k) acc = fma(-lr[k], readlane_f64(acc, k), acc);  // Lt' u = D^-1 v
        }
    if (live) out[lane] = acc;
    LMPC_SYNC();
    return acc;
}

// t = R_r . vec (row r): 16-column blocks up to the level's live tiles, each block's 32 loads issued ahead of
// its fmas (columns nd..16 nt - 1 of R and of vec are zero)
template <int NP>
__device__ __attribute__((HQ_ATTR_row_dot)) double row_dot(const HS& S_, int ls, int nd, int r, const ldouble* vec) {
    const HS S = S_;
    ls = uni(ls);
    const int nt = nd_tiles(uni(nd));
    double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int J = 0; J < NP / 16; ++J)
        if (J == 0 || J < nt) {
            double rv[16], vv[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                rv[u] = S.R[r * ls + 16 * J + u];
                vv[u] = vec[16 * J + u];
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u & 3] = fma(rv[u], vv[u], a[u & 3]);
        }
    return (a[0] + a[1]) + (a[2] + a[3]);
}
// (R' q)_j for lane j: 16-row blocks, each block's 32 loads issued ahead of its fmas; rows past nr are never
// read (that LDS is not written at this level)
__device__ __attribute__((HQ_ATTR_rt_dot)) double rt_dot(const HS& S_, int ls, int nr, const ldouble* q, int lane) {
    const HS S = S_;
    nr = uni(nr);
    ls = uni(ls);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    int r = 0;
    for (; r + 16 <= nr; r += 16) {
        double rv[16], qv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            rv[u] = S.R[(r + u) * ls + lane];
            qv[u] = q[r + u];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u & 3] = fma(rv[u], qv[u], a[u & 3]);
    }
    if (r < nr) {
        double rv[16], qv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            rv[u] = r + u < nr ? S.R[(r + u) * ls + lane] : 0.0;
            qv[u] = r + u < nr ? q[r + u] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u & 3] = fma(rv[u], qv[u], a[u & 3]);
    }
    return (a[0] + a[1]) + (a[2] + a[3]);
}
// (Hy y)_j for lane j < nd (Hy in global scratch, np x np)
// every live 16-row block loaded in one batch (one global round trip); rows nd..16 nt - 1 of Hg and y are
// zero, so the block-wide sum is exact
template <int NP>
__device__ __attribute__((HQ_ATTR_hy_dot)) double hy_dot(const HoqpDev& P_, const gdouble* Hg, const ldouble* y, int nd,
                                                   int lane) {
    const HoqpDev P = uniform(P_);
    const int nt = nd_tiles(uni(nd));
    double hv[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) hv[i] = (i < 16 * nt) ? Hg[(int64_t)i * NP + lane] : 0.0;
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int i = 0; i < NP; i += 2)
        if (i < 16 * nt) {
            a0 = fma(hv[i], y[i], a0);
            a1 = fma(hv[i + 1], y[i + 1], a1);
        }
    return a0 + a1;
}

// Eigen FullPivLU of G (m x nd in S.KL) and Z' = Z ker(G) into Zn (n x np); returns the new nd.
// Restates Eigen/src/LU/FullPivLU.h (3.3): compute() and kernel_retval::evalTo (tests/test_hoqp_oracle.py
// pins the CPU restatement, oracle/hoqp.py fullpivlu / fullpivlu_kernel, that this follows step by step).
__device__ __attribute__((noinline)) int fullpivlu_kernel(const HoqpDev& P_, const HS& S_, int m, int nd, const gdouble* Z, gdouble* Zn,
                                int lane) {
    const HS S = S_;
    const HoqpDev P = uniform(P_);
    m = uni(m);
    nd = uni(nd);
    const int ls = hq_ls(P);
    const int size = m < nd ? m : nd;
    int nonzero = size;
    double maxpiv = 0.0;
    if (lane < 64) {
        S.rt[lane] = lane;
        S.ct[lane] = lane;
    }
    LMPC_SYNC();
    for (int k = 0; k < size; ++k) {
        // largest |G_ij| over i >= k, j >= k; the first in column-major order wins a tie (maxCoeff)
        double best = -1.0;
        int brow = k;
        if (lane >= k && lane < nd)
            for (int i = k; i < m; ++i) {
                const double a = fabs(S.KL[i * ls + lane]);
                if (a > best) {
                    best = a;
                    brow = i;
                }
            }
        const double wbest = wave_max(best);
        if (wbest == 0.0) {
            nonzero = k;
            break;
        }
        const unsigned long long hit = __ballot(best == wbest && lane >= k && lane < nd);
        const int c = __ffsll((long long)hit) - 1;
        const int r = __builtin_amdgcn_readlane(brow, c);
        maxpiv = fmax(maxpiv, wbest);
        if (lane == 0) {
            S.rt[k] = r;
            S.ct[k] = c;
        }
        if (r != k && lane < nd) {  // swap rows k, r
            const double a = S.KL[k * ls + lane], b = S.KL[r * ls + lane];
            S.KL[k * ls + lane] = b;
            S.KL[r * ls + lane] = a;
        }
        LMPC_SYNC();
        if (c != k && lane < m) {  // swap columns k, c
            const double a = S.KL[lane * ls + k], b = S.KL[lane * ls + c];
            S.KL[lane * ls + k] = b;
            S.KL[lane * ls + c] = a;
        }
        LMPC_SYNC();
        const double pk = S.KL[k * ls + k];
        if (lane > k && lane < m) {
            const double l = S.KL[lane * ls + k] / pk;
            S.KL[lane * ls + k] = l;
            int j = k + 1;
            for (; j + 8 <= nd; j += 8) {  // loads of a block ahead of its updates
                double a[8], u[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    a[t] = S.KL[lane * ls + j + t];
                    u[t] = S.KL[k * ls + j + t];
                }
#pragma unroll
                for (int t = 0; t < 8; ++t) S.KL[lane * ls + j + t] = a[t] - l * u[t];
            }
            for (; j < nd; ++j) S.KL[lane * ls + j] -= l * S.KL[k * ls + j];
        }
        LMPC_SYNC();
    }
    // permutation Q from the column transpositions, applied in increasing k (m_q)
    if (lane == 0) {
        for (int j = 0; j < nd; ++j) S.qp[j] = j;
        for (int k = 0; k < size; ++k) {
            const int a = S.qp[k], b = S.qp[S.ct[k]];
            S.qp[k] = b;
            S.qp[S.ct[k]] = a;
        }
    }
    // rank: pivots above eps * diagonalSize * maxpivot (rank(), kernel())
    const double thr = maxpiv * (DBL_EPSILON * (double)size);
    int rank = 0;
    if (lane == 0)
        for (int i = 0; i < nonzero; ++i)
            if (fabs(S.KL[i * ls + i]) > thr) S.pv[rank++] = i;
    rank = __builtin_amdgcn_readfirstlane(rank);
    LMPC_SYNC();
    const int dimker = nd - rank;
    if (dimker == 0) {  // trivial kernel: Eigen returns one zero column
        for (int j = 0; j < P.np; ++j)
            if (lane < P.n) Zn[(int64_t)lane * P.np + j] = 0.0;
        return 1;
    }
    // trapezoid m (rank x nd) in place: row i <- U row pv[i] from column i on, head zero
    for (int i = 0; i < rank; ++i) {
        const int src = S.pv[i];
        double v = 0.0;
        if (lane < nd && lane >= i) v = S.KL[src * ls + lane];
        LMPC_SYNC();
        if (lane < nd) S.KL[i * ls + lane] = v;
        LMPC_SYNC();
    }
    // bring the non-negligible pivots onto the diagonal (column swaps), solve U11 M = U12, swap back
    for (int i = 0; i < rank; ++i) {
        const int pc = S.pv[i];
        if (pc != i && lane < rank) {
            const double a = S.KL[lane * ls + i], b = S.KL[lane * ls + pc];
            S.KL[lane * ls + i] = b;
            S.KL[lane * ls + pc] = a;
        }
        LMPC_SYNC();
    }
    if (lane < dimker) {  // back substitution, one right-hand side per lane
        const int col = rank + lane;
        for (int i = rank - 1; i >= 0; --i) {
            double a = S.KL[i * ls + col];
            for (int j = i + 1; j < rank; ++j) a -= S.KL[i * ls + j] * S.KL[j * ls + col];
            S.KL[i * ls + col] = a / S.KL[i * ls + i];
        }
    }
    LMPC_SYNC();
    for (int i = rank - 1; i >= 0; --i) {
        const int pc = S.pv[i];
        if (pc != i && lane < rank) {
            const double a = S.KL[lane * ls + i], b = S.KL[lane * ls + pc];
            S.KL[lane * ls + i] = b;
            S.KL[lane * ls + pc] = a;
        }
        LMPC_SYNC();
    }
    // basis K (nd x dimker): row Q[i] = -M[i] (i < rank), row Q[rank + k] = e_k.  Z' = Z K on the matrix cores,
    // K's entries generated from M and the inverse permutation (S.rt reused: qinv[j] = position of j in Q)
    if (lane < nd) S.rt[S.qp[lane]] = lane;
    LMPC_SYNC();
    const int kq = lane >> 4, mm = lane & 15;
    const int ntk = nd_tiles(dimker);  // Z' column tiles the next level reads (columns dimker..16 ntk - 1 zero)
    for (int I = 0; I * 16 < P.n; ++I) {
        const int zrow = 16 * I + mm;
        d4 acc[4];
#pragma unroll
        for (int J = 0; J < 4; ++J) acc[J] = d4{0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < nd; k0 += 4) {
            const int j = k0 + kq;
            const double a = (zrow < P.n && j < nd) ? (Z ? (double)Z[(int64_t)zrow * P.np + j] : (zrow == j ? 1.0 : 0.0))
                                                    : 0.0;
            const int qi = j < nd ? S.rt[j] : -1;
#pragma unroll
            for (int J = 0; J < 4; ++J)
                if (J < ntk) {
                    const int c = 16 * J + mm;
                    double bk = 0.0;
                    if (qi >= 0 && c < dimker) bk = qi < rank ? -S.KL[qi * ls + rank + c] : (qi - rank == c ? 1.0 : 0.0);
                    acc[J] = MFMA64(a, bk, acc[J]);
                }
        }
#pragma unroll
        for (int J = 0; J < 4; ++J)
            if (J < ntk) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 16 * I + 4 * i + kq;
                    if (row < P.n) Zn[(int64_t)row * P.np + 16 * J + mm] = acc[J][i];
                }
            }
    }
    return dimker;
}

// g . x over n entries of a global row (per-lane rows: uncoalesced), loads issued eight at a time ahead of their
// fmas; amax = max |g_j|
__device__ __forceinline__ double gdot(const double* g, const ldouble* x, int n, double& amax) {
    double a0 = 0.0, a1 = 0.0, mx = 0.0;
    int j = 0;
    for (; j + 8 <= n; j += 8) {
        double gv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) gv[u] = g[j + u];
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            a0 = fma(gv[u], x[j + u], a0);
            a1 = fma(gv[u + 1], x[j + u + 1], a1);
            mx = fmax(mx, fmax(fabs(gv[u]), fabs(gv[u + 1])));
        }
    }
    for (; j < n; ++j) {
        a0 = fma(g[j], x[j], a0);
        mx = fmax(mx, fabs(g[j]));
    }
    amax = mx;
    return a0 + a1;
}

// Level setup: G = A Z (into S.KL), c = G'(A x - b) (S.c), Hy = G'G + 1e-12 I (Hg, full symmetric, the
// 16-wide tiles that cover nd; row stride np).
template <int NP>
__device__ __attribute__((noinline)) void level_setup(const HoqpDev& P_, const HS& S_, const double* rec, int l,
                                                      int nd, const gdouble* Z, gdouble* Hg, int lane) {
    const HS S = S_;
    const HoqpDev P = uniform(P_);
    l = uni(l);
    nd = uni(nd);
    const int ls = hq_ls(P), m = P.m[l], nt = nd_tiles(nd);
    if (lane < P.np) S.c[lane] = 0.0;
    d4 acc[10];
#pragma unroll
    for (int t = 0; t < 10; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    if (m > 0) {
        const double* A = lev_a(P, rec, l);
        gemm_xz<NP>(P, [&](int r) { return A + (int64_t)r * P.n; }, m, Z, nt, S.KL, ls, lane);
        if (lane < m) {
            double amx;
            S.vb[lane] = gdot(A + (int64_t)lane * P.n, S.x, P.n, amx) - lev_b(P, rec, l)[lane];
        }
        LMPC_SYNC();
        if (lane < nd) {
            double a = 0.0;
            for (int i = 0; i < m; ++i) a = fma(S.KL[i * ls + lane], S.vb[i], a);
            S.c[lane] = a;
        }
        sym_tiles(S.KL, ls, m, nullptr, nt, acc, lane);
    }
    const int g = lane >> 4, cc = lane & 15;
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J)
            if (I < nt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 16 * I + 4 * i + g, col = 16 * J + cc;
                    double v = acc[tid(I, J)][i];
                    if (row == col && row < nd) v += HQ_REG;
                    Hg[(int64_t)row * P.np + col] = v;
                    Hg[(int64_t)col * P.np + row] = v;
                }
            }
}

// K = Hy + R' diag(wh) R on the matrix cores (lower tiles covering nd) into S.KL.
__device__ __attribute__((HQ_ATTR_form_K)) void form_K(const HoqpDev& P_, const HS& S_, int nr, int nd, const gdouble* Hg,
                                                 int lane) {
    const HS S = S_;
    const HoqpDev P = uniform(P_);
    nr = uni(nr);
    nd = uni(nd);
    const int ls = hq_ls(P), g = lane >> 4, cc = lane & 15, nt = nd_tiles(nd);
    d4 acc[10];
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J) {
            acc[tid(I, J)] = d4{0.0, 0.0, 0.0, 0.0};
            if (I < nt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[tid(I, J)][i] = Hg[(int64_t)(16 * I + 4 * i + g) * P.np + 16 * J + cc];
            }
        }
    sym_tiles(S.R, ls, nr, S.wh, nt, acc, lane);
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = 0; J <= I; ++J)
            if (I < nt) {
#pragma unroll
                for (int i = 0; i < 4; ++i) S.KL[(16 * I + 4 * i + g) * ls + 16 * J + cc] = acc[tid(I, J)][i];
            }
    LMPC_SYNC();
}

// Constraint rows R = [D_stack; D_l] Z (rows 0..nr-1 of S.R).
template <int NP>
__device__ __attribute__((noinline)) void build_rows(const HoqpDev& P_, const HS& S_, const double* rec, int l, int p,
                                                     int nr, const gdouble* Z, int nd, int lane) {
    const HS S = S_;
    const HoqpDev P = uniform(P_);
    l = uni(l);
    p = uni(p);
    nr = uni(nr);
    gemm_xz<NP>(P, [&](int r) { double f; return cons_row(P, rec, l, p, r, f); }, nr, Z, nd_tiles(uni(nd)), S.R,
                hq_ls(P), lane);
}

// Exact crossover (round 3) after an interior point that stopped short of its clean criterion (degenerate
// rows whose slack and multiplier both vanish, a non-finite direction, the iteration cap): the level's KKT
// system on the active set the iterate identifies (prototyped step for step in tools/hoqp_proto.py, EXACT=1):
//   frozen rows (r < p) active where z > s:        R_A y = h_A, multipliers lambda_A >= 0
//   own rows (r >= p) violated where zg > sg (the row constraint D y - v <= g, not v >= 0: for an inactive own
//   row both v and its multiplier vanish):           the penalty 1/2 (R_r y - g_r)^2, i.e. R_r'R_r in the matrix
// solved as a correction from the iterate y_i, so that where K is singular to rounding (Hy is along ker G: the
// level's objective is flat there) the floored pivots keep the iterate's components, which satisfy the inactive
// rows:  K_A = Hy + sum_violated R_r'R_r + rho R_A'R_A (an augmented-Lagrangian term: the same constrained
// optimum, and K_A invertible where only the active rows bind), d0 = K_A^-1 (rhs - K_A y_i), y0 = y_i + d0,
// T = K_A^-1 R_A' (one solve per active row), (R_A T) lambda = R_A y0 - h_A (LDL' with the same pivot floor),
// y = y0 - T lambda.  The classification is repaired for up to XO_ROUNDS rounds -- the most negative multiplier
// out, the most violated inactive frozen row in, own rows moved to the side they land on -- and the answer is
// taken only if it then verifies: lambda >= 0, every row on its side, and the stationarity residual
// Hy y + c + R'z within 1e-9 of the level's scale; otherwise the iterate is kept.  Returns the verdict
// (uniform); on success S.y holds the exact y.  The reference solves each level exactly with qpOASES
// (HoQp.cpp:158-174), an active-set method: this makes the degenerate levels exact too.
// Repair rounds (round 6: 12, was 6; profiles/r06/hoqp/): on the 1024 distinct bench chains, with 6 rounds 34
// level-2 crossovers failed after the first pass (the level resumed the interior point and tried again) and 27
// levels kept the iterate in the end; with 12, 10 and 7 (9 rounds: 10 kept, 16: 7).  Fewer resumed levels make the
// 4096-chain launch 2 % faster (4.35 vs 4.44 ms); every golden level verifies either way.
#ifndef LMPC_HQ_XO_ROUNDS  // -D: diagnostic A/B builds only
#define LMPC_HQ_XO_ROUNDS 12
#endif
constexpr int XO_ROUNDS = LMPC_HQ_XO_ROUNDS;
#ifdef LMPC_HQ_ITDIAG  // diagnostic builds only: why the last crossover of a chain failed (bits 28-30 of the word)
__device__ int lmpc_hq_xo_reason[65536];
__device__ int lmpc_hq_nnls[65536];  // NNLS calls (low 6 bits) and successes (x 64)
#define HQ_XO_FAIL(code) do { if (threadIdx.x == 0 && blockIdx.x < 65536) lmpc_hq_xo_reason[blockIdx.x] = (code); } while (0)
#else
#define HQ_XO_FAIL(code) do {} while (0)
#endif
constexpr double HQ_HFLOOR = 1e-10;  // interior-point margin on exactly tight frozen rows (kernel, below)
#ifndef LMPC_HQ_XO_TOL
#define LMPC_HQ_XO_TOL 1e-9
#endif
constexpr double HQ_XO_TOL = LMPC_HQ_XO_TOL;  // first-pass interior-point stop ahead of the crossover (two passes)
// Diagnostic A/B (tools/build): the first pass also stops after this many iterations (0 = no cap) and hands its
// iterate to the crossover; a level whose crossover does not verify resumes as after a first-pass stop.
#ifndef LMPC_HQ_XO_EARLY
#define LMPC_HQ_XO_EARLY 0
#endif
constexpr int HQ_XO_EARLY = LMPC_HQ_XO_EARLY;
// Multipliers of a degenerate active set (round 6).  Where the active frozen rows are linearly dependent (a foot at
// the apex of its friction pyramid: four faces tight in three dimensions), the Schur complement R_A T' is singular,
// its floored LDL' picks one multiplier vector of many and that one can have negative entries although a non-negative
// one exists; the repair rule then drops a row, the point leaves the vertex, the row re-enters, and the rounds cycle.
// This finds multipliers lambda >= 0 with R_A' lambda = gr (gr = -(Hy y + c + own rows' terms): the stationarity the
// verification checks) by Lawson-Hanson NNLS on the active rows (normal equations of the passive set by chol_floor /
// chol_solve; passive sets of at most na rows, at most 3 na + 3 outer steps).  Returns lambda in lane a (active row
// S.rt[a]) and whether its residual is within tol.  Uses S.vb, S.KL, S.dI and (through chol_floor) S.dy.
#ifndef LMPC_HQ_XO_NNLS
#define LMPC_HQ_XO_NNLS 1
#endif
template <int NP>
__device__ __attribute__((noinline)) double nnls_rows(const HS& S_, int ls, int na, int nd, double gr, double tol,
                                                      bool& ok, int lane) {
    const HS S = S_;
    ls = uni(ls);
    na = uni(na);
    nd = uni(nd);
    const int nt = nd_tiles(nd);
    const int ra = lane < na ? S.rt[lane] : 0;
    // R_a' u for lane a (u in S.vb, zero past nd)
    auto rdot = [&](int r) {
        double a0 = 0.0, a1 = 0.0;
        for (int j = 0; j < 16 * nt; j += 2) {
            a0 = fma(S.R[r * ls + j], S.vb[j], a0);
            a1 = fma(S.R[r * ls + j + 1], S.vb[j + 1], a1);
        }
        return a0 + a1;
    };
    // u_j = (R_A' lambda)_j for lane j
    auto rtl = [&](double lam) {
        double u = 0.0;
        for (int a = 0; a < na; ++a) {
            const double la = readlane_f64(lam, a);
            if (la != 0.0 && lane < nd) u = fma(la, S.R[uni(S.rt[a]) * ls + lane], u);
        }
        return u;
    };
    LMPC_SYNC();
    if (lane < NP) S.vb[lane] = lane < nd ? gr : 0.0;
    LMPC_SYNC();
    const double rg = lane < na ? rdot(ra) : 0.0;  // (R_A gr)_a
    const double eps = 1e-13 * (1.0 + wave_max(fabs(rg)));
    double lam = 0.0;
    unsigned long long pas = 0;  // passive set: bit a
    for (int outer = 0; outer < 3 * na + 3; ++outer) {
        // w = R_A (gr - R_A' lambda); the most positive w outside the passive set enters
        const double u = rtl(lam);
        LMPC_SYNC();
        if (lane < NP) S.vb[lane] = lane < nd ? u : 0.0;
        LMPC_SYNC();
        const bool mem0 = lane < 64 && ((pas >> lane) & 1);
        const double w = (lane < na && !mem0) ? rg - rdot(ra) : -INFINITY;
        const double wmax = wave_max(w);
        if (!(wmax > eps)) break;
        pas |= 1ull << (__ffsll((long long)__ballot(w == wmax)) - 1);
        for (int inner = 0; inner <= na && pas; ++inner) {
            const bool mem = (pas >> lane) & 1;
            const int m = __popcll(pas);
            const int pos = __popcll(pas & ((1ull << lane) - 1ull));
            // the passive rows' Gram matrix into S.KL (row / column = rank in the passive set), zero-padded to whole tiles
            LMPC_SYNC();
            unsigned long long rem = pas;
            int ai = 0;  // lane i < m: the row index a of the i-th passive row
            for (int col = 0; rem; ++col) {
                const int b = __ffsll((long long)rem) - 1;
                rem &= rem - 1;
                if (col == lane) ai = b;
                const int rb = uni(S.rt[b]);
                if (mem) {
                    double g0 = 0.0, g1 = 0.0;
                    for (int j = 0; j < 16 * nt; j += 2) {
                        g0 = fma(S.R[ra * ls + j], S.R[rb * ls + j], g0);
                        g1 = fma(S.R[ra * ls + j + 1], S.R[rb * ls + j + 1], g1);
                    }
                    S.KL[pos * ls + col] = g0 + g1;
                }
            }
            const int nts = nd_tiles(m);
            if (mem)
                for (int j = m; j < 16 * nts; ++j) S.KL[pos * ls + j] = 0.0;
            const double rsh = __shfl(rg, ai);  // every lane takes part: the source lanes must be active
            const double rhs = lane < m ? rsh : 0.0;
            LMPC_SYNC();
            chol_floor<NP>(S, ls, m, lane);
            const double sv = chol_solve<NP>(S, ls, m, rhs, S.vb, lane);  // lane i: the i-th passive row's value
            const double sp = __shfl(sv, mem ? pos : 0);
            const double sa = mem ? sp : 0.0;
            if (!__any(mem && !(sa > 0.0))) {
                lam = sa;
                break;
            }
            // move toward the passive solution until the first passive multiplier reaches zero, drop the zeros
            const double ratio = (mem && !(sa > 0.0) && lam - sa > 0.0) ? lam / (lam - sa) : INFINITY;
            const double alpha = fmin(1.0, wave_min(ratio));
            lam = mem ? fma(alpha, sa - lam, lam) : 0.0;
            pas &= ~__ballot(mem && !(lam > 0.0));
            lam = ((pas >> lane) & 1) ? lam : 0.0;
        }
    }
    const double u = rtl(lam);
    ok = wave_max(lane < nd ? fabs(u - gr) : 0.0) <= tol && !__any(lane < na && !(lam >= 0.0));
    return lam;
}

template <int NP>
__device__ __attribute__((noinline)) bool crossover(const HoqpDev& P_, const HS& S_, int p, int nr, int nd, double bd0,
                                                    double bd1, int fl0, int fl1, double scale, const gdouble* Hg,
                                                    gdouble* Tg, int lane) {
    const HS S = S_;
    const HoqpDev P = uniform(P_);
    p = uni(p);
    nr = uni(nr);
    nd = uni(nd);
    const int ls = hq_ls(P), np = P.np;
    const double bd[2] = {bd0, bd1};
    int fl[2] = {fl0, fl1};  // bit 0: frozen row active, bit 1: own row violated
    const double yi = lane < nd ? (double)S.y[lane] : 0.0;  // the interior-point iterate (S.y kept until success)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int r = lane + 64 * k;
        if (r < P.rmax) S.t[r] = r < nr ? bd[k] : 0.0;  // every row's bound, for the lanes that own its Schur row
    }
    const double rho = fmax(1.0, wave_max(lane < nd ? (double)Hg[(int64_t)lane * np + lane] : 0.0));
    const double tol = 1e-9 * scale;
    double tyi[2];  // R_r y_i
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int r = lane + 64 * k;
        tyi[k] = r < nr ? row_dot<NP>(S, ls, nd, r, S.y) : 0.0;
    }
    for (int rd = 0; rd < XO_ROUNDS; ++rd) {
        // weights of K_A and the correction's right-hand side: rhs - K_A y_i = -c - Hy y_i + R' (w (bd - R y_i))
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = lane + 64 * k;
            if (r < P.rmax) {
                const double w = r < nr ? ((fl[k] & 1) ? rho : (fl[k] & 2) ? 1.0 : 0.0) : 0.0;
                S.wh[r] = w;
                S.q[r] = r < nr ? w * (bd[k] - tyi[k]) : 0.0;
            }
        }
        LMPC_SYNC();
        form_K(P, S, nr, nd, Hg, lane);
        chol_floor<NP>(S, ls, nd, lane);
        double rr = 0.0;
        if (lane < nd) rr = -S.c[lane] - hy_dot<NP>(P, Hg, S.y, nd, lane) + rt_dot(S, ls, nr, S.q, lane);
        const double d0 = chol_solve<NP>(S, ls, nd, rr, S.vb, lane);
        const double y0 = lane < nd ? yi + d0 : 0.0;
        if (lane < np) S.dy[lane] = y0;
        const unsigned long long m0 = __ballot(fl[0] & 1), m1 = __ballot(fl[1] & 1);
        const int na = __popcll(m0) + __popcll(m1);
        if (na > np || na > 64) { HQ_XO_FAIL(1); return false; }
        LMPC_SYNC();
        // T rows a = K_A^-1 R_{r_a}' (global scratch); active row indices in S.rt
        unsigned long long w0 = m0, w1 = m1;
        for (int a = 0; a < na; ++a) {
            int r;
            if (w0) {
                r = __ffsll((long long)w0) - 1;
                w0 &= w0 - 1;
            } else {
                r = 64 + __ffsll((long long)w1) - 1;
                w1 &= w1 - 1;
            }
            r = uni(r);
            const double rj = lane < nd ? (double)S.R[r * ls + lane] : 0.0;
            const double t = chol_solve<NP>(S, ls, nd, rj, S.vb, lane);
            if (lane < np) Tg[(int64_t)a * np + lane] = lane < nd ? t : 0.0;
            if (lane == 0) S.rt[a] = r;
        }
        LMPC_GSYNC();  // T and the row list visible to every lane
        double lam = 0.0, y = y0;
        if (na > 0) {
            // Schur complement Sm = R_A T' (symmetric): lane b < na holds T row b, forms row b of Sm into S.KL (K_A's
            // factor is no longer needed) and e_b = R_{r_b} y0 - h_{r_b}
            const bool lb = lane < na;
            const int nt = nd_tiles(nd);
            double tb[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) tb[j] = 0.0;
            if (lb) {
#pragma unroll
                for (int J = 0; J < NP / 16; ++J)
                    if (J < nt) {
#pragma unroll
                        for (int j = 16 * J; j < 16 * J + 16; ++j) tb[j] = Tg[(int64_t)lane * np + j];
                    }
            }
            for (int a = 0; a < na; ++a) {
                const int ra = uni(S.rt[a]);
                double v0 = 0.0, v1 = 0.0;
#pragma unroll
                for (int J = 0; J < NP / 16; ++J)
                    if (J < nt) {
#pragma unroll
                        for (int j = 16 * J; j < 16 * J + 16; j += 2) {
                            v0 = fma(S.R[ra * ls + j], tb[j], v0);
                            v1 = fma(S.R[ra * ls + j + 1], tb[j + 1], v1);
                        }
                    }
                if (lb) S.KL[lane * ls + a] = v0 + v1;
            }
            double e = 0.0;
            if (lb) {
                const int rb = S.rt[lane];
                e = row_dot<NP>(S, ls, nd, rb, S.dy) - S.t[rb];
            }
            const int nts = nd_tiles(na);  // padding columns na..16 nts - 1 zero (chol_floor loads whole tiles)
            if (lb)
                for (int j = na; j < 16 * nts; ++j) S.KL[lane * ls + j] = 0.0;
            LMPC_SYNC();
            chol_floor<NP>(S, ls, na, lane);
            lam = chol_solve<NP>(S, ls, na, e, S.vb, lane);  // lane a: lambda_a
            const bool degen = __any(lane < na && S.dI[lane] < 1e-60);  // a floored pivot: dependent active rows
            for (int a = 0; a < na; ++a) {
                const double la = readlane_f64(lam, a);
                if (lane < nd) y = fma(-la, Tg[(int64_t)a * np + lane], y);
            }
            if (lane < np) S.dy[lane] = lane < nd ? y : 0.0;
            LMPC_SYNC();
#if LMPC_HQ_XO_NNLS
            // dependent active rows with a negative multiplier: non-negative multipliers for the same point, if some
            // exist (nnls_rows); the point y is the one above either way
            // (only where the point meets every active row: dependent rows whose bounds disagree have no such point)
            double ares = 0.0;
            if (degen && lane < na) {
                const int rb = S.rt[lane];
                ares = fabs(row_dot<NP>(S, ls, nd, rb, S.dy) - S.t[rb]);
            }
            if (degen && wave_min(lane < na ? lam : INFINITY) < -tol && wave_max(ares) <= tol) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int r = lane + 64 * k;
                    if (r < P.rmax) S.q[r] = (r < nr && r >= p && (fl[k] & 2)) ? row_dot<NP>(S, ls, nd, r, S.dy) - bd[k] : 0.0;
                }
                LMPC_SYNC();
                const double gr = lane < nd ? -(hy_dot<NP>(P, Hg, S.dy, nd, lane) + S.c[lane] + rt_dot(S, ls, nr, S.q, lane)) : 0.0;
                bool ok = false;
                const double ln = nnls_rows<NP>(S, ls, na, nd, gr, tol, ok, lane);
#ifdef LMPC_HQ_ITDIAG
                if (lane == 0 && blockIdx.x < 65536) lmpc_hq_nnls[blockIdx.x] += ok ? 65 : 1;
#endif
                if (lane < np) S.dy[lane] = lane < nd ? y : 0.0;  // chol_floor's column buffer
                LMPC_SYNC();
                if (ok) lam = ln;
            }
#endif
        }
        // verification, and the repair of the classification
        double t[2];
        bool flip = false;
        double vin = -INFINITY;  // most violated inactive frozen row
        bool abad = false;       // an active frozen row the point does not meet (dependent rows with disagreeing bounds)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = lane + 64 * k;
            t[k] = 0.0;
            if (r < nr) {
                t[k] = row_dot<NP>(S, ls, nd, r, S.dy) - bd[k];
                if (r < p) {
                    if (!(fl[k] & 1)) vin = fmax(vin, t[k]);
                    else abad |= !(fabs(t[k]) <= tol);
                } else {
                    const bool fk = (fl[k] & 2) ? !(t[k] >= -tol) : !(t[k] <= tol);
                    flip |= fk;
                }
            }
        }
        const double lmin = wave_min(lane < na ? lam : INFINITY);
        const double vmax = wave_max(vin);
        const bool anyflip = __any(flip);
        if (!(lmin == lmin) || !(vmax == vmax)) { HQ_XO_FAIL(2); return false; }  // non-finite
        bool changed = false;
        if (lmin < -tol) {  // the most negative multiplier's row leaves the active set
            const int a = __ffsll((long long)__ballot(lane < na && lam == lmin)) - 1;
            const int r = uni(S.rt[a]);
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (lane + 64 * k == r) fl[k] &= ~1;
            changed = true;
        }
        if (vmax > tol) {  // the most violated inactive frozen row enters
            int r = -1;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const unsigned long long b = __ballot(lane + 64 * k < p && !(fl[k] & 1) && t[k] == vmax);
                if (r < 0 && b) r = 64 * k + __ffsll((long long)b) - 1;
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (lane + 64 * k == r) fl[k] |= 1;
            changed = true;
        }
        if (anyflip) {  // own rows to the side they land on
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int r = lane + 64 * k;
                if (r >= p && r < nr && ((fl[k] & 2) ? !(t[k] >= -tol) : !(t[k] <= tol))) fl[k] ^= 2;
            }
            changed = true;
        }
        if (changed) continue;
        if (__any(abad)) {
            HQ_XO_FAIL(5);
            return false;
        }
        // stationarity: Hy y + c + R'z, z = lambda on the active frozen rows, R y - g on the violated own rows
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = lane + 64 * k;
            if (r < P.rmax) S.q[r] = (r < nr && (fl[k] & 2)) ? t[k] : 0.0;
        }
        LMPC_SYNC();
        if (lane < na) S.q[S.rt[lane]] = lam;
        LMPC_SYNC();
        double st = 0.0;
        if (lane < nd) st = hy_dot<NP>(P, Hg, S.dy, nd, lane) + S.c[lane] + rt_dot(S, ls, nr, S.q, lane);
        if (__any(!(fabs(st) <= tol) || !(y == y))) { HQ_XO_FAIL(3); return false; }  // NaN fails every comparison
        if (lane < np) S.y[lane] = lane < nd ? y : 0.0;
        LMPC_SYNC();
        HQ_XO_FAIL(0);
        return true;
    }
    HQ_XO_FAIL(4);
    return false;
}

// Interior-point state of the level's rows, slot k = row lane + 64 k (rows < nr = p + s, own rows r >= p).
struct Rows {
    double s1[2], z1[2], v[2];  // own rows: -v <= 0 with slack s1
    double sg[2], zg[2];        // frozen rows: P y <= h; own rows: Dz y - v <= g
    double bd[2];               // h or g
};

}  // namespace

template <int NP>
__global__ void __launch_bounds__(64) lmpc_hoqp_kernel(const HoqpDev P, const double* __restrict__ recs,
                                                       double* __restrict__ xout, double* __restrict__ wout,
                                                       int32_t* __restrict__ status, int32_t* __restrict__ iters,
                                                       double* __restrict__ zout, int32_t* __restrict__ zcols,
                                                       double* __restrict__ scratch, int batch) {
    extern __shared__ __attribute__((aligned(16))) double hq_smem[];
    const int b = blockIdx.x;
    if (b >= batch) return;
    const int lane = threadIdx.x;
    const HS S = carve((ldouble*)hq_smem, P);
    const int ls = hq_ls(P);
    const double* rec = recs + (int64_t)b * P.rec_len;
    gdouble* zbuf[2] = {(gdouble*)(scratch + (int64_t)b * P.scratch_len),
                        (gdouble*)(scratch + (int64_t)b * P.scratch_len + (int64_t)P.n * P.np)};
    gdouble* Hg = (gdouble*)(scratch + (int64_t)b * P.scratch_len + 2 * (int64_t)P.n * P.np);
    gdouble* Tg = Hg + (int64_t)P.np * P.np;  // crossover: K_A^-1 R_A' rows (np x np)
    gdouble* wo = (gdouble*)(wout + (int64_t)b * P.slack_len);
    int zc = 0;
    // a non-finite record entry reaches the first residuals of its level (the residual maximum propagates NaN);
    // so does an overflow: zeros and LMPC_QP_NAN, as the MPC path returns zero forces for a NaN solve
    // (ConvexQPSolver.cpp:321-326)
    bool nonfin = false;
    // x = 0; Z = I is generated, not stored, until the first level with equalities (zident)
    bool zident = true;
    bool any_exact = false;  // some level above took its crossover answer (its active rows are exactly tight)
    if (lane < P.np) S.x[lane] = 0.0;
    LMPC_GSYNC();
    int nd = P.n, p = 0, st = 0;
    HSTAMP_DECL
    HQSUB_DECL
    for (int l = 0; l < P.L; ++l) {
        const int m = P.m[l], s = P.s[l], nr = p + s;
        const gdouble* Z = zident ? nullptr : zbuf[zc];
        // ---- setup: G = A Z into KL, A x - b, c = G'(A x - b), Hy = G'G + 1e-12 I ---------------
        level_setup<NP>(P, S, rec, l, nd, Z, Hg, lane);
        LMPC_GSYNC();
        HSTAMP(0);
        // ---- next basis Z' = Z ker(G) (HoQp.cpp:147-156), before K reuses the buffer ----------------
        int nd_next = nd;
        if (m > 0) nd_next = fullpivlu_kernel(P, S, m, nd, Z, zbuf[zc ^ 1], lane);
        HSTAMP(1);
        // ---- constraint rows R = [D_stack; D_l] Z and their bounds -----------------------------------
        build_rows<NP>(P, S, rec, l, p, nr, Z, nd, lane);
        // A higher level's row that lies in the span of the equalities fixed since (its projection D Z is zero
        // up to rounding) constrains no y: 0 <= h, with h at rounding level when the row was active.  It is
        // dropped (R row zeroed, h = 1) rather than left to make the level infeasible by one ulp.
        double zmax = 0.0;
        if (zident) {
            zmax = 1.0;
        } else {
            if (lane < P.n)
                for (int j = 0; j < nd; ++j) zmax = fmax(zmax, fabs(Z[(int64_t)lane * P.np + j]));
            zmax = wave_max(zmax);
        }
        LMPC_SYNC();
        Rows W;
        double bmax = 0.0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = lane + 64 * k;
            W.s1[k] = W.z1[k] = 1.0;
            W.v[k] = 0.0;
            W.sg[k] = W.zg[k] = 1.0;
            W.bd[k] = 0.0;
            if (r < nr) {
                double f;
                const double* dr = cons_row(P, rec, l, p, r, f);
                double dmx;
                double a = f - gdot(dr, S.x, P.n, dmx);
                if (r < p) {
                    a += wo[r];  // frozen slack, stacked current-last (HoQp.cpp:141-142, :176-182)
                    double rmx = 0.0;
                    for (int j = 0; j < nd; ++j) rmx = fmax(rmx, fabs(S.R[r * ls + j]));
                    if (rmx <= 1e-12 * dmx * zmax) {
                        for (int j = 0; j < P.np; ++j) S.R[r * ls + j] = 0.0;
                        a = 1.0;
                    }
                }
                W.bd[k] = a;
                bmax = fmax(bmax, fabs(a));
                if (r < p) {
                    W.sg[k] = fmax(a, 1.0);
                } else {
                    W.v[k] = fmax(0.0, -a) + 1.0;
                    W.s1[k] = fmax(W.v[k], 1.0);
                    W.sg[k] = fmax(a + W.v[k], 1.0);
                }
            }
        }
        if (lane < P.np) {
            S.y[lane] = 0.0;
            S.dy[lane] = 0.0;
        }
        LMPC_SYNC();
        const double scale = 1.0 + fmax(wave_max(lane < nd ? fabs(S.c[lane]) : 0.0), wave_max(bmax));
        // A frozen row the crossover of a level above left exactly tight has h = 0 up to rounding (or one ulp
        // below).  Several such rows around a vertex leave the level's feasible set without an interior, and the
        // interior point then stalls (slacks to the bottom of the range, multipliers unbounded).  Once a level above
        // took its crossover answer, the interior point sees those bounds raised to HQ_HFLOOR of the scale -- the
        // margin a level-above iterate would have left -- and the crossover then solves with the true bounds.
        const double hb_true[2] = {W.bd[0], W.bd[1]};
        const bool raised = any_exact;  // the interior point below sees the raised bounds
        if (any_exact) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (lane + 64 * k < p) W.bd[k] = fmax(W.bd[k], HQ_HFLOOR * scale);
        }
        const double mc = (double)(p + 2 * s);
        HSTAMP(2);
        // ---- interior point --------------------------------------------------------------------------
        int it = 0;
        bool numstop = false;  // left on a non-finite Newton direction
        bool clean = false;    // stopped on the clean criterion (complementarity and residuals within tolerance)
        double mu_last = 0.0, res_last = 0.0;
        // Two passes (round 3): with the crossover on, the interior point first stops at HQ_XO_TOL (or tol_mu, if
        // looser) and hands its iterate to the crossover; only a level whose crossover does not verify resumes the
        // interior point from that iterate down to tol_mu and tries the crossover again.  The verified answer is
        // the active-set optimum either way.  At 1e-9 every level of the committed WBC golden chains verifies
        // (4.83 -> 4.43 ms per 4096 WBC chains); at 1e-7 (4.00 ms) one of their 48 levels keeps its iterate
        // (1.6e-9 off), because the flat-direction components of the exact answers above it change
        // (tools/hoqp_xo_check.py, profiles/r03/hoqp_2pass/).
        const bool two_pass = P.crossover && P.tol_mu < HQ_XO_TOL;
        bool exact = false;
        int xo = 0;  // iteration word bits 16-17: 1 crossover tried, 2 verified and taken
#ifdef LMPC_HQ_ITDIAG
        int it_p0 = 0;
#endif
        for (int pass = two_pass ? 0 : 1; pass < 2; ++pass) {
            const double tmu = pass == 0 ? HQ_XO_TOL : P.tol_mu;
            for (;; ++it) {
                // residuals: r_d = H x + c + C'z, r_p = C x + slack - d
                double rp1[2], rpg[2], rdv[2];
                double cs = 0.0, res = 0.0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int r = lane + 64 * k;
                    rp1[k] = rpg[k] = rdv[k] = 0.0;
                    if (r < nr) {
                        const double ty = row_dot<NP>(S, ls, nd, r, S.y);
                        S.q[r] = W.zg[k];
                        if (r < p) {
                            rpg[k] = ty + W.sg[k] - W.bd[k];
                            cs += W.sg[k] * W.zg[k];
                        } else {
                            rpg[k] = ty - W.v[k] + W.sg[k] - W.bd[k];
                            rp1[k] = -W.v[k] + W.s1[k];
                            rdv[k] = W.v[k] - W.z1[k] - W.zg[k];
                            cs += W.sg[k] * W.zg[k] + W.s1[k] * W.z1[k];
                        }
                        res = nan_max(res, nan_max(fabs(rpg[k]), nan_max(fabs(rp1[k]), fabs(rdv[k]))));
                    }
                }
                LMPC_SYNC();
                double rdy = 0.0;
                if (lane < nd) {
                    double a = S.c[lane] + rt_dot(S, ls, nr, S.q, lane);
                    a += hy_dot<NP>(P, Hg, S.y, nd, lane);
                    rdy = a;
                    res = nan_max(res, fabs(a));
                }
                const double mu = mc > 0.0 ? wave_sum(cs) / mc : 0.0;
                mu_last = mu;
                res = wave_reduce<OpNanMax>(res);
                res_last = res;
                HSTAMP(3);
                if (!(isfinite(mu) && isfinite(res))) {
                    nonfin = true;
                    break;
                }
                // converged; or degenerate (rows whose slack and multiplier both vanish): complementarity 1e3 below
                // its tolerance while the dual residual stalls within 1e3 of its own, where the huge weights z/s
                // of those rows leave the Newton directions no more accurate than the iterate already is
                clean = mu <= tmu * scale && res <= P.tol_res * scale;
                if (clean || (mu <= 1e-3 * tmu * scale && res <= 1e3 * P.tol_res * scale) || it >= P.max_iter ||
                    (HQ_XO_EARLY > 0 && pass == 0 && it >= HQ_XO_EARLY))
                    break;
                // weights and K = Hy + R' diag(wh) R
                double w1[2], wg[2], dl[2], is1[2], isg[2], idl[2];  // weights and the reciprocals both Newton
#pragma unroll                                                        // systems divide by
                for (int k = 0; k < 2; ++k) {
                    const int r = lane + 64 * k;
                    is1[k] = 1.0 / W.s1[k];
                    isg[k] = 1.0 / W.sg[k];
                    w1[k] = W.z1[k] * is1[k];
                    wg[k] = W.zg[k] * isg[k];
                    dl[k] = 1.0 + w1[k] + wg[k];
                    idl[k] = 1.0 / dl[k];
                    if (r < P.rmax) S.wh[r] = r >= nr ? 0.0 : (r < p ? wg[k] : wg[k] * (1.0 + w1[k]) * idl[k]);
                }
                LMPC_SYNC();
                form_K(P, S, nr, nd, Hg, lane);
                HSTAMP(4);
                chol_floor<NP>(S, ls, nd, lane);
                HSTAMP(5);
                // Newton system for a complementarity target rc (per row): returns dy (lane j) and per-row
                // directions; dz = W C dx + (z r_p - rc)/s, (H + C'WC) dx = -r_d - C'(z r_p - rc)/s
                double ds1[2], dsg[2], dz1[2], dzg[2], dv[2];
                auto newton = [&](const double rc1[2], const double rcg[2]) {
                    HQSUB_START();
                    double rv[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int r = lane + 64 * k;
                        rv[k] = 0.0;
                        if (r < nr) {
                            const double eg = (W.zg[k] * rpg[k] - rcg[k]) * isg[k];
                            if (r < p) {
                                S.q[r] = -eg;
                            } else {
                                const double e1 = (W.z1[k] * rp1[k] - rc1[k]) * is1[k];
                                rv[k] = -rdv[k] + e1 + eg;
                                S.q[r] = -eg + wg[k] * rv[k] * idl[k];
                            }
                        }
                    }
                    LMPC_SYNC();
                    HQSUB(0);
                    const double rhs = lane < nd ? -rdy + rt_dot(S, ls, nr, S.q, lane) : 0.0;
                    HQSUB(1);
                    chol_solve<NP>(S, ls, nd, rhs, S.dy, lane);
                    HQSUB(2);
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int r = lane + 64 * k;
                        ds1[k] = dsg[k] = dz1[k] = dzg[k] = dv[k] = 0.0;
                        if (r < nr) {
                            const double td = row_dot<NP>(S, ls, nd, r, S.dy);
                            double cg = td;
                            if (r >= p) {
                                dv[k] = (rv[k] + wg[k] * td) * idl[k];
                                cg = td - dv[k];
                                ds1[k] = -rp1[k] + dv[k];
                                dz1[k] = (-rc1[k] - W.z1[k] * ds1[k]) * is1[k];
                            }
                            dsg[k] = -rpg[k] - cg;
                            dzg[k] = (-rcg[k] - W.zg[k] * dsg[k]) * isg[k];
                        }
                    }
                    HQSUB(3);
                };
                auto max_step = [&]() {
                    double a = 1.0;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int r = lane + 64 * k;
                        if (r < nr) {
                            if (dsg[k] < 0.0) a = fmin(a, -W.sg[k] / dsg[k]);
                            if (dzg[k] < 0.0) a = fmin(a, -W.zg[k] / dzg[k]);
                            if (r >= p) {
                                if (ds1[k] < 0.0) a = fmin(a, -W.s1[k] / ds1[k]);
                                if (dz1[k] < 0.0) a = fmin(a, -W.z1[k] / dz1[k]);
                            }
                        }
                    }
                    return wave_min(a);
                };
                double rc1[2], rcg[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    rc1[k] = W.s1[k] * W.z1[k];
                    rcg[k] = W.sg[k] * W.zg[k];
                }
                newton(rc1, rcg);
                const double a_aff = max_step();
                HQSUB(4);
                double ca = 0.0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int r = lane + 64 * k;
                    if (r < nr) {
                        ca += (W.sg[k] + a_aff * dsg[k]) * (W.zg[k] + a_aff * dzg[k]);
                        if (r >= p) ca += (W.s1[k] + a_aff * ds1[k]) * (W.z1[k] + a_aff * dz1[k]);
                    }
                }
                const double mu_aff = mc > 0.0 ? wave_sum(ca) / mc : 0.0;
                const double sig = mu > 0.0 ? (mu_aff / mu) * (mu_aff / mu) * (mu_aff / mu) * mu : 0.0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    rc1[k] = W.s1[k] * W.z1[k] + ds1[k] * dz1[k] - sig;
                    rcg[k] = W.sg[k] * W.zg[k] + dsg[k] * dzg[k] - sig;
                }
                HQSUB(5);
                newton(rc1, rcg);
                const double a = fmin(1.0, HQ_FRAC * max_step());
                HQSUB(4);
                // a non-finite direction (weights z/s overflowing as a degenerate level's slacks reach the bottom
                // of the double range) ends the level on the current iterate, which is kept
                bool fin = isfinite(a) && (lane >= nd || isfinite((double)S.dy[lane]));
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    fin = fin && isfinite(dv[k]) && isfinite(ds1[k]) && isfinite(dz1[k]) && isfinite(dsg[k]) &&
                          isfinite(dzg[k]);
                if (__ballot(!fin)) {
                    numstop = true;
                    break;
                }
                if (lane < nd) S.y[lane] += a * S.dy[lane];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    W.v[k] += a * dv[k];
                    W.s1[k] += a * ds1[k];
                    W.z1[k] += a * dz1[k];
                    W.sg[k] += a * dsg[k];
                    W.zg[k] += a * dzg[k];
                }
                LMPC_SYNC();
                HQSUB(6);
                HSTAMP(6);
            }
            // the exact crossover on the identified active set, taken when it verifies: the clean stop's residual
            // tolerance (1e-7 of the scale by default) is far looser than the active-set answer
            if (P.crossover && !nonfin && nr > 0 && nd > 0) {
                int fl[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int r = lane + 64 * k;
                    fl[k] = 0;
                    if (r < p) fl[k] = W.zg[k] > W.sg[k] ? 1 : 0;
                    else if (r < nr) fl[k] = W.zg[k] > W.sg[k] ? 2 : 0;
                }
                exact = crossover<NP>(P, S, p, nr, nd, hb_true[0], hb_true[1], fl[0], fl[1], scale, Hg, Tg, lane);
                xo = exact ? 3 : 1;
                any_exact = any_exact || exact;
            }
#ifdef LMPC_HQ_ITDIAG  // diagnostic builds only: the first pass's iteration count in bits 20-27 of the word
            if (pass == 0) it_p0 = it;
#endif
            // resume only from a finite iterate that stopped on its criterion (not the cap, not a non-finite direction)
            if (exact || nonfin || numstop || it >= P.max_iter || !(nr > 0 && nd > 0)) break;
        }
        const bool xo_verified = exact;
        exact = exact || clean;
        // LMPC_QP_CONVERGED: the clean stop, a verified crossover, or -- documented in lmpc_hoqp.h -- the relaxed
        // degenerate stop (complementarity 1e3 below its tolerance, residuals within 1e3 of theirs); a level left on
        // the iteration cap or on a non-finite direction short of that reports LMPC_QP_MAX_ITER
        const bool relaxed = mu_last <= 1e-3 * P.tol_mu * scale && res_last <= 1e3 * P.tol_res * scale;  // final pass
        if (!exact && (it >= P.max_iter || (numstop && !relaxed))) st = 1;
        // The interior point judged its stop against the raised frozen-row bounds (above).  When this level keeps
        // its iterate (no verified crossover), the iterate is checked against the TRUE bounds of the higher levels:
        // a frozen row beyond its true bound by more than the residual tolerance is LMPC_QP_MAX_ITER.
        if (raised && !xo_verified && st == 0) {
            double viol = 0.0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int r = lane + 64 * k;
                if (r < p) viol = fmax(viol, row_dot<NP>(S, ls, nd, r, S.y) - hb_true[k]);
            }
            if (wave_max(viol) > P.tol_res * scale) st = 1;
        }
#ifdef LMPC_HQ_ITDIAG
        const int xr = (xo & 1) ? lmpc_hq_xo_reason[b < 65536 ? b : 0] : 0;
        if (lane == 0 && iters && b < 65536 && l == P.L - 1) lmpc_hq_xo_reason[b] = lmpc_hq_nnls[b];
        if (iters && lane == 0) iters[(int64_t)b * P.L + l] = it | (xo << 16) | (it_p0 << 20) | (xr << 28);
#else
        if (iters && lane == 0) iters[(int64_t)b * P.L + l] = it | (xo << 16);
#endif
        // ---- outputs: w_l = max(0, D_l Z y - g) for the final y, x += Z y ------------------------------
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = lane + 64 * k;
            if (r >= p && r < nr) wo[r] = fmax(0.0, row_dot<NP>(S, ls, nd, r, S.y) - W.bd[k]);
        }
        double xn = 0.0;
        if (lane < P.n) {
            double a = S.x[lane];
            if (zident) {
                a += S.y[lane];
            } else {
                const gdouble* zr = Z + (int64_t)lane * P.np;
                for (int j = 0; j < nd; ++j) a = fma(zr[j], S.y[j], a);
            }
            xn = a;
            xout[((int64_t)b * P.L + l) * P.n + lane] = a;
        }
        LMPC_SYNC();
        if (lane < P.n) S.x[lane] = xn;
        LMPC_GSYNC();
        if (m > 0) {
            zc ^= 1;  // fullpivlu wrote Z' into zbuf[zc ^ 1]
            zident = false;
            nd = nd_next;
        }
        if (zout) {
            // getStackedZMatrix() of this level (HoQp.h:26-29): the basis the levels below work in, n x nd, in an
            // n x n block whose columns nd.. are zero (rows written coalesced, lane = column)
            gdouble* zo = (gdouble*)(zout + ((int64_t)b * P.L + l) * P.n * P.n);
            const gdouble* Zl = zident ? nullptr : zbuf[zc];
            for (int r = 0; r < P.n; ++r)
                if (lane < P.n)
                    zo[(int64_t)r * P.n + lane] =
                        lane < nd ? (Zl ? (double)Zl[(int64_t)r * P.np + lane] : (r == lane ? 1.0 : 0.0)) : 0.0;
            if (zcols && lane == 0) zcols[(int64_t)b * P.L + l] = nd;
        }
        p = nr;
        HSTAMP(7);
        if (nonfin) {
            // the levels below are not solved: their iteration counts read 0
            if (iters && lane == 0)
                for (int l2 = l + 1; l2 < P.L; ++l2) iters[(int64_t)b * P.L + l2] = 0;
            break;
        }
    }
    HSTAMP_FLUSH(b);
    // non-finite result or residuals: zeros, LMPC_QP_NAN
    bool bad = false;
    for (int l = 0; l < P.L; ++l)
        if (lane < P.n && !isfinite(xout[((int64_t)b * P.L + l) * P.n + lane])) bad = true;
    for (int r = lane; r < P.slack_len; r += 64)
        if (!isfinite(wout[(int64_t)b * P.slack_len + r])) bad = true;
    if (__ballot(bad) || nonfin) {
        for (int l = 0; l < P.L; ++l)
            if (lane < P.n) xout[((int64_t)b * P.L + l) * P.n + lane] = 0.0;
        for (int r = lane; r < P.slack_len; r += 64) wout[(int64_t)b * P.slack_len + r] = 0.0;
        if (zout) {
            for (int64_t e = lane; e < (int64_t)P.L * P.n * P.n; e += 64) zout[(int64_t)b * P.L * P.n * P.n + e] = 0.0;
            if (zcols && lane < P.L) zcols[(int64_t)b * P.L + lane] = 0;
        }
        st = 2;
    }
    if (status && lane == 0) status[b] = st;
}

#ifdef LMPC_HQ_ITDIAG
extern "C" int lmpc_debug_hoqp_nnls(int* out, int n) {
    if (n > 65536) n = 65536;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_hq_nnls), (size_t)n * sizeof(int)) == hipSuccess ? n : -1;
}
#endif
#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_hoqp_stamps(unsigned long long* out, int n) {
    if (n > 4096) n = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_hoqp_stamps), (size_t)n * 8 * sizeof(unsigned long long)) ==
                   hipSuccess ? n : -1;
}
extern "C" int lmpc_debug_hoqp_substamps(unsigned long long* out, int n) {
    if (n > 4096) n = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_hoqp_substamps), (size_t)n * 8 * sizeof(unsigned long long)) ==
                   hipSuccess ? n : -1;
}
#endif

hipError_t launch_hoqp(const HoqpDev& P, const double* rec, int batch, double* x, double* w, int32_t* status,
                       int32_t* iters, double* zout, int32_t* zcols, double* scratch, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    const size_t lds = hq_lds_doubles(P) * sizeof(double);
    switch (P.np) {
        case 16:
            hipLaunchKernelGGL(lmpc_hoqp_kernel<16>, dim3(batch), dim3(64), lds, stream, P, rec, x, w, status, iters,
                               zout, zcols, scratch, batch);
            break;
        case 32:
            hipLaunchKernelGGL(lmpc_hoqp_kernel<32>, dim3(batch), dim3(64), lds, stream, P, rec, x, w, status, iters,
                               zout, zcols, scratch, batch);
            break;
        case 48:
            hipLaunchKernelGGL(lmpc_hoqp_kernel<48>, dim3(batch), dim3(64), lds, stream, P, rec, x, w, status, iters,
                               zout, zcols, scratch, batch);
            break;
        case 64:
            hipLaunchKernelGGL(lmpc_hoqp_kernel<64>, dim3(batch), dim3(64), lds, stream, P, rec, x, w, status, iters,
                               zout, zcols, scratch, batch);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace lmpc

// lmpc_gi.hip -- dual active-set (Goldfarb-Idnani) solve of the condensed GRF QP on gfx950, one
// wavefront per QP, for QPs with 1..20 stance leg-steps (every Go1 trot at H=10).
//
// The reference hands the QP to OSQP (ConvexQPSolver.cpp:182-194, 314-327), which stops at
// eps_abs 1e-3; the parity target is the exact optimum.  A dual active-set method
// reaches it in a finite number of rank-one steps from the unconstrained minimiser, and every
// step is O(N^2) lane-parallel work with short serial chains -- where the interior point
// (lmpc_dense.hip) needs ~10 Cholesky factorisations, each a chain of 20 serial 3x3 pivots.
//
// Problem (after lmpc_dense_common.h's condensation; u = the stance forces, contact frame):
//     min 1/2 u'Hu + g'u   s.t. per stance leg-step b: C u_b + c0 >= 0 (4 pyramid faces, f_max - fz)
// fz >= 0 is implied by the pyramid and not carried.  The CPU checker in oracle/ runs the same method
// (Goldfarb & Idnani 1983) on the same reduced QP; the kernel differs only in representation:
//   - J (J J' = H^-1) starts as U^-1 with H = U'U from the tiled fp64-MFMA Cholesky, one row per lane
//     in registers (64 doubles: row v = variable v of the padded 4x16 layout);
//   - an add turns J's inactive columns with one Householder reflection (the checker: a Givens sweep);
//   - R (J1' N_A, upper triangular) is never formed: its inverse is kept packed in LDS, so r = R^-1 d1
//     is a lane-parallel product (no serial back-substitution).  An add appends the column
//     (-r/|d2|, 1/|d2|); a drop applies the adjacent-column rotations that zero row lpos of R^-1
//     (they are the oracle's re-triangularising Givens, up to sign) to the columns of R^-1 and of J
//     (one carried sweep over the register row) and deletes row lpos.
// Every step is the oracle's: most violated constraint (tol 1e-11 (1 + |x|_inf)), full / partial
// step lengths, dependent-normal test |J2'n|^2 > 1e-24 |J'n|^2.  A QP that hits the step cap or a
// non-finite step is left to the Riccati kernel (flag 0 in `done`).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_dense_common.h"
#include "lmpc_device.h"
#include "lmpc_kernel_common.h"

namespace lmpc {

// Diagnostic build only (-DLMPC_STAMPS): per-phase cycle counters of QP 0..4095 (tools/dense_check.py).
#ifdef LMPC_STAMPS
__device__ unsigned long long lmpc_gi_stamps[4096][8];
#define GSTAMP_DECL unsigned long long _gs_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long _gs_t0 = __builtin_readcyclecounter();
#define GSTAMP(i) do { const unsigned long long _t = __builtin_readcyclecounter(); _gs_acc[i] += _t - _gs_t0; _gs_t0 = _t; } while (0)
#define GSTAMP_FLUSH(qp) do { if (threadIdx.x == 0 && (qp) < 4096) for (int _i = 0; _i < 8; ++_i) lmpc_gi_stamps[qp][_i] = _gs_acc[_i]; } while (0)
#else
#define GSTAMP_DECL
#define GSTAMP(i) do {} while (0)
#define GSTAMP_FLUSH(qp) do {} while (0)
#endif

#ifdef LMPC_KKT_DIAG
// diagnostic build (tools/kkt_diag.py): per QP, the certificate's stationarity residual / gscale and its verdict
__device__ double lmpc_kkt_diag_gi[LMPC_KKT_DIAG_QPS][4];
extern "C" int lmpc_debug_kkt_gi(double* out, int nqp) {
    if (nqp > LMPC_KKT_DIAG_QPS) nqp = LMPC_KKT_DIAG_QPS;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_kkt_diag_gi), (size_t)nqp * 4 * sizeof(double)) == hipSuccess ? nqp
                                                                                                                 : -1;
}
#endif

constexpr int GI_EXTRA = 3 * 64 + 3 * 64 + 2 * 64;  // LDS doubles ahead of the DSmem area

struct GSmem {
    ldouble* rows;  // 3 x 64: n_a * J[v_a][:] for the three variables of the entering constraint
    ldouble* dv;    // 64: d = J' n_p (broadcast for r = R^-1 d1)
    ldouble* dm;    // 64: d restricted to the inactive columns (c >= q)
    ldouble* hv;    // 64: Householder vector
    ldouble* gcs;   // 2 x 64: Givens (c, s) of a drop, per column pair (j, j+1)
};
__device__ __forceinline__ GSmem gcarve(ldouble* p) {
    GSmem g;
    g.rows = p; p += 3 * 64;
    g.dv = p; p += 64;
    g.dm = p; p += 64;
    g.hv = p; p += 64;
    g.gcs = p;
    return g;
}
// packed upper-triangular R^-1: column c at c(c+3)/2, rows 0..c+1 (one subdiagonal slot for the drop)
__device__ __forceinline__ int roff(int c) { return c * (c + 3) / 2; }

// constraint value s_f(u) = C_f u + c0_f (>= 0 feasible): faces fx + mu fz, -fx + mu fz, fy + mu fz,
// -fy + mu fz, fmax - fz  (= -cons_resid)
__device__ __forceinline__ double face_val(int f, double u0, double u1, double u2, double mu, double fzmax) {
    return f == 0 ? u0 + mu * u2 : f == 1 ? -u0 + mu * u2 : f == 2 ? u1 + mu * u2 : f == 3 ? -u1 + mu * u2 : fzmax - u2;
}
__device__ __forceinline__ double face_n(int f, int a, double mu) {
    if (a == 2) return f == 4 ? -1.0 : mu;
    if (a == 0) return f == 0 ? 1.0 : f == 1 ? -1.0 : 0.0;
    return f == 2 ? 1.0 : f == 3 ? -1.0 : 0.0;
}

// Materialise a value at this point.  LLVM's IR passes otherwise sink the arithmetic of the chunked
// loops below past every chunk fence (to its first use, even past a loop) while the operand loads
// stay put: all 64 loads then hold 128 VGPRs at once and the J row spills to AGPRs.
__device__ __forceinline__ double pin(double v) {
    asm volatile("" : "+v"(v));
    return v;
}
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2v ld2;
// The LDS vectors below are read 8 doubles at a time (4 x ds_read_b128) with a scheduling barrier
// between chunks: left alone, the scheduler hoists all 64 loads ahead of the FMAs and the J row
// (128 VGPRs) no longer fits.
#define GI_CHUNK_FENCE() __builtin_amdgcn_sched_barrier(0)

// two / three wave reductions interleaved (independent DPP chains)
__device__ __forceinline__ void wave_max2(double& a, double& b) {
    a = fmax(a, dpp_f64<DPP_QP_1032>(a));
    b = fmax(b, dpp_f64<DPP_QP_1032>(b));
    a = fmax(a, dpp_f64<DPP_QP_2301>(a));
    b = fmax(b, dpp_f64<DPP_QP_2301>(b));
    a = fmax(a, dpp_f64<DPP_ROR4>(a));
    b = fmax(b, dpp_f64<DPP_ROR4>(b));
    a = fmax(a, dpp_f64<DPP_ROR8>(a));
    b = fmax(b, dpp_f64<DPP_ROR8>(b));
    a = fmax(fmax(readlane_f64(a, 0), readlane_f64(a, 16)), fmax(readlane_f64(a, 32), readlane_f64(a, 48)));
    b = fmax(fmax(readlane_f64(b, 0), readlane_f64(b, 16)), fmax(readlane_f64(b, 32), readlane_f64(b, 48)));
}
__device__ __forceinline__ void wave_sum3(double& a, double& b, double& c) {
    a += dpp_f64<DPP_QP_1032>(a);
    b += dpp_f64<DPP_QP_1032>(b);
    c += dpp_f64<DPP_QP_1032>(c);
    a += dpp_f64<DPP_QP_2301>(a);
    b += dpp_f64<DPP_QP_2301>(b);
    c += dpp_f64<DPP_QP_2301>(c);
    a += dpp_f64<DPP_ROR4>(a);
    b += dpp_f64<DPP_ROR4>(b);
    c += dpp_f64<DPP_ROR4>(c);
    a += dpp_f64<DPP_ROR8>(a);
    b += dpp_f64<DPP_ROR8>(b);
    c += dpp_f64<DPP_ROR8>(c);
    a = (readlane_f64(a, 0) + readlane_f64(a, 16)) + (readlane_f64(a, 32) + readlane_f64(a, 48));
    b = (readlane_f64(b, 0) + readlane_f64(b, 16)) + (readlane_f64(b, 32) + readlane_f64(b, 48));
    c = (readlane_f64(c, 0) + readlane_f64(c, 16)) + (readlane_f64(c, 32) + readlane_f64(c, 48));
}

// 8 doubles of an LDS vector (broadcast reads, 4 x ds_read_b128)
struct Chunk8 {
    d2v p[4];
};
__device__ __forceinline__ Chunk8 ld_chunk(const ld2* v2, int c) {
    Chunk8 k;
#pragma unroll
    for (int i = 0; i < 4; ++i) k.p[i] = v2[c / 2 + i];
    return k;
}

// Dot of the register row with an LDS vector (zero below the first inactive column q), 4 independent
// chains, all 64 columns: a uniform branch per chunk to skip those below q cost more (waits at the block
// joins) than it saved.  Chunk k+1's loads are issued before chunk k's FMAs into a static double buffer
// (no register copies).
__device__ __forceinline__ double row_dot(const double (&Jr)[64], const ldouble* v) {
    const ld2* v2 = (const ld2*)v;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    Chunk8 buf[2];
    buf[0] = ld_chunk(v2, 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (k + 1 < 8) buf[(k + 1) & 1] = ld_chunk(v2, 8 * (k + 1));
        {
            const Chunk8& cur = buf[k & 1];
            const int c = 8 * k;
            a0 = fma(Jr[c], cur.p[0].x, a0);
            a1 = fma(Jr[c + 1], cur.p[0].y, a1);
            a2 = fma(Jr[c + 2], cur.p[1].x, a2);
            a3 = fma(Jr[c + 3], cur.p[1].y, a3);
            a0 = fma(Jr[c + 4], cur.p[2].x, a0);
            a1 = fma(Jr[c + 5], cur.p[2].y, a1);
            a2 = fma(Jr[c + 6], cur.p[3].x, a2);
            a3 = fma(Jr[c + 7], cur.p[3].y, a3);
            a0 = pin(a0);
            a1 = pin(a1);
            a2 = pin(a2);
            a3 = pin(a3);
        }
        GI_CHUNK_FENCE();
    }
    return pin((a0 + a1) + (a2 + a3));
}
// Jr -= w * v (v zero below q), pipelined like row_dot
__device__ __forceinline__ void row_axpy(double (&Jr)[64], double w, const ldouble* v) {
    const ld2* v2 = (const ld2*)v;
    Chunk8 buf[2];
    buf[0] = ld_chunk(v2, 0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (k + 1 < 8) buf[(k + 1) & 1] = ld_chunk(v2, 8 * (k + 1));
        {
            const Chunk8& cur = buf[k & 1];
            const int c = 8 * k;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                Jr[c + 2 * i] = pin(fma(-w, cur.p[i].x, Jr[c + 2 * i]));
                Jr[c + 2 * i + 1] = pin(fma(-w, cur.p[i].y, Jr[c + 2 * i + 1]));
            }
        }
        GI_CHUNK_FENCE();
    }
}

template <bool TERRAIN>
__global__ void __launch_bounds__(64) lmpc_gi_kernel(const DevParams prm, const double* __restrict__ rec,
                                                     const uint8_t* __restrict__ contact,
                                                     const double* __restrict__ normals, int batch,
                                                     double* __restrict__ grf, int32_t* __restrict__ status,
                                                     int32_t* __restrict__ iters, uint8_t* __restrict__ done) {
    extern __shared__ __attribute__((aligned(16))) double gi_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    const bool stl = lane < 4 * H && contact[(size_t)qp * 4 * H + lane] != 0;
    const unsigned long long smask = __ballot(stl);
    const int nls = __popcll(smask);
    if (nls > DENSE_MAX_LS || nls == 0) return;  // Riccati kernel (it also owns the all-swing QPs)
    const GSmem G = gcarve((ldouble*)gi_smem);  // GI buffers first, then the dense-path carve
    const DSmem S = dcarve(gi_smem + GI_EXTRA, H);
    const double mu = prm.mu, fzmax = prm.fmax;
    GSTAMP_DECL

    const int rank = dense_prologue<TERRAIN>(prm, S, rec, normals, qp, H, smask, stl, lane);
    dense_condense<TERRAIN>(prm, S, H, nls, smask, lane);
    GSTAMP(0);  // prologue + condensation

    const int lc = lane & 15, lr = lane >> 4;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    double Jr[64];
    double xv;
    {
        // ---- H = U'U on the matrix cores (lmpc_dense.hip's tiled Cholesky, D = 0) ----
        d4 Tl[10], Ui[4], UiT[4];
#pragma unroll
        for (int t = 0; t < 10; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) Tl[t][i] = S.Ht[t * DN_TILE + i * 64 + lane];
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            {
                const DiagInv di = diag_inverse(S.scr, Tl[tix(b, b)], tile_mask(S, b, nls, false), lane);
                Ui[b] = di.ui;
                UiT[b] = di.uit;
            }
#pragma unroll
            for (int c = b + 1; c < 4; ++c) Tl[tix(b, c)] = tprod(Ui[b], Tl[tix(b, c)], zero);  // U_bc
#pragma unroll
            for (int c = b + 1; c < 4; ++c) {
#pragma unroll
                for (int d = c; d < 4; ++d) Tl[tix(c, d)] = tprod_sub(Tl[tix(b, c)], Tl[tix(b, d)], Tl[tix(c, d)]);
            }
        }
        // ---- unconstrained minimiser x0 = -H^-1 g: U'y = -g, U x = y ----
        {
            d4 y[4], x[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
#pragma unroll
                for (int i = 0; i < 4; ++i) y[b][i] = -S.gv[16 * b + lr + 4 * i];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                d4 acc = y[b];
#pragma unroll
                for (int a = 0; a < b; ++a) acc = tprod_sub(Tl[tix(a, b)], y[a], acc);
                y[b] = tprod(Ui[b], acc, zero);
            }
            double xcol[4];
#pragma unroll
            for (int b = 3; b >= 0; --b) {
                d4 acc = y[b];
                if (b < 3) {
                    double part[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int c = b + 1; c < 4; ++c) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) part[i] = fma(Tl[tix(b, c)][i], xcol[c], part[i]);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i] -= row_sum(part[i]);
                }
                x[b] = tprod(UiT[b], acc, zero);
                if (lc == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) S.vec[16 * b + lr + 4 * i] = x[b][i];
                }
                LMPC_SYNC();
                if (b > 0) xcol[b] = S.vec[16 * b + lc];
            }
            xv = S.vec[lane];
        }
        // ---- J = U^-1, built as its transpose Y = U^-T (lower): Y_bb = U_bb^-T,
        //      Y_cb = -U_cc^-T sum_{k=b}^{c-1} U_kc' Y_kb  (X'Y products only, no tile transposes) ----
        d4 Y[10];  // Y_cb at tix(b, c)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            Y[tix(b, b)] = UiT[b];
#pragma unroll
            for (int c = b + 1; c < 4; ++c) {
                d4 acc = zero;
#pragma unroll
                for (int k = b; k < c; ++k) acc = tprod(Tl[tix(k, c)], Y[tix(b, k)], acc);
                const d4 yc = tprod(Ui[c], acc, zero);
                Y[tix(b, c)] = -yc;
            }
        }
        // Y tiles back into the Ht slots (same packing: tile (b, c), b <= c, holds Y_cb): the tile
        // registers die here, so the J row below is allocated fresh (VGPRs, not AGPR spill space)
#pragma unroll
        for (int t = 0; t < 10; ++t) {
#pragma unroll
            for (int i = 0; i < 4; ++i) S.Ht[t * DN_TILE + i * 64 + lane] = Y[t][i];
        }
    }
    LMPC_SYNC();
    // ---- J row v = lane: J(v, col) = Y(col, v) = element (col & 15, v & 15) of tile (v >> 4, col >> 4) ----
    {
        const int rt = lane >> 4, w = lane & 15;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            const ldouble* base = S.Ht + tix(rt <= ct ? rt : 0, ct) * DN_TILE + w;
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) Jr[16 * ct + cc] = (rt <= ct) ? base[toff(cc, 0)] : 0.0;
        }
    }
    GSTAMP(1);  // Cholesky, x0, J

    // ---- dual active-set iterations ----
    // lane k < q: active slot k (constraint id actc = 5 b + f, multiplier uu); R^-1 packed in LDS
    // lane b < nls: stance leg-step b (bit f of lact = face f active)
    ldouble* const Ri = S.Ht;
    int q = 0, it = 0, lact = 0, actc = 0, ndrop = 0;
    double uu = 0.0;
    bool ok = true;
    const int lvb = (lane < nls) ? lane : 0;
    const int lv0 = vidx(lvb, 0);
    for (;;) {
        // ---- most violated inactive constraint ----
        S.vec[lane] = xv;  // broadcast copy of x
        LMPC_SYNC();
        double best = INFINITY;
        int bestid = 0;
        if (lane < nls) {
            const double u0 = S.vec[lv0], u1 = S.vec[lv0 + 1], u2 = S.vec[lv0 + 2];
#pragma unroll
            for (int f = 0; f < 5; ++f) {
                const double v = face_val(f, u0, u1, u2, mu, fzmax);
                if (!((lact >> f) & 1) && v < best) {
                    best = v;
                    bestid = 5 * lane + f;
                }
            }
        }
        double xn = fabs(xv), nb = -best;
        wave_max2(xn, nb);
        const double smin = -nb;
        GSTAMP(2);  // violation search
        if (!(smin < -1e-11 * (1.0 + xn))) break;
        const unsigned long long wm = __ballot(best == smin);
        const int p = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_readlane(bestid, (int)__builtin_ctzll(wm)));
        const int bp = p / 5, fp = p - 5 * bp;
        const int vp = vidx(bp, 0);
        const double n0 = face_n(fp, 0, mu), n1 = face_n(fp, 1, mu), n2 = face_n(fp, 2, mu);
        double sp = smin, uuq = 0.0;
        for (;;) {
            if (++it > prm.gi_max_steps) {  // (configs 2/4: mean 27, max 75 steps)
                ok = false;
                break;
            }
            // ---- d = J' n_p: the entering constraint's three rows of J, scaled ----
            {
                // raw rows (the face normal is applied on the read side: 3 FMAs, not 64 multiplies)
                const int a = lane - vp;
                if (a >= 0 && a < 3) {
                    ld2* row = (ld2*)(G.rows + 64 * a);
#pragma unroll
                    for (int c = 0; c < 64; c += 2) {
                        d2v w2;
                        w2.x = Jr[c];
                        w2.y = Jr[c + 1];
                        row[c / 2] = w2;
                    }
                }
            }
            LMPC_SYNC();
            const double dc = fma(n0, G.rows[lane], fma(n1, G.rows[64 + lane], n2 * G.rows[128 + lane]));
            const double dmc = lane >= q ? dc : 0.0;
            G.dv[lane] = dc;
            G.dm[lane] = dmc;
            double dd = dc * dc, dd2 = dmc * dmc, tail = lane > q ? dc * dc : 0.0;
            wave_sum3(dd, dd2, tail);
            LMPC_SYNC();
            GSTAMP(3);  // d = J'n, norms
            // ---- z = J2 d2 (lane i = variable i) ----
            const double z = row_dot(Jr, G.dm);
            // ---- r = R^-1 d1 (lane k < q): independent products, no serial chain; the loads of the next
            //      group of 8 columns are issued before this group's FMAs ----
            double rk;
            {
                double r0 = 0.0, r1 = 0.0;
                double a[8], dvv[8];
#pragma unroll
                for (int i2 = 0; i2 < 8; ++i2) {
                    a[i2] = (lane <= i2 && i2 < q) ? Ri[roff(i2) + lane] : 0.0;
                    dvv[i2] = G.dv[i2];
                }
                for (int c0 = 0; c0 < q; c0 += 8) {
                    double an[8], dn[8];
#pragma unroll
                    for (int i2 = 0; i2 < 8; ++i2) {
                        const int c = c0 + 8 + i2;
                        an[i2] = (lane <= c && c < q) ? Ri[roff(c) + lane] : 0.0;
                        dn[i2] = G.dv[c < 64 ? c : 63];
                    }
#pragma unroll
                    for (int i2 = 0; i2 < 8; i2 += 2) {
                        r0 = fma(a[i2], dvv[i2], r0);
                        r1 = fma(a[i2 + 1], dvv[i2 + 1], r1);
                    }
#pragma unroll
                    for (int i2 = 0; i2 < 8; ++i2) {
                        a[i2] = an[i2];
                        dvv[i2] = dn[i2];
                    }
                }
                rk = lane < q ? r0 + r1 : 0.0;
            }
            GSTAMP(4);  // z, r
            // ---- step lengths ----
            const double cand = (lane < q && rk > 0.0) ? uu / rk : INFINITY;
            const double t1 = wave_min(cand);
            const bool zfree = dd2 > 1e-24 * dd;
            const double t2 = zfree ? -sp / dd2 : INFINITY;
            const double ts = fmin(t1, t2);
            if (!(ts < INFINITY)) {
                ok = false;
                break;
            }
            if (zfree) xv = fma(ts, z, xv);
            if (lane < q) uu = fma(-ts, rk, uu);
            uuq += ts;
            if (zfree && ts == t2) {
                // at most 3 independent faces per leg-step, so q <= 60 in exact arithmetic; the cap keeps
                // R^-1 (packed, 64 columns) and the Givens buffer inside their LDS regions regardless
                if (q >= 3 * DENSE_MAX_LS) {
                    ok = false;
                    break;
                }
                // ---- add p: Householder on J's columns q.. so that d2 -> |d2| e_q ----
                const double nrm = sqrt(dd2);
                if (tail > 0.0) {
                    const double dq = readlane_f64(dc, q);
                    const double v0 = dq <= 0.0 ? dq - nrm : -tail / (dq + nrm);
                    const double beta = 2.0 / (v0 * v0 + tail);
                    G.hv[lane] = lane > q ? dc : lane == q ? v0 : 0.0;
                    LMPC_SYNC();
                    const double w = beta * row_dot(Jr, G.hv);
                    row_axpy(Jr, w, G.hv);
                }
                // R^-1 column q = (-r / |d2|, 1 / |d2|)
                const double inrm = 1.0 / nrm;
                if (lane <= q) Ri[roff(q) + lane] = lane < q ? -rk * inrm : inrm;
                if (lane == q) {
                    actc = p;
                    uu = uuq;
                }
                if (lane == bp) lact |= 1 << fp;
                ++q;
                LMPC_SYNC();
                GSTAMP(5);  // step + add
                break;
            }
            // ---- drop the blocking constraint (partial step, or n_p dependent on the active normals) ----
            ++ndrop;
            const unsigned long long lm = __ballot(lane < q && cand == t1);
            const int lpos = (int)__builtin_ctzll(lm);
            {
                const int ida = __builtin_amdgcn_readlane(actc, lpos);
                const int ba = ida / 5;
                if (lane == ba) lact &= ~(1 << (ida - 5 * ba));
            }
            // slots above lpos move down one
            {
                const int src = lane + 1 < 64 ? lane + 1 : 63;
                const double uun = __shfl(uu, src);
                const int actn = __shfl(actc, src);
                if (lane >= lpos) {
                    uu = uun;
                    actc = actn;
                }
            }
            // rotations on column pairs (j, j+1), j = lpos..q-2, that zero row lpos of R^-1 (a scalar
            // chain: every lane computes the same (c, s); lane 0 publishes them).  Loads are
            // unconditional from clamped addresses (no exec-mask branches); a group of 8 is loaded first.
            const int jn = q - 1 - lpos;  // number of rotations
            {
                double carry = Ri[roff(lpos) + lpos];
                for (int j0 = 0; j0 < jn; j0 += 8) {
                    double bj[8];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = lpos + j0 + jj;
                        bj[jj] = Ri[roff(j < q - 1 ? j + 1 : q - 1) + lpos];
                    }
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = lpos + j0 + jj;
                        const bool on = j0 + jj < jn;
                        const double b = on ? bj[jj] : 0.0;
                        const double h2 = fma(carry, carry, b * b);
                        const double ih = h2 > 0.0 ? rsq_nr(h2) : 0.0;
                        const double cg = h2 > 0.0 ? b * ih : 1.0, sg = -carry * ih;
                        if (on && lane == 0) {
                            d2v w2;
                            w2.x = cg;
                            w2.y = sg;
                            ((ld2*)G.gcs)[j] = w2;
                        }
                        carry = on ? h2 * ih : carry;
                    }
                }
            }
            LMPC_SYNC();
            // the rotations on the columns of R^-1: lane k = row k, carried through the pairs
            {
                const ld2* gc2 = (const ld2*)G.gcs;
                double carry = Ri[roff(lpos) + (lane <= lpos ? lane : 0)];
                carry = lane <= lpos ? carry : 0.0;
                for (int j0 = 0; j0 < jn; j0 += 8) {
                    double bj[8];
                    d2v cs[8];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = lpos + j0 + jj;
                        const int jc = j < q - 1 ? j + 1 : q - 1;
                        const double v = Ri[roff(jc) + (lane <= jc ? lane : 0)];
                        bj[jj] = lane <= jc ? v : 0.0;
                        cs[jj] = gc2[j < 63 ? j : 62];
                    }
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = lpos + j0 + jj;
                        if (j0 + jj >= jn) break;
                        const double nj = fma(cs[jj].x, carry, cs[jj].y * bj[jj]);
                        if (lane <= j + 1) Ri[roff(j) + lane] = nj;
                        carry = fma(-cs[jj].y, carry, cs[jj].x * bj[jj]);
                    }
                }
            }
            LMPC_SYNC();
            // delete row lpos of R^-1 (rows below move up; column c keeps rows 0..c), 8 columns per group
            for (int c0 = lpos; c0 < q - 1; c0 += 8) {
                double v[8];
                const bool lk = lane >= lpos;
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const int c = c0 + cc < q - 1 ? c0 + cc : q - 2;
                    v[cc] = Ri[roff(c) + (lane <= c ? lane + 1 : 0)];
                }
                LMPC_SYNC();  // lane k-1 reads what lane k overwrites: no store may move above these loads
#pragma unroll
                for (int cc = 0; cc < 8; ++cc) {
                    const int c = c0 + cc;
                    if (c < q - 1 && lk && lane <= c) Ri[roff(c) + lane] = v[cc];
                }
            }
            // the same rotations on J's columns: one carried sweep over the 8-column chunks that meet
            // [lpos, q-1] (uniform branch per chunk), identity rotations elsewhere in those chunks
            {
                const int jlo = lpos, jhi = q - 2;
                const ld2* gc2 = (const ld2*)G.gcs;
#pragma unroll
                for (int j0 = 0; j0 < 63; j0 += 8) {
                    if (j0 + 7 < jlo || j0 > jhi) continue;
                    d2v cs[8];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) cs[jj] = gc2[j0 + jj < 63 ? j0 + jj : 62];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int j = j0 + jj;
                        if (j >= 63) continue;
                        const bool on = j >= jlo && j <= jhi;
                        const double cg = on ? cs[jj].x : 1.0, sg = on ? cs[jj].y : 0.0;
                        const double a = Jr[j], b = Jr[j + 1];
                        Jr[j] = pin(fma(cg, a, sg * b));
                        Jr[j + 1] = pin(fma(-sg, a, cg * b));
                    }
                    GI_CHUNK_FENCE();
                }
            }
            --q;
            // constraint value of p at the (possibly moved) x
            {
                const double u0 = readlane_f64(xv, vp), u1 = readlane_f64(xv, vp + 1), u2 = readlane_f64(xv, vp + 2);
                sp = face_val(fp, u0, u1, u2, mu, fzmax);
            }
            LMPC_SYNC();
            GSTAMP(6);  // step + drop
        }
        if (!ok) break;
    }
    if (!__builtin_amdgcn_readfirstlane((int)ok) || !__all(xv == xv)) {
        if (lane == 0) done[qp] = 0;  // the Riccati kernel solves this QP
        GSTAMP_FLUSH(qp);
        return;
    }
    // ---- KKT certificate, independent of the active-set algebra (J, R^-1, the multipliers uu): the gradient
    //      H x + g from the condensed QP itself (its tiles and g rebuilt: R^-1 overwrote them), then per stance
    //      leg-step primal feasibility, the least-squares multipliers of its active faces (sign) and the stationarity
    //      residual on its free directions; the apex by the cone test.  A QP that fails it is left to the Riccati
    //      kernel, like one that hits the step cap ----
    {
        LMPC_SYNC();
        dense_condense<TERRAIN>(prm, S, H, nls, smask, lane);
        S.vec2[lane] = xv;
        LMPC_SYNC();
        const double gl = h_matvec(S, S.vec2, S.scr, lane) + S.gv[lane];
        LMPC_SYNC();
        S.vec[lane] = gl;
        LMPC_SYNC();
        double g[3] = {0.0, 0.0, 0.0}, u[3] = {0.0, 0.0, 0.0};
        double gloc = 1.0;
        if (lane < nls) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                g[p] = S.vec[lv0 + p];
                u[p] = S.vec2[lv0 + p];
                gloc = fmax(gloc, fabs(g[p]));
            }
        }
        const double gscale = wave_max(gloc);
        double sres = 0.0;
        bool fail = false;
        if (lane < nls) {
            double o[5];
            cons_resid(u, mu, fzmax, o);
#pragma unroll
            for (int i = 0; i < 5; ++i) fail |= o[i] > prm.tol_p * fzmax;
            if ((lact & 3) == 3 || (lact & 12) == 12) {  // apex (f = 0): the cone test
                fail |= g[2] / mu < fabs(g[0]) + fabs(g[1]) - prm.tol_d * gscale;
            } else {
                const LegKkt kk = leg_kkt(lact, g, mu, -prm.tol_d * gscale);
                fail |= kk.drop >= 0;
                sres = kk.res;
            }
        }
        const double sr = wave_max(sres);
#ifdef LMPC_KKT_DIAG
        if (lane == 0 && qp < LMPC_KKT_DIAG_QPS) {
            lmpc_kkt_diag_gi[qp][0] = sr / gscale;
            lmpc_kkt_diag_gi[qp][1] = __any(fail) ? 1.0 : 0.0;
            lmpc_kkt_diag_gi[qp][2] = gscale;
            lmpc_kkt_diag_gi[qp][3] = 1.0;
        }
#endif
#ifndef LMPC_KKT_OFF
        if (__any(fail) || !(sr <= prm.tol_d * gscale)) {
            if (lane == 0) done[qp] = 0;  // the Riccati kernel solves this QP
            GSTAMP_FLUSH(qp);
            return;
        }
#endif
        LMPC_SYNC();
    }
    // ---- output: stance forces through LDS to the lane of leg-step 4k + j ----
    S.vec[lane] = xv;
    LMPC_SYNC();
    double fo[3] = {0.0, 0.0, 0.0};
    if (lane < nls) {
        const double u0 = S.vec[lv0], u1 = S.vec[lv0 + 1], u2 = S.vec[lv0 + 2];
        fo[0] = u0;
        fo[1] = u1;
        fo[2] = u2;
        if constexpr (TERRAIN) {
            const int lj = S.lsm[lane] & 3;
            const ldouble* Rj = S.tf + 9 * lj;
#pragma unroll
            for (int pp = 0; pp < 3; ++pp) fo[pp] = Rj[3 * pp] * u0 + Rj[3 * pp + 1] * u1 + Rj[3 * pp + 2] * u2;
        }
    }
    LMPC_SYNC();
    if (lane < nls) {
#pragma unroll
        for (int pp = 0; pp < 3; ++pp) S.vec2[3 * lane + pp] = fo[pp];
    }
    LMPC_SYNC();
    double* gout = grf + (size_t)qp * 12 * H;
    if (lane < 4 * H) {
#pragma unroll
        for (int pp = 0; pp < 3; ++pp) gout[3 * lane + pp] = stl ? S.vec2[3 * rank + pp] : 0.0;
    }
    if (lane == 0) {
        if (status) status[qp] = LMPC_QP_CONVERGED;
        if (iters) iters[qp] = it | (ndrop << 16);  // active-set steps | drops
        done[qp] = 1;
    }
    GSTAMP(7);  // output
    GSTAMP_FLUSH(qp);
}

template __global__ void lmpc_gi_kernel<false>(const DevParams, const double*, const uint8_t*, const double*, int,
                                               double*, int32_t*, int32_t*, uint8_t*);
template __global__ void lmpc_gi_kernel<true>(const DevParams, const double*, const uint8_t*, const double*, int,
                                              double*, int32_t*, int32_t*, uint8_t*);

#ifdef LMPC_STAMPS
extern "C" int lmpc_debug_gi_stamps(unsigned long long* out, int nqp) {
    if (nqp > 4096) nqp = 4096;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(lmpc_gi_stamps), (size_t)nqp * 8 * sizeof(unsigned long long)) ==
                   hipSuccess ? nqp : -1;
}
#endif

size_t gi_lds_bytes(int H) {
    return dense_lds_bytes(H) + (size_t)GI_EXTRA * sizeof(double);
}

hipError_t launch_gi(const DevParams& prm, const double* rec, const uint8_t* contact, const double* normals,
                     int batch, double* grf, int32_t* status, int32_t* iters, uint8_t* done, hipStream_t stream) {
    const size_t lds = gi_lds_bytes(prm.H);
    const dim3 grid(batch), block(LMPC_WAVE);
    if (normals) {
        (void)hipFuncSetAttribute((const void*)lmpc_gi_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_gi_kernel<true>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_gi_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL(lmpc_gi_kernel<false>, grid, block, lds, stream, prm, rec, contact, normals, batch, grf,
                           status, iters, done);
    }
    return hipGetLastError();
}

}  // namespace lmpc

// lmpc_kernel_common.h -- device helpers shared by the two QP kernels (lmpc_kernels.hip: the
// Riccati path; lmpc_dense.hip: the condensed dense path): wave-scope LDS ordering, DPP wave
// reductions, fp64 reciprocal / rsqrt with Newton refinement, the friction-pyramid rows
// (ConvexQPSolver.cpp:131-172) and the per-leg null-space basis of the active-set polish.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace lmpc {

// One workgroup = one wavefront (blockDim 64, __launch_bounds__(64)): cross-lane exchange through LDS
// needs only wavefront-scope ordering -- LDS operations of one wave are performed in order -- so the
// "barrier" is a release/acquire fence pair at wavefront scope around a code-motion barrier.  Unlike
// __syncthreads() it emits no s_waitcnt lgkmcnt(0): loads issued ahead (prefetches) stay in flight.
constexpr int LMPC_WAVE = 64;
// interior point: fraction of the step to the boundary (tools/variant_sweep.py builds other values)
#ifndef LMPC_STEP_FRAC
#define LMPC_STEP_FRAC 0.99
#endif
// Hand-over to the polish: a face is guessed active where z > LMPC_ACT_RATIO * s.  At the hand-over
// (mean complementarity tol_mu, default 1e-4) an active face has z/s ~ z^2/mu >> 1 and an inactive one ~ mu/s^2 << 1; the
// faces in between are near-degenerate, and guessing them active costs fewer polish rounds than guessing
// them inactive (a wrong active face leaves in the same round a missing one would enter; missing faces
// enter one per leg-step per round).  numpy replica (tools/polish_guess_proto.py, 1280 config-2 QPs):
// 1.91 -> 1.13 polish rounds per QP at 1e-3 against the z > s rule.
// Corrector step: separate primal (f, s) and dual (z) step lengths, each LMPC_STEP_FRAC of its distance to the
// boundary (0: one common step).  numpy replica (tools/polish_guess_proto.py, 512 config-2 QPs at the 1e-5
// hand-over): 6.49 -> 6.09 interior-point iterations per QP, modelled slowest QP -8 %.
#ifndef LMPC_SPLIT_STEP
#define LMPC_SPLIT_STEP 1
#endif
#ifndef LMPC_ACT_RATIO
#define LMPC_ACT_RATIO 1e-3
#endif
// diagnostic builds only (-DLMPC_KKT_DIAG, -DLMPC_REFINE_DIAG): per-QP certificate residuals kept for this many QPs
#if defined(LMPC_KKT_DIAG) || defined(LMPC_REFINE_DIAG)
#define LMPC_KKT_DIAG_QPS 65536
#endif
#define LMPC_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

// LMPC_SYNC that also orders the wave's global (per-QP scratch) stores before its later loads of the
// same words by other lanes (workgroup scope = s_waitcnt vmcnt(0) here: one wave per workgroup)
#define LMPC_GSYNC()                                             \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   \
    } while (0)

// Explicit LDS address space: every shared access compiles to ds_read/ds_write
// (a generic pointer would fall back to flat_load/flat_store).
typedef __attribute__((address_space(3))) double ldouble;
// Explicit global address space for the per-QP scratch (outlined functions would otherwise use flat ops).
typedef __attribute__((address_space(1))) double gdouble;

// ---- wave reductions without LDS: DPP inside 16-lane rows, readlane across the 4 rows ----
// Every DPP move here has old = 0, so bound_ctrl (an invalid source lane reads 0) gives the same value as keeping
// old; with it set the compiler drops the v_mov that initialises old (-300 instructions in the two-wave Riccati
// kernel, 1-2 % on configs 2-5)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
constexpr int DPP_QP_1032 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_QP_2301 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int DPP_ROR4 = 0x124;    // row_ror:4
constexpr int DPP_ROR8 = 0x128;    // row_ror:8
struct OpSum { __device__ static double f(double a, double b) { return a + b; } };
struct OpMin { __device__ static double f(double a, double b) { return fmin(a, b); } };
struct OpMax { __device__ static double f(double a, double b) { return fmax(a, b); } };
template <class Op>
__device__ __forceinline__ double wave_reduce(double v) {
    v = Op::f(v, dpp_f64<DPP_QP_1032>(v));
    v = Op::f(v, dpp_f64<DPP_QP_2301>(v));
    v = Op::f(v, dpp_f64<DPP_ROR4>(v));
    v = Op::f(v, dpp_f64<DPP_ROR8>(v));  // every lane holds its row's result
    return Op::f(Op::f(readlane_f64(v, 0), readlane_f64(v, 16)), Op::f(readlane_f64(v, 32), readlane_f64(v, 48)));
}
__device__ __forceinline__ double wave_sum(double v) { return wave_reduce<OpSum>(v); }
__device__ __forceinline__ double wave_min(double v) { return wave_reduce<OpMin>(v); }
__device__ __forceinline__ double wave_max(double v) { return wave_reduce<OpMax>(v); }
// sum over the 4 lanes of a stage (lanes 4q..4q+3 = legs of one stage)
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_f64<DPP_QP_1032>(v);
    v += dpp_f64<DPP_QP_2301>(v);
    return v;
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

// Interior-point stop of retry attempt `att` (>= 1) after a polish that did not verify: 1e-3 tighter than the
// previous attempt's, and never looser than a fixed floor (1e-8 for the second attempt, 1e-12 for the third, 1e-4
// lower each further one), so the last attempt's iterate is as converged as before the default hand-over moved to
// 1e-4 (round 3).  Shared by every kernel's retry ladder; lmpc.h (lmpc_options.max_attempts) documents it.
__device__ __forceinline__ double retry_tol(double tol, int att) {
    double floor = 1e-8;
    for (int a = 1; a < att; ++a) floor *= 1e-4;
    return fmin(tol * 1e-3, floor);
}

// 1/sqrt(x): hardware estimate + one Newton step (cheaper than the correctly-rounded sqrt + divide).
__device__ __forceinline__ double rsq_nr(double x) {
    // v_rsq_f64 is good to 2^-24 on gfx950 (tools/ubench/rsq_acc.hip); one Newton step -> ~4e-15
    double y = __builtin_amdgcn_rsq(x);
    y = y * fma(-0.5 * x * y, y, 1.5);
    return y;
}

// 1/x to full fp64 precision: hardware estimate + two Newton steps
__device__ __forceinline__ double rcp_nr(double x) {
    double y = __builtin_amdgcn_rcp(x);
    y = fma(y, fma(-x, y, 1.0), y);
    y = fma(y, fma(-x, y, 1.0), y);
    return y;
}

typedef double d4 __attribute__((ext_vector_type(4)));
#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)


// Up to three active faces of a leg-step, in face order (slot k: face index, 7 = unused slot).
// Everything below is statically indexed over 3 slots (a dynamically indexed per-lane array is
// placed in scratch memory: 30+ scratch round trips per polish round in both QP kernels).
struct ActiveRows {
    int i0, i1, i2, nr;
};
__device__ __forceinline__ ActiveRows active_rows(int act) {
    ActiveRows r;
    int m = act & 31;
    r.i0 = m ? __builtin_ctz(m) : 7;
    m &= m - 1;
    r.i1 = m ? __builtin_ctz(m) : 7;
    m &= m - 1;
    r.i2 = m ? __builtin_ctz(m) : 7;
    r.nr = (r.i0 < 5) + (r.i1 < 5) + (r.i2 < 5);
    return r;
}

// Null-space parametrisation of one leg-step for active set `act` (bit i = row ci):
// f = up + T y, T columns orthonormal.  Returns true at the pyramid apex (f = 0).
__device__ __forceinline__ bool leg_basis(int act, double mu, double fzmax, double T[9], double up[3]) {
#pragma unroll
    for (int i = 0; i < 9; ++i) T[i] = 0.0;
    up[0] = up[1] = up[2] = 0.0;
    if ((act & 3) == 3 || (act & 12) == 12) return true;
    const ActiveRows ar = active_rows(act);
    const int nr = ar.nr;
    double r0[3], r1[3], r2[3];
    cons_rowvec(ar.i0, mu, r0);
    cons_rowvec(ar.i1, mu, r1);
    cons_rowvec(ar.i2, mu, r2);
    const double b0 = ar.i0 == 4 ? fzmax : 0.0, b1 = ar.i1 == 4 ? fzmax : 0.0, b2 = ar.i2 == 4 ? fzmax : 0.0;
    // Gram-Schmidt (slots beyond nr are computed on dummy rows and never used)
    double q0[3], q1[3], q2[3];
    {
        const double n = 1.0 / sqrt(r0[0] * r0[0] + r0[1] * r0[1] + r0[2] * r0[2]);
        q0[0] = r0[0] * n;
        q0[1] = r0[1] * n;
        q0[2] = r0[2] * n;
    }
    {
        double v[3] = {r1[0], r1[1], r1[2]};
        const double d = q0[0] * v[0] + q0[1] * v[1] + q0[2] * v[2];
        v[0] -= d * q0[0];
        v[1] -= d * q0[1];
        v[2] -= d * q0[2];
        const double n = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        q1[0] = v[0] * n;
        q1[1] = v[1] * n;
        q1[2] = v[2] * n;
    }
    {
        double v[3] = {r2[0], r2[1], r2[2]};
        double d = q0[0] * v[0] + q0[1] * v[1] + q0[2] * v[2];
        v[0] -= d * q0[0];
        v[1] -= d * q0[1];
        v[2] -= d * q0[2];
        d = q1[0] * v[0] + q1[1] * v[1] + q1[2] * v[2];
        v[0] -= d * q1[0];
        v[1] -= d * q1[1];
        v[2] -= d * q1[2];
        const double n = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        q2[0] = v[0] * n;
        q2[1] = v[1] * n;
        q2[2] = v[2] * n;
    }
    // particular solution up = sum_a beta_a q_a with rows_a . up = b_a
    if (nr >= 1) {
        const double beta0 = b0 / (r0[0] * q0[0] + r0[1] * q0[1] + r0[2] * q0[2]);
        double beta1 = 0.0, beta2 = 0.0;
        if (nr >= 2) {
            const double s1 = b1 - (r1[0] * q0[0] + r1[1] * q0[1] + r1[2] * q0[2]) * beta0;
            beta1 = s1 / (r1[0] * q1[0] + r1[1] * q1[1] + r1[2] * q1[2]);
        }
        if (nr >= 3) {
            const double s2 = b2 - (r2[0] * q0[0] + r2[1] * q0[1] + r2[2] * q0[2]) * beta0 -
                              (r2[0] * q1[0] + r2[1] * q1[1] + r2[2] * q1[2]) * beta1;
            beta2 = s2 / (r2[0] * q2[0] + r2[1] * q2[1] + r2[2] * q2[2]);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) up[i] = beta0 * q0[i] + (nr >= 2 ? beta1 * q1[i] : 0.0) + (nr >= 3 ? beta2 * q2[i] : 0.0);
    }
    if (nr == 0) {
        T[0] = T[4] = T[8] = 1.0;
    } else if (nr == 1) {
        const double* n = q0;
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
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            T[i * 3 + 0] = t1[i];
            T[i * 3 + 1] = t2[i];
        }
    } else if (nr == 2) {
        double t[3] = {q0[1] * q1[2] - q0[2] * q1[1], q0[2] * q1[0] - q0[0] * q1[2], q0[0] * q1[1] - q0[1] * q1[0]};
        const double in = 1.0 / sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
#pragma unroll
        for (int i = 0; i < 3; ++i) T[i * 3 + 0] = t[i] * in;
    }
    return false;
}

// KKT certificate of one (non-apex) stance leg-step with active faces `act` (ConvexQPSolver.cpp:131-172 rows) at the
// gradient g = dJ/df of the leg's force: the least-squares multipliers z of C_S' z = -g (C_S = the <= 3 active rows,
// full row rank; none when act = 0), by Gaussian elimination on the Gram matrix C_S C_S' padded to 3x3 with
// identity rows.  `drop`: the face whose multiplier is the most negative below zmin (the one to drop), or -1.
// `res`: the stationarity residual |g + C_S' z|_inf -- the part of g on the leg's free directions (the null space of
// C_S), which the polish's equality-constrained solve makes zero: a verified active set must also have res at
// rounding level, or the returned forces are not the optimum whatever the multiplier signs say.
struct LegKkt {
    int drop;
    double res;
};
__device__ __forceinline__ LegKkt leg_kkt(int act, const double g[3], double mu, double zmin) {
    const ActiveRows ar = active_rows(act);
    const int nr = ar.nr;
    double C[3][3];
    cons_rowvec(ar.i0, mu, C[0]);
    cons_rowvec(ar.i1, mu, C[1]);
    cons_rowvec(ar.i2, mu, C[2]);
    double Gm[3][3], rhs[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        rhs[a] = a < nr ? -(C[a][0] * g[0] + C[a][1] * g[1] + C[a][2] * g[2]) : 0.0;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const double v = C[a][0] * C[b][0] + C[a][1] * C[b][1] + C[a][2] * C[b][2];
            Gm[a][b] = (a < nr && b < nr) ? v : (a == b ? 1.0 : 0.0);
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int b = a + 1; b < 3; ++b) {
            const double fct = Gm[b][a] / Gm[a][a];
#pragma unroll
            for (int c = a; c < 3; ++c) Gm[b][c] -= fct * Gm[a][c];
            rhs[b] -= fct * rhs[a];
        }
    }
    double zz[3];
#pragma unroll
    for (int a = 2; a >= 0; --a) {
        double v = rhs[a];
#pragma unroll
        for (int b = a + 1; b < 3; ++b) v -= Gm[a][b] * zz[b];
        zz[a] = v / Gm[a][a];
    }
    LegKkt o;
    o.drop = -1;
    double zm = zmin;
    const int fi[3] = {ar.i0, ar.i1, ar.i2};
#pragma unroll
    for (int a = 0; a < 3; ++a)
        if (a < nr && zz[a] < zm) {
            zm = zz[a];
            o.drop = fi[a];
        }
    // r = g + C_S' z (slots beyond nr carry z = 0 from the padded rows)
    o.res = 0.0;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        double r = g[p];
#pragma unroll
        for (int a = 0; a < 3; ++a) r += (a < nr ? zz[a] : 0.0) * C[a][p];
        o.res = fmax(o.res, fabs(r));
    }
    return o;
}

// Polish verification of one (non-apex) leg-step: the face to drop (leg_kkt without the residual).
__device__ __forceinline__ int leg_drop_face(int act, const double g[3], double mu, double zmin) {
    const ActiveRows ar = active_rows(act);
    const int nr = ar.nr;
    double C[3][3];
    cons_rowvec(ar.i0, mu, C[0]);
    cons_rowvec(ar.i1, mu, C[1]);
    cons_rowvec(ar.i2, mu, C[2]);
    double Gm[3][3], rhs[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        rhs[a] = a < nr ? -(C[a][0] * g[0] + C[a][1] * g[1] + C[a][2] * g[2]) : 0.0;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const double v = C[a][0] * C[b][0] + C[a][1] * C[b][1] + C[a][2] * C[b][2];
            Gm[a][b] = (a < nr && b < nr) ? v : (a == b ? 1.0 : 0.0);
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int b = a + 1; b < 3; ++b) {
            const double fct = Gm[b][a] / Gm[a][a];
#pragma unroll
            for (int c = a; c < 3; ++c) Gm[b][c] -= fct * Gm[a][c];
            rhs[b] -= fct * rhs[a];
        }
    }
    double zz[3];
#pragma unroll
    for (int a = 2; a >= 0; --a) {
        double v = rhs[a];
#pragma unroll
        for (int b = a + 1; b < 3; ++b) v -= Gm[a][b] * zz[b];
        zz[a] = v / Gm[a][a];
    }
    int face = -1;
    double zm = zmin;
    const int fi[3] = {ar.i0, ar.i1, ar.i2};
#pragma unroll
    for (int a = 0; a < 3; ++a)
        if (a < nr && zz[a] < zm) {
            zm = zz[a];
            face = fi[a];
        }
    return face;
}

}  // namespace lmpc

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
//      Newton step is an LQR Riccati recursion over the horizon (state
//      elimination by dynamic programming = condensation done stage-wise,
//      O(H * 12^3) instead of O((12H)^3)); swing legs are eliminated exactly;
//   4. polishes: takes the IPM active set, re-solves the equality-constrained
//      LQR exactly (per-leg null-space parametrisation), verifies primal
//      feasibility and multiplier signs, adjusts and repeats if needed
//      (a dual active-set refinement), so the result is the exact optimum;
//   5. writes u_0..u_{H-1} (world frame GRFs) -- grf[0..11] is what the
//      reference's compute_grfs returns (ConvexQPSolver.cpp:314-327).
//
// All arithmetic is fp64 (the QP has cond(H_c) ~ 4e4..6e5 and IPM systems far
// worse; fp32 cannot meet the 1e-4 parity bar).  The bound is FP64 VALU
// latency/throughput, not HBM: each QP moves ~2.2 KB (H=10) over HBM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"
#include "lmpc_device.h"

namespace lmpc {

#define LMPC_SYNC() __syncthreads()

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

// ---- friction pyramid, flat ground (ConvexQPSolver.cpp:131-172) -----------
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
// C' w
__device__ __forceinline__ void cons_tw(const double w[5], double mu, double o[3]) {
    o[0] = -w[0] + w[1];
    o[1] = -w[2] + w[3];
    o[2] = -mu * (w[0] + w[1] + w[2] + w[3]) + w[4];
}

// ---- per-stage LDS records -----------------------------------------------
// leg record (24 doubles): Rt[9] (input Hessian block, f coords) | rt[3] | T[9] (f = up + T y) | up[3]
constexpr int LR_RT = 0, LR_LIN = 9, LR_T = 12, LR_UP = 21, LR_SIZE = 24;

struct Smem {
    double* G0;   // 6 x 12
    double* cs;   // H x (cos, sin) of yaw_ref
    double* xr;   // H x 12 reference states
    double* hdr;  // x0(12) R(9) feet(12)
    double* LR;   // 4H leg records
    double* Yk;   // H x 144   Y_k = L_k^-1 Gux_k (column-major)
    double* Li;   // H x 144   L_k^-1 (column-major)
    double* vk;   // H x 12    P_{k+1} d_k
    double* yk;   // H x 12    L_k^-1 gu_k (vector pass) / gradient (adjoint)
    double* uk;   // H x 12    inputs
    double* xk;   // (H+1) x 12 states
    double* P;    // 144
    double* PB;   // 144
    double* W1;   // 144
    double* col;  // 16
    double* vec;  // 64
};

__device__ __forceinline__ Smem carve(double* sm, int H) {
    Smem s;
    double* p = sm;
    s.G0 = p; p += 72;
    s.cs = p; p += 2 * H;
    s.xr = p; p += 12 * H;
    s.hdr = p; p += 40;
    s.LR = p; p += 96 * H;
    s.Yk = p; p += 144 * H;
    s.Li = p; p += 144 * H;
    s.vk = p; p += 12 * H;
    s.yk = p; p += 12 * H;
    s.uk = p; p += 12 * H;
    s.xk = p; p += 12 * (H + 1);
    s.P = p; p += 144;
    s.PB = p; p += 144;
    s.W1 = p; p += 144;
    s.col = p; p += 16;
    s.vec = p; p += 64;
    return s;
}

// M(yaw) = [c s 0; -s c 0; 0 0 1]  (ang_vel_to_rpy_rate, ConvexQPSolver.cpp:220-222)
__device__ __forceinline__ double Myaw(double c, double s, int i, int j) {
    if (i == 2) return j == 2 ? 1.0 : 0.0;
    if (j == 2) return 0.0;
    if (i == 0) return j == 0 ? c : s;
    return j == 0 ? -s : c;
}

// ---------------------------------------------------------------------------
// Riccati factorisation (backward pass, matrix part).
// Per stage k, input u_k = up_k + T_k y_k (per-leg blocks), stage Hessian
// T'Rt T, B_k = B T_k.  Stores Y_k = L_k^-1 Gux_k, Linv_k and v_k = P_{k+1} d_k.
// ---------------------------------------------------------------------------
__device__ void riccati_factor(const DevParams& prm, const Smem& S, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    for (int e = lane; e < 144; e += 64) {
        const int r = e / 12, c = e % 12;
        S.P[e] = (r == c) ? prm.q[r] : 0.0;
    }
    LMPC_SYNC();
    for (int k = H - 1; k >= 0; --k) {
        const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
        const double* lr = S.LR + k * 4 * LR_SIZE;
        // Bt = G0 T_k (6x12) -> W1 ; G0 up_k -> vec[0..5]
        for (int e = lane; e < 72; e += 64) {
            const int r = e / 12, c = e % 12, j = c / 3, cc = c % 3;
            const double* T = lr + j * LR_SIZE + LR_T;
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 3; ++m) v += S.G0[r * 12 + 3 * j + m] * T[m * 3 + cc];
            S.W1[e] = v;
        }
        if (lane < 6) {
            double v = 0.0;
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int m = 0; m < 3; ++m) v += S.G0[lane * 12 + 3 * j + m] * lr[j * LR_SIZE + LR_UP + m];
            S.vec[lane] = v;
        }
        LMPC_SYNC();
        // PB = P[:, 6:12] Bt (12x12);  v_k = P d_k with d_k = [0; G0 up] - g dt e11
        if (lane < 48) {
            const int r = lane >> 2, cg = lane & 3;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int c = 3 * cg + i;
                double v = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) v += S.P[r * 12 + 6 + m] * S.W1[m * 12 + c];
                S.PB[r * 12 + c] = v;
            }
        } else if (lane < 60) {
            const int r = lane - 48;
            double v = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) {
                const double d = S.vec[m] + (m == 5 ? -prm.grav * dt : 0.0);
                v += S.P[r * 12 + 6 + m] * d;
            }
            S.vk[k * 12 + r] = v;
        }
        LMPC_SYNC();
        // augmented column per lane: [Guu | Gux | I]
        double a[12];
        if (lane < 12) {
            const int c = lane, j = c / 3, cc = c % 3;
            const double* T = lr + j * LR_SIZE + LR_T;
            const double* Rt = lr + j * LR_SIZE + LR_RT;
            const bool fixed = (T[cc] == 0.0 && T[3 + cc] == 0.0 && T[6 + cc] == 0.0);
#pragma unroll
            for (int r = 0; r < 12; ++r) {
                double v = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) v += S.W1[m * 12 + r] * S.PB[(6 + m) * 12 + c];
                if (r / 3 == j) {
                    const int rr = r % 3;
                    double t = 0.0;
#pragma unroll
                    for (int p = 0; p < 3; ++p)
#pragma unroll
                        for (int q = 0; q < 3; ++q) t += T[p * 3 + rr] * Rt[p * 3 + q] * T[q * 3 + cc];
                    v += t;
                }
                a[r] = v;
            }
            if (fixed) {
#pragma unroll
                for (int r = 0; r < 12; ++r) a[r] = (r == c) ? 1.0 : 0.0;
            }
        } else if (lane < 24) {
            const int c = lane - 12;
#pragma unroll
            for (int r = 0; r < 12; ++r) {
                double v = S.PB[c * 12 + r];
                if (c >= 6 && c < 9) {
                    double t = 0.0;
#pragma unroll
                    for (int i = 0; i < 3; ++i) t += S.PB[i * 12 + r] * Myaw(ck, sk, i, c - 6);
                    v += dt * t;
                } else if (c >= 9) {
                    v += dt * S.PB[(c - 6) * 12 + r];
                }
                a[r] = v;
            }
        } else if (lane < 36) {
#pragma unroll
            for (int r = 0; r < 12; ++r) a[r] = (r == lane - 24) ? 1.0 : 0.0;
        } else {
#pragma unroll
            for (int r = 0; r < 12; ++r) a[r] = 0.0;
        }
        // right-looking Cholesky on Guu applied to the whole augmented row block:
        // afterwards lane c holds column c of L^-1 [Guu | Gux | I] = [L' | Y | Linv]
#pragma unroll
        for (int jj = 0; jj < 12; ++jj) {
            if (lane == jj) {
                const double d = a[jj];
                const double piv = (d > 1e-280) ? sqrt(d) : 1e140;  // dead direction -> frozen
                const double inv = 1.0 / piv;
#pragma unroll
                for (int r = 0; r < 12; ++r) S.col[r] = (r > jj) ? a[r] * inv : 0.0;
                S.col[jj] = piv;
            }
            LMPC_SYNC();
            double l[12];
#pragma unroll
            for (int r = 0; r < 12; ++r) l[r] = S.col[r];
            const double t = a[jj] / l[jj];
            a[jj] = t;
#pragma unroll
            for (int r = jj + 1; r < 12; ++r) a[r] -= l[r] * t;
            LMPC_SYNC();
        }
        if (lane >= 12 && lane < 24) {
#pragma unroll
            for (int r = 0; r < 12; ++r) S.Yk[k * 144 + (lane - 12) * 12 + r] = a[r];
        } else if (lane >= 24 && lane < 36) {
#pragma unroll
            for (int r = 0; r < 12; ++r) S.Li[k * 144 + (lane - 24) * 12 + r] = a[r];
        }
        LMPC_SYNC();
        if (k > 0) {
            // PA = P (I + dt N_k) -> PB
            if (lane < 48) {
                const int r = lane >> 2, cg = lane & 3;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int c = 3 * cg + i;
                    double v = S.P[r * 12 + c];
                    if (c >= 6 && c < 9) {
                        double t = 0.0;
#pragma unroll
                        for (int m = 0; m < 3; ++m) t += S.P[r * 12 + m] * Myaw(ck, sk, m, c - 6);
                        v += dt * t;
                    } else if (c >= 9) {
                        v += dt * S.P[r * 12 + c - 6];
                    }
                    S.PB[r * 12 + c] = v;
                }
            }
            LMPC_SYNC();
            // P_k = Q + (I + dt N')PA - Y'Y
            if (lane < 48) {
                const int r = lane >> 2, cg = lane & 3;
                const double* Y = S.Yk + k * 144;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const int c = 3 * cg + i;
                    double v = S.PB[r * 12 + c];
                    if (r >= 6 && r < 9) {
                        double t = 0.0;
#pragma unroll
                        for (int m = 0; m < 3; ++m) t += Myaw(ck, sk, m, r - 6) * S.PB[m * 12 + c];
                        v += dt * t;
                    } else if (r >= 9) {
                        v += dt * S.PB[(r - 6) * 12 + c];
                    }
                    if (r == c) v += prm.q[r];
                    double yy = 0.0;
#pragma unroll
                    for (int m = 0; m < 12; ++m) yy += Y[r * 12 + m] * Y[c * 12 + m];
                    S.W1[r * 12 + c] = v - yy;
                }
            }
            LMPC_SYNC();
            // symmetrise into P
            for (int e = lane; e < 144; e += 64) {
                const int r = e / 12, c = e % 12;
                S.P[e] = 0.5 * (S.W1[r * 12 + c] + S.W1[c * 12 + r]);
            }
            LMPC_SYNC();
        }
    }
}

// ---------------------------------------------------------------------------
// Vector pass: backward affine recursion + forward rollout.  Produces u_k
// (S.uk) and, if store_x, the state trajectory (S.xk).
// ---------------------------------------------------------------------------
__device__ void riccati_solve(const DevParams& prm, const Smem& S, int lane, bool store_x) {
    const int H = prm.H;
    const double dt = prm.dt;
    double* p = S.vec;
    double* w = S.vec + 12;
    double* e = S.vec + 24;
    double* t = S.vec + 36;
    double* xv = S.vec + 48;
    if (lane < 12) p[lane] = -prm.q[lane] * S.xr[(H - 1) * 12 + lane];
    LMPC_SYNC();
    for (int k = H - 1; k >= 0; --k) {
        const double* lr = S.LR + k * 4 * LR_SIZE;
        if (lane < 12) w[lane] = S.vk[k * 12 + lane] + p[lane];
        LMPC_SYNC();
        if (lane < 12) {
            const int c = lane, j = c / 3, cc = c % 3;
            double h = 0.0;
#pragma unroll
            for (int m = 0; m < 6; ++m) h += S.G0[m * 12 + c] * w[6 + m];
            const double* L = lr + j * LR_SIZE;
            double ru = L[LR_LIN + cc];
#pragma unroll
            for (int m = 0; m < 3; ++m) ru += L[LR_RT + cc * 3 + m] * L[LR_UP + m];
            e[c] = h + ru;
        }
        LMPC_SYNC();
        if (lane < 12) {
            const int c = lane, j = c / 3, cc = c % 3;
            const double* T = lr + j * LR_SIZE + LR_T;
            t[c] = T[cc] * e[3 * j] + T[3 + cc] * e[3 * j + 1] + T[6 + cc] * e[3 * j + 2];
        }
        LMPC_SYNC();
        if (lane < 12) {
            double y = 0.0;
#pragma unroll
            for (int c = 0; c < 12; ++c) y += S.Li[k * 144 + c * 12 + lane] * t[c];
            S.yk[k * 12 + lane] = y;
        }
        LMPC_SYNC();
        if (k > 0 && lane < 12) {
            const int r = lane;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            double v = -prm.q[r] * S.xr[(k - 1) * 12 + r] + w[r];
            if (r >= 6 && r < 9) {
                double tt = 0.0;
#pragma unroll
                for (int m = 0; m < 3; ++m) tt += Myaw(ck, sk, m, r - 6) * w[m];
                v += dt * tt;
            } else if (r >= 9) {
                v += dt * w[r - 6];
            }
            double yy = 0.0;
#pragma unroll
            for (int m = 0; m < 12; ++m) yy += S.Yk[k * 144 + r * 12 + m] * S.yk[k * 12 + m];
            p[r] = v - yy;
        }
        LMPC_SYNC();
    }
    // forward rollout
    if (lane < 12) {
        xv[lane] = S.hdr[lane];
        if (store_x) S.xk[lane] = S.hdr[lane];
    }
    LMPC_SYNC();
    for (int k = 0; k < H; ++k) {
        const double* lr = S.LR + k * 4 * LR_SIZE;
        if (lane < 12) {
            double v = S.yk[k * 12 + lane];
#pragma unroll
            for (int c = 0; c < 12; ++c) v += S.Yk[k * 144 + c * 12 + lane] * xv[c];
            t[lane] = v;
        }
        LMPC_SYNC();
        if (lane < 12) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < 12; ++r) v += S.Li[k * 144 + lane * 12 + r] * t[r];
            e[lane] = -v;
        }
        LMPC_SYNC();
        if (lane < 12) {
            const int c = lane, j = c / 3, cc = c % 3;
            const double* L = lr + j * LR_SIZE;
            const double u = L[LR_UP + cc] + L[LR_T + cc * 3 + 0] * e[3 * j] +
                             L[LR_T + cc * 3 + 1] * e[3 * j + 1] + L[LR_T + cc * 3 + 2] * e[3 * j + 2];
            S.uk[k * 12 + c] = u;
            w[c] = u;
        }
        LMPC_SYNC();
        double xn = 0.0;
        if (lane < 12) {
            const int r = lane;
            const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
            xn = xv[r];
            if (r < 3) {
                double tt = 0.0;
#pragma unroll
                for (int m = 0; m < 3; ++m) tt += Myaw(ck, sk, r, m) * xv[6 + m];
                xn += dt * tt;
            } else if (r < 6) {
                xn += dt * xv[r + 6];
            } else {
                double bu = 0.0;
#pragma unroll
                for (int m = 0; m < 12; ++m) bu += S.G0[(r - 6) * 12 + m] * w[m];
                xn += bu;
                if (r == 11) xn -= prm.grav * dt;
            }
        }
        LMPC_SYNC();
        if (lane < 12) {
            xv[lane] = xn;
            if (store_x) S.xk[(k + 1) * 12 + lane] = xn;
        }
        LMPC_SYNC();
    }
}

// Adjoint pass: gradient of the (condensed) cost w.r.t. every u_k at the
// current trajectory, g_k = R u_k + B' lambda_{k+1}.  Written to S.yk.
__device__ void adjoint_grad(const DevParams& prm, const Smem& S, int lane) {
    const int H = prm.H;
    const double dt = prm.dt;
    double* lam = S.vec;
    double* ln = S.vec + 12;
    if (lane < 12) lam[lane] = prm.q[lane] * (S.xk[H * 12 + lane] - S.xr[(H - 1) * 12 + lane]);
    LMPC_SYNC();
    for (int k = H - 1; k >= 0; --k) {
        if (lane < 12) {
            const int c = lane;
            double g = prm.r[c] * S.uk[k * 12 + c];
#pragma unroll
            for (int m = 0; m < 6; ++m) g += S.G0[m * 12 + c] * lam[6 + m];
            S.yk[k * 12 + c] = g;
            if (k > 0) {
                const int r = lane;
                const double ck = S.cs[2 * k], sk = S.cs[2 * k + 1];
                double v = prm.q[r] * (S.xk[k * 12 + r] - S.xr[(k - 1) * 12 + r]) + lam[r];
                if (r >= 6 && r < 9) {
                    double tt = 0.0;
#pragma unroll
                    for (int m = 0; m < 3; ++m) tt += Myaw(ck, sk, m, r - 6) * lam[m];
                    v += dt * tt;
                } else if (r >= 9) {
                    v += dt * lam[r - 6];
                }
                ln[r] = v;
            }
        }
        LMPC_SYNC();
        if (k > 0 && lane < 12) lam[lane] = ln[lane];
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
    // orthonormal row basis (Gram-Schmidt)
    double qv[3][3];
    for (int a = 0; a < nr; ++a) {
        double v[3] = {rows[a][0], rows[a][1], rows[a][2]};
        for (int b = 0; b < a; ++b) {
            const double d = qv[b][0] * v[0] + qv[b][1] * v[1] + qv[b][2] * v[2];
            v[0] -= d * qv[b][0]; v[1] -= d * qv[b][1]; v[2] -= d * qv[b][2];
        }
        const double n = 1.0 / sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        qv[a][0] = v[0] * n; qv[a][1] = v[1] * n; qv[a][2] = v[2] * n;
    }
    // particular solution: min-norm f with rows f = bs  (f = sum_a qv_a * beta_a)
    // rows = Lr * qv (lower-triangular Lr from Gram-Schmidt): solve Lr beta = bs
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
        if (fabs(n[0]) < 0.9) e[0] = 1.0; else e[1] = 1.0;
        const double d = n[0] * e[0] + n[1] * e[1] + n[2] * e[2];
        double t1[3] = {e[0] - d * n[0], e[1] - d * n[1], e[2] - d * n[2]};
        const double in = 1.0 / sqrt(t1[0] * t1[0] + t1[1] * t1[1] + t1[2] * t1[2]);
        t1[0] *= in; t1[1] *= in; t1[2] *= in;
        const double t2[3] = {n[1] * t1[2] - n[2] * t1[1], n[2] * t1[0] - n[0] * t1[2], n[0] * t1[1] - n[1] * t1[0]};
        for (int i = 0; i < 3; ++i) { T[i * 3 + 0] = t1[i]; T[i * 3 + 1] = t2[i]; }
    } else if (nr == 2) {
        double t[3] = {qv[0][1] * qv[1][2] - qv[0][2] * qv[1][1], qv[0][2] * qv[1][0] - qv[0][0] * qv[1][2],
                       qv[0][0] * qv[1][1] - qv[0][1] * qv[1][0]};
        const double in = 1.0 / sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        for (int i = 0; i < 3; ++i) T[i * 3 + 0] = t[i] * in;
    }
    return false;
}

// ---------------------------------------------------------------------------
// The fused per-QP kernel.  LS = leg-steps owned per lane = ceil(4H / 64).
// ---------------------------------------------------------------------------
template <int LS>
__global__ void __launch_bounds__(64) lmpc_qp_kernel(const DevParams prm, const double* __restrict__ rec,
                                                     const uint8_t* __restrict__ contact, int batch,
                                                     double* __restrict__ grf, int32_t* __restrict__ status,
                                                     int32_t* __restrict__ iters) {
    extern __shared__ __attribute__((aligned(16))) double lmpc_smem[];
    const int qp = blockIdx.x;
    if (qp >= batch) return;
    const int lane = threadIdx.x;
    const int H = prm.H;
    const int RL = 33 + 12 * H;
    const Smem S = carve(lmpc_smem, H);
    const double mu = prm.mu, fzmax = prm.fmax, dt = prm.dt;

    // ---- load the record (coalesced, one pass) ----
    const double* rin = rec + (size_t)qp * RL;
    for (int i = lane; i < RL; i += 64) {
        const double v = rin[i];
        if (i < 33) S.hdr[i] = v;
        else S.xr[i - 33] = v;
    }
    LMPC_SYNC();
    // I_w^-1 = (R I_b R')^-1
    if (lane == 0) {
        const double* R = S.hdr + LMPC_REC_ROT;
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
        S.col[0] = c00 * id;
        S.col[1] = (Iw[2] * Iw[7] - Iw[1] * Iw[8]) * id;
        S.col[2] = (Iw[1] * Iw[5] - Iw[2] * Iw[4]) * id;
        S.col[3] = c01 * id;
        S.col[4] = (Iw[0] * Iw[8] - Iw[2] * Iw[6]) * id;
        S.col[5] = (Iw[2] * Iw[3] - Iw[0] * Iw[5]) * id;
        S.col[6] = c02 * id;
        S.col[7] = (Iw[1] * Iw[6] - Iw[0] * Iw[7]) * id;
        S.col[8] = (Iw[0] * Iw[4] - Iw[1] * Iw[3]) * id;
    }
    for (int k = lane; k < H; k += 64) {
        double sn, cn;
        sincos(S.xr[12 * k + 2], &sn, &cn);
        S.cs[2 * k] = cn;
        S.cs[2 * k + 1] = sn;
    }
    LMPC_SYNC();
    // G0 = dt [I_w^-1 skew(r_j) ; I/m]  (Utils::skew, Utils.cpp:89-95)
    for (int e = lane; e < 72; e += 64) {
        const int r = e / 12, c = e % 12, j = c / 3, cc = c % 3;
        double v;
        if (r < 3) {
            const double* ft = S.hdr + LMPC_REC_FEET + 3 * j;
            double sk[3];  // column cc of skew(ft)
            if (cc == 0) { sk[0] = 0.0; sk[1] = ft[2]; sk[2] = -ft[1]; }
            else if (cc == 1) { sk[0] = -ft[2]; sk[1] = 0.0; sk[2] = ft[0]; }
            else { sk[0] = ft[1]; sk[1] = -ft[0]; sk[2] = 0.0; }
            v = dt * (S.col[r * 3 + 0] * sk[0] + S.col[r * 3 + 1] * sk[1] + S.col[r * 3 + 2] * sk[2]);
        } else {
            v = (r - 3 == cc) ? dt / prm.mass : 0.0;
        }
        S.G0[e] = v;
    }

    // ---- leg-step ownership and IPM state ----
    bool st[LS], valid[LS];
    int lsk[LS], lsj[LS];
    double f[LS][3], s[LS][5], z[LS][5];
    int nst_loc = 0;
#pragma unroll
    for (int t = 0; t < LS; ++t) {
        const int ls = lane + 64 * t;
        valid[t] = ls < 4 * H;
        lsk[t] = ls >> 2;
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
    }
    const double nst = wave_sum((double)nst_loc);
    LMPC_SYNC();
    int qstatus = LMPC_QP_CONVERGED;
    int ipm_it = 0, prounds = 0;
    if (nst < 0.5) {
        for (int i = lane; i < 12 * H; i += 64) S.uk[i] = 0.0;
        LMPC_SYNC();
    } else {
        const double mc = 5.0 * nst;
        double tol = prm.tol_mu;
        bool done = false;
        for (int att = 0; att < prm.max_attempts && !done; ++att) {
            // ================= interior point =================
            const int it_end = prm.max_iter * (att + 1);
            for (; ipm_it < it_end; ++ipm_it) {
                double loc = 0.0;
#pragma unroll
                for (int t = 0; t < LS; ++t)
                    if (st[t])
#pragma unroll
                        for (int i = 0; i < 5; ++i) loc += s[t][i] * z[t][i];
                const double mu_c = wave_sum(loc) / mc;
                if (mu_c < tol) break;
                // stage records: Rt = diag(r) + C'WC, rt = C'(W(s-b)), T = I/0, up = 0
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!valid[t]) continue;
                    double* L = S.LR + (lsk[t] * 4 + lsj[t]) * LR_SIZE;
                    double W[5] = {0, 0, 0, 0, 0}, wv[5] = {0, 0, 0, 0, 0};
                    if (st[t]) {
#pragma unroll
                        for (int i = 0; i < 5; ++i) {
                            W[i] = z[t][i] / s[t][i];
                            wv[i] = W[i] * (s[t][i] - (i == 4 ? fzmax : 0.0));
                        }
                    }
                    const double sx = W[0] + W[1], sy = W[2] + W[3];
                    const double r0 = st[t] ? prm.r[3 * lsj[t] + 0] : 0.0;
                    const double r1 = st[t] ? prm.r[3 * lsj[t] + 1] : 0.0;
                    const double r2 = st[t] ? prm.r[3 * lsj[t] + 2] : 0.0;
                    L[LR_RT + 0] = r0 + sx;
                    L[LR_RT + 1] = 0.0;
                    L[LR_RT + 2] = mu * (W[0] - W[1]);
                    L[LR_RT + 3] = 0.0;
                    L[LR_RT + 4] = r1 + sy;
                    L[LR_RT + 5] = mu * (W[2] - W[3]);
                    L[LR_RT + 6] = mu * (W[0] - W[1]);
                    L[LR_RT + 7] = mu * (W[2] - W[3]);
                    L[LR_RT + 8] = r2 + mu * mu * (sx + sy) + W[4];
                    double ct[3];
                    cons_tw(wv, mu, ct);
                    L[LR_LIN + 0] = ct[0]; L[LR_LIN + 1] = ct[1]; L[LR_LIN + 2] = ct[2];
#pragma unroll
                    for (int i = 0; i < 9; ++i) L[LR_T + i] = (st[t] && (i % 4 == 0)) ? 1.0 : 0.0;
                    L[LR_UP + 0] = L[LR_UP + 1] = L[LR_UP + 2] = 0.0;
                }
                LMPC_SYNC();
                riccati_factor(prm, S, lane);
                riccati_solve(prm, S, lane, false);
                // predictor analysis
                double dsa[LS][5], dza[LS][5];
                double amax = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    const double* u = S.uk + lsk[t] * 12 + 3 * lsj[t];
                    const double fa[3] = {u[0], u[1], u[2]};
                    double o[5];
                    cons_resid(fa, mu, fzmax, o);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        dsa[t][i] = -o[i] - s[t][i];
                        dza[t][i] = -z[t][i] - (z[t][i] / s[t][i]) * dsa[t][i];
                        if (dsa[t][i] < 0.0) amax = fmin(amax, -s[t][i] / dsa[t][i]);
                        if (dza[t][i] < 0.0) amax = fmin(amax, -z[t][i] / dza[t][i]);
                    }
                }
                const double aa = wave_min(amax);
                loc = 0.0;
#pragma unroll
                for (int t = 0; t < LS; ++t)
                    if (st[t])
#pragma unroll
                        for (int i = 0; i < 5; ++i) loc += (s[t][i] + aa * dsa[t][i]) * (z[t][i] + aa * dza[t][i]);
                const double mu_a = wave_sum(loc) / mc;
                const double ratio = mu_a / mu_c;
                const double sig = ratio * ratio * ratio;
                const double smu = sig * mu_c;
                // corrector right-hand side
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    double* L = S.LR + (lsk[t] * 4 + lsj[t]) * LR_SIZE;
                    double wv[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        wv[i] = (z[t][i] / s[t][i]) * (s[t][i] - (i == 4 ? fzmax : 0.0)) +
                                (smu - dsa[t][i] * dza[t][i]) / s[t][i];
                    double ct[3];
                    cons_tw(wv, mu, ct);
                    L[LR_LIN + 0] = ct[0]; L[LR_LIN + 1] = ct[1]; L[LR_LIN + 2] = ct[2];
                }
                LMPC_SYNC();
                riccati_solve(prm, S, lane, false);
                double fn[LS][3], ds[LS][5], dz[LS][5];
                amax = 1.0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    const double* u = S.uk + lsk[t] * 12 + 3 * lsj[t];
                    fn[t][0] = u[0]; fn[t][1] = u[1]; fn[t][2] = u[2];
                    double o[5];
                    cons_resid(fn[t], mu, fzmax, o);
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
                    for (int m = 0; m < 3; ++m) f[t][m] += alpha * (fn[t][m] - f[t][m]);
#pragma unroll
                    for (int i = 0; i < 5; ++i) {
                        s[t][i] += alpha * ds[t][i];
                        z[t][i] += alpha * dz[t][i];
                    }
                }
                LMPC_SYNC();
            }
            // ================= active-set polish =================
            int act[LS];
#pragma unroll
            for (int t = 0; t < LS; ++t) {
                act[t] = 0;
                if (!st[t]) continue;
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    if (z[t][i] > s[t][i]) act[t] |= 1 << i;
                const double fm = fmax(fabs(f[t][0]), fmax(fabs(f[t][1]), fabs(f[t][2])));
                if (fm < 1e-6 * fzmax) act[t] = 15;  // lift-off: pyramid apex
            }
            for (int rd = 0; rd < prm.max_rounds; ++rd) {
                ++prounds;
                bool apex[LS];
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    apex[t] = false;
                    if (!valid[t]) continue;
                    double* L = S.LR + (lsk[t] * 4 + lsj[t]) * LR_SIZE;
                    double T[9], up[3];
                    if (st[t]) {
                        apex[t] = leg_basis(act[t], mu, fzmax, T, up);
                    } else {
#pragma unroll
                        for (int i = 0; i < 9; ++i) T[i] = 0.0;
                        up[0] = up[1] = up[2] = 0.0;
                    }
#pragma unroll
                    for (int i = 0; i < 9; ++i) {
                        L[LR_T + i] = T[i];
                        L[LR_RT + i] = (i % 4 == 0) ? prm.r[3 * lsj[t] + i / 4] : 0.0;
                    }
                    L[LR_LIN + 0] = L[LR_LIN + 1] = L[LR_LIN + 2] = 0.0;
                    L[LR_UP + 0] = up[0]; L[LR_UP + 1] = up[1]; L[LR_UP + 2] = up[2];
                }
                LMPC_SYNC();
                riccati_factor(prm, S, lane);
                riccati_solve(prm, S, lane, true);
                adjoint_grad(prm, S, lane);
                double gloc = 1.0;
                for (int i = lane; i < 12 * H; i += 64) gloc = fmax(gloc, fabs(S.yk[i]));
                const double gscale = wave_max(gloc);
                int changed = 0;
#pragma unroll
                for (int t = 0; t < LS; ++t) {
                    if (!st[t]) continue;
                    const double* u = S.uk + lsk[t] * 12 + 3 * lsj[t];
                    const double* g = S.yk + lsk[t] * 12 + 3 * lsj[t];
                    const double fu[3] = {u[0], u[1], u[2]};
                    double o[5];
                    cons_resid(fu, mu, fzmax, o);
                    int imax = -1;
                    double vmax = prm.tol_p * fzmax;
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        if (!((act[t] >> i) & 1) && o[i] > vmax) { vmax = o[i]; imax = i; }
                    if (imax >= 0) {
                        act[t] |= 1 << imax;
                        changed = 1;
                        continue;
                    }
                    if (apex[t]) {
                        if (g[2] / mu < fabs(g[0]) + fabs(g[1]) - prm.tol_d * gscale) {
                            act[t] = (g[0] < 0.0 ? 2 : 1) | (g[1] < 0.0 ? 8 : 4);
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
                        rhs[a] = -(Cs[a][0] * g[0] + Cs[a][1] * g[1] + Cs[a][2] * g[2]);
                    }
                    for (int a = 0; a < nr; ++a)
                        for (int b2 = 0; b2 < nr; ++b2)
                            Gm[a][b2] = Cs[a][0] * Cs[b2][0] + Cs[a][1] * Cs[b2][1] + Cs[a][2] * Cs[b2][2];
                    // Gaussian elimination (SPD, no pivoting)
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
                        if (zz[a] < zmin) { zmin = zz[a]; amin = a; }
                    if (amin >= 0) {
                        act[t] &= ~(1 << idx[amin]);
                        changed = 1;
                    }
                }
                LMPC_SYNC();
                if (!__any(changed)) {
                    done = true;
                    break;
                }
            }
            if (!done) tol *= 1e-3;
        }
        if (!done) {
            // no verified active set: return the (feasible) interior-point iterate
            qstatus = LMPC_QP_MAX_ITER;
#pragma unroll
            for (int t = 0; t < LS; ++t) {
                if (!valid[t]) continue;
                double* u = S.uk + lsk[t] * 12 + 3 * lsj[t];
                u[0] = f[t][0]; u[1] = f[t][1]; u[2] = f[t][2];
            }
            LMPC_SYNC();
        }
    }
    // ---- NaN guard (reference: NaN -> zeros, ConvexQPSolver.cpp:321-326) and output ----
    int bad = 0;
    for (int i = lane; i < 12 * H; i += 64) bad |= (S.uk[i] != S.uk[i]) ? 1 : 0;
    const bool anybad = __any(bad);
    double* gout = grf + (size_t)qp * 12 * H;
    for (int i = lane; i < 12 * H; i += 64) gout[i] = anybad ? 0.0 : S.uk[i];
    if (lane == 0) {
        if (status) status[qp] = anybad ? LMPC_QP_NAN : qstatus;
        if (iters) iters[qp] = ipm_it | (prounds << 16);
    }
}

template __global__ void lmpc_qp_kernel<1>(const DevParams, const double*, const uint8_t*, int, double*, int32_t*, int32_t*);
template __global__ void lmpc_qp_kernel<2>(const DevParams, const double*, const uint8_t*, int, double*, int32_t*, int32_t*);

// Host-side launcher (called from lmpc_capi.cpp).
hipError_t launch_qp(const DevParams& prm, const double* rec, const uint8_t* contact, int batch, double* grf,
                     int32_t* status, int32_t* iters, hipStream_t stream) {
    const size_t lds = (size_t)lds_doubles(prm.H) * sizeof(double);
    const dim3 grid(batch), block(64);
    if (4 * prm.H <= 64) {
        (void)hipFuncSetAttribute((const void*)lmpc_qp_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lmpc_qp_kernel<1>, grid, block, lds, stream, prm, rec, contact, batch, grf, status, iters);
    } else {
        (void)hipFuncSetAttribute((const void*)lmpc_qp_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(lmpc_qp_kernel<2>, grid, block, lds, stream, prm, rec, contact, batch, grf, status, iters);
    }
    return hipGetLastError();
}

}  // namespace lmpc

/*
 * lmpc_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY; see lmpc_oracle.h).
 *
 * Restates the reference's ConvexQPSolver QP assembly on plain arrays and
 * solves the resulting strictly convex QP exactly (dense Goldfarb-Idnani dual
 * active set, fp64), returning a KKT certificate.  Parity unpinned (no
 * reference fixtures exist for this path; see header).
 */
#define _GNU_SOURCE
#include "lmpc_oracle.h"

#include <complex.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------
 * Small 3x3 helpers
 * ------------------------------------------------------------------------- */
static void mat3_mul(const double* a, const double* b, double* c) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += a[3 * i + k] * b[3 * k + j];
            c[3 * i + j] = s;
        }
}

static void mat3_inv(const double* m, double* inv) {
    const double c00 = m[4] * m[8] - m[5] * m[7];
    const double c01 = m[5] * m[6] - m[3] * m[8];
    const double c02 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
    const double id = 1.0 / det;
    inv[0] = c00 * id;
    inv[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    inv[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    inv[3] = c01 * id;
    inv[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    inv[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    inv[6] = c02 * id;
    inv[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    inv[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

/* Utils::skew (Utils.cpp:89-95) */
static void skew3(const double* v, double* s) {
    s[0] = 0.0;   s[1] = -v[2]; s[2] = v[1];
    s[3] = v[2];  s[4] = 0.0;   s[5] = -v[0];
    s[6] = -v[1]; s[7] = v[0];  s[8] = 0.0;
}

/* ConvexQPSolver::update_A_matrix (ConvexQPSolver.cpp:214-228) */
void oracle_update_A(double dt, double yaw, double Ad[144]) {
    const double c = cos(yaw), s = sin(yaw);
    memset(Ad, 0, 144 * sizeof(double));
    for (int i = 0; i < 12; ++i) Ad[13 * i] = 1.0;
    /* Ac.block<3,3>(0,6) = [c s 0; -s c 0; 0 0 1] */
    Ad[0 * 12 + 6] += c * dt; Ad[0 * 12 + 7] += s * dt;
    Ad[1 * 12 + 6] += -s * dt; Ad[1 * 12 + 7] += c * dt;
    Ad[2 * 12 + 8] += 1.0 * dt;
    /* Ac.block<3,3>(3,9) = I */
    Ad[3 * 12 + 9] += dt; Ad[4 * 12 + 10] += dt; Ad[5 * 12 + 11] += dt;
}

/* ConvexQPSolver::update_B_matrix (ConvexQPSolver.cpp:198-212) */
void oracle_update_B(const oracle_params* p, const double rot[9], const double feet[12],
                     double Bd[144]) {
    double tmp[9], rt[9], Iw[9], Iwinv[9], sk[9], blk[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) rt[3 * i + j] = rot[3 * j + i];
    mat3_mul(rot, p->trunk_inertia, tmp);
    mat3_mul(tmp, rt, Iw);
    mat3_inv(Iw, Iwinv);
    memset(Bd, 0, 144 * sizeof(double));
    for (int leg = 0; leg < 4; ++leg) {
        skew3(feet + 3 * leg, sk);
        mat3_mul(Iwinv, sk, blk);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Bd[(6 + r) * 12 + 3 * leg + c] = blk[3 * r + c] * p->dt;
        for (int r = 0; r < 3; ++r) Bd[(9 + r) * 12 + 3 * leg + r] = (1.0 / p->robot_mass) * p->dt;
    }
}

/* Sparsity patterns a_trp_/b_trp_ (ConvexQPSolver.cpp:61-98). */
static int in_a_pattern(int r, int c) {
    if (r == c) return 1;
    if (r < 3 && c >= 6 && c < 9) return 1;
    if (r >= 3 && r < 6 && c == r + 6) return 1;
    return 0;
}
static int in_b_pattern(int r, int c) {
    if (r >= 6 && r < 9) return 1;
    if (r >= 9 && r < 12 && (c % 3) == (r - 9)) return 1;
    return 0;
}

/* Terrain extension: contact frame of a unit ground normal n.
 * Columns of R (row-major) are t1, t2, n; R is the minimal rotation taking e_z
 * to n (Rodrigues about e_z x n), so n = e_z gives R = I exactly and the
 * rotated pyramid below is the reference's. */
void oracle_terrain_frame(const double nin[3], double R[9]) {
    const double nn = sqrt(nin[0] * nin[0] + nin[1] * nin[1] + nin[2] * nin[2]);
    const double nx = nin[0] / nn, ny = nin[1] / nn, c = nin[2] / nn;
    const double h = 1.0 / (1.0 + c);
    R[0] = 1.0 - nx * nx * h; R[1] = -nx * ny * h;      R[2] = nx;
    R[3] = -nx * ny * h;      R[4] = 1.0 - ny * ny * h; R[5] = ny;
    R[6] = -nx;               R[7] = -ny;               R[8] = c;
}

void oracle_build_sparse_qp(const oracle_params* p, int H, const double* rec,
                            const uint8_t* contact, double* P_diag, double* q,
                            double* A, double* l, double* u) {
    oracle_build_sparse_qp_ex(p, H, rec, contact, NULL, P_diag, q, A, l, u);
}

void oracle_build_sparse_qp_ex(const oracle_params* p, int H, const double* rec,
                               const uint8_t* contact, const double* normals, double* P_diag,
                               double* q, double* A, double* l, double* u) {
    const int n = 24 * H, m = 32 * H;
    const int dyn = 12 * H, fric = 16 * H;
    const double* x0 = rec + ORACLE_REC_X0;
    const double* rot = rec + ORACLE_REC_ROT;
    const double* feet = rec + ORACLE_REC_FEET;
    const double* xref = rec + ORACLE_REC_XREF;
    double Ad[144], Bd[144];

    /* Hessian diag [r(12), q(12)] x H  (ConvexQPSolver.cpp:33-50) */
    for (int i = 0; i < H; ++i)
        for (int k = 0; k < 12; ++k) {
            P_diag[24 * i + k] = p->r_weights[k];
            P_diag[24 * i + 12 + k] = p->q_weights[k];
        }
    memset(q, 0, (size_t)n * sizeof(double));
    memset(A, 0, (size_t)m * n * sizeof(double));
    memset(l, 0, (size_t)m * sizeof(double));
    memset(u, 0, (size_t)m * sizeof(double));

    /* -I blocks (value -1, ConvexQPSolver.cpp:116-121) */
    for (int i = 0; i < H; ++i)
        for (int k = 0; k < 12; ++k) A[(size_t)(12 * i + k) * n + 24 * i + 12 + k] = -1.0;

    /* per-leg contact frames (terrain extension; flat ground = identity) */
    double Rn[4][9];
    for (int j = 0; j < 4; ++j) {
        if (normals) oracle_terrain_frame(normals + 3 * j, Rn[j]);
        else for (int e = 0; e < 9; ++e) Rn[j][e] = (e % 4 == 0) ? 1.0 : 0.0;
    }
    /* friction rows (ConvexQPSolver.cpp:131-158), on g = R'f: rows t1+-mu n, t2+-mu n */
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < 4; ++j) {
            const int row = dyn + 16 * i + 4 * j;
            const int cx = 24 * i + 3 * j;
            if (!normals) {
                A[(size_t)(row + 0) * n + cx + 0] = 1.0; A[(size_t)(row + 0) * n + cx + 2] = p->mu;
                A[(size_t)(row + 1) * n + cx + 0] = 1.0; A[(size_t)(row + 1) * n + cx + 2] = -p->mu;
                A[(size_t)(row + 2) * n + cx + 1] = 1.0; A[(size_t)(row + 2) * n + cx + 2] = p->mu;
                A[(size_t)(row + 3) * n + cx + 1] = 1.0; A[(size_t)(row + 3) * n + cx + 2] = -p->mu;
            } else {
                const double* R = Rn[j];
                for (int k = 0; k < 3; ++k) {
                    A[(size_t)(row + 0) * n + cx + k] = R[3 * k + 0] + p->mu * R[3 * k + 2];
                    A[(size_t)(row + 1) * n + cx + k] = R[3 * k + 0] - p->mu * R[3 * k + 2];
                    A[(size_t)(row + 2) * n + cx + k] = R[3 * k + 1] + p->mu * R[3 * k + 2];
                    A[(size_t)(row + 3) * n + cx + k] = R[3 * k + 1] - p->mu * R[3 * k + 2];
                }
            }
            l[row + 0] = 0.0;          u[row + 0] = ORACLE_INF;
            l[row + 1] = -ORACLE_INF;  u[row + 1] = 0.0;
            l[row + 2] = 0.0;          u[row + 2] = ORACLE_INF;
            l[row + 3] = -ORACLE_INF;  u[row + 3] = 0.0;
        }
    /* bound rows (ConvexQPSolver.cpp:161-172) + contact schedule (:329-346) */
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < 4; ++j) {
            const int row = dyn + fric + 4 * i + j;
            if (!normals) A[(size_t)row * n + 24 * i + 3 * j + 2] = 1.0;
            else for (int k = 0; k < 3; ++k) A[(size_t)row * n + 24 * i + 3 * j + k] = Rn[j][3 * k + 2];
            l[row] = 0.0;
            u[row] = (double)contact[4 * i + j] * p->f_max;
        }
        /* gravity on row 12i+11 (ConvexQPSolver.cpp:174-176) */
        l[12 * i + 11] = p->gravity * p->dt;
        u[12 * i + 11] = l[12 * i + 11];
    }

    /* calc_mpc_reference loop (ConvexQPSolver.cpp:262-309) */
    oracle_update_B(p, rot, feet, Bd); /* identical for every step (:280-283) */
    for (int i = 0; i < H; ++i) {
        const double* xr = xref + 12 * i;
        oracle_update_A(p->dt, xr[2], Ad);
        for (int r = 0; r < 12; ++r)
            for (int c = 0; c < 12; ++c)
                if (in_b_pattern(r, c)) A[(size_t)(12 * i + r) * n + 24 * i + c] = Bd[12 * r + c];
        if (i == 0) {
            for (int r = 0; r < 12; ++r) {
                double s = 0.0;
                for (int c = 0; c < 12; ++c) s += Ad[12 * r + c] * x0[c];
                u[r] = -s;
            }
            u[11] = u[11] + p->gravity * p->dt;
            for (int r = 0; r < 12; ++r) l[r] = u[r];
        } else {
            for (int r = 0; r < 12; ++r)
                for (int c = 0; c < 12; ++c)
                    if (in_a_pattern(r, c))
                        A[(size_t)(12 * i + r) * n + 24 * i - 12 + c] = Ad[12 * r + c];
        }
        for (int k = 0; k < 12; ++k) q[24 * i + 12 + k] = -p->q_weights[k] * xr[k];
    }
}

/* ---------------------------------------------------------------------------
 * Condensation: generic elimination of the dynamics rows of the sparse QP.
 *   row block i:  E_u u_i + E_x x_i - x_{i+1} = l_i   (x_0 folded into l_0)
 *   => x_{i+1} = E_x x_i + E_u u_i - l_i
 * ------------------------------------------------------------------------- */
int oracle_condense(int H, const double* P_diag, const double* q, const double* A,
                    const double* l, double* Hc, double* g, double* Tout, double* cout) {
    const int n = 24 * H, N = 12 * H;
    double* T = (double*)calloc((size_t)12 * H * N, sizeof(double));
    double* c = (double*)calloc((size_t)12 * H, sizeof(double));
    int rc = 0;
    if (!T || !c) { free(T); free(c); return -1; }

    for (int i = 0; i < H; ++i) {
        const double* rows = A + (size_t)(12 * i) * n;
        double* Ti = T + (size_t)(12 * i) * N;    /* x_{i+1} */
        double* ci = c + 12 * i;
        /* coefficient of x_{i+1} must be -I */
        for (int r = 0; r < 12; ++r)
            for (int k = 0; k < 12; ++k) {
                const double v = rows[(size_t)r * n + 24 * i + 12 + k];
                if (v != (r == k ? -1.0 : 0.0)) rc = -2;
            }
        for (int r = 0; r < 12; ++r) {
            for (int k = 0; k < 12; ++k) Ti[(size_t)r * N + 12 * i + k] = rows[(size_t)r * n + 24 * i + k];
            ci[r] = -l[12 * i + r];
            if (i > 0) {
                const double* Tp = T + (size_t)(12 * (i - 1)) * N;
                const double* cp = c + 12 * (i - 1);
                for (int k = 0; k < 12; ++k) {
                    const double e = rows[(size_t)r * n + 24 * i - 12 + k];
                    if (e == 0.0) continue;
                    for (int col = 0; col < 12 * i; ++col) Ti[(size_t)r * N + col] += e * Tp[(size_t)k * N + col];
                    ci[r] += e * cp[k];
                }
            }
        }
    }
    /* Hc = diag(P_u) + sum_k T_k' diag(P_x,k) T_k ;  g = q_u + sum_k T_k'(P_x c + q_x) */
    memset(Hc, 0, (size_t)N * N * sizeof(double));
    for (int i = 0; i < H; ++i)
        for (int k = 0; k < 12; ++k) {
            Hc[(size_t)(12 * i + k) * N + 12 * i + k] = P_diag[24 * i + k];
            g[12 * i + k] = q[24 * i + k];
        }
    for (int i = 0; i < H; ++i) {
        const int ncol = 12 * (i + 1);
        const double* Ti = T + (size_t)(12 * i) * N;
        for (int r = 0; r < 12; ++r) {
            const double w = P_diag[24 * i + 12 + r];
            const double* tr = Ti + (size_t)r * N;
            const double gr = w * c[12 * i + r] + q[24 * i + 12 + r];
            for (int a = 0; a < ncol; ++a) {
                const double ta = tr[a];
                if (ta == 0.0) continue;
                g[a] += ta * gr;
                if (w == 0.0) continue;
                const double wa = w * ta;
                double* hrow = Hc + (size_t)a * N;
                for (int b = 0; b < ncol; ++b) hrow[b] += wa * tr[b];
            }
        }
    }
    if (Tout) memcpy(Tout, T, (size_t)12 * H * N * sizeof(double));
    if (cout) memcpy(cout, c, (size_t)12 * H * sizeof(double));
    free(T);
    free(c);
    return rc;
}

/* ---------------------------------------------------------------------------
 * Goldfarb-Idnani dual active-set method (Math. Programming 27, 1983),
 * with sparse constraint rows (CSR: ptr/idx/val).
 * ------------------------------------------------------------------------- */
typedef struct gi_cons {
    int m;
    const int* ptr;
    const int* idx;
    const double* val;
    const double* c0;
} gi_cons;

static double gi_dot(const gi_cons* C, int i, const double* x) {
    double s = C->c0[i];
    for (int k = C->ptr[i]; k < C->ptr[i + 1]; ++k) s += C->val[k] * x[C->idx[k]];
    return s;
}

/* d = J' n_i  (J row-major n x n) */
static void gi_Jt_n(int n, const double* J, const gi_cons* C, int i, double* d) {
    memset(d, 0, (size_t)n * sizeof(double));
    for (int k = C->ptr[i]; k < C->ptr[i + 1]; ++k) {
        const double v = C->val[k];
        const double* row = J + (size_t)C->idx[k] * n;
        for (int c = 0; c < n; ++c) d[c] += v * row[c];
    }
}

static void gi_givens(double a, double b, double* c, double* s, double* h) {
    *h = hypot(a, b);
    *c = a / *h;
    *s = b / *h;
}

static int gi_solve_sparse(int n, const double* G, const double* g0, const gi_cons* C,
                           double* x, double* lambda, int* n_active, double* work) {
    double* L = work;                 /* n*n */
    double* J = L + (size_t)n * n;    /* n*n */
    double* R = J + (size_t)n * n;    /* n*n */
    double* d = R + (size_t)n * n;    /* n */
    double* z = d + n;                /* n */
    double* r = z + n;                /* n */
    double* uu = r + n;               /* n+1 */
    double* s = uu + n + 1;           /* m */
    int* act = (int*)(s + C->m);      /* n+1 */
    char* inact = (char*)(act + n + 1); /* m */
    const int m = C->m;

    /* Cholesky G = L L' */
    for (int j = 0; j < n; ++j) {
        double v = G[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) v -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
        if (!(v > 0.0)) return -1;
        const double ljj = sqrt(v);
        L[(size_t)j * n + j] = ljj;
        for (int i = j + 1; i < n; ++i) {
            double w = G[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) w -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
            L[(size_t)i * n + j] = w / ljj;
        }
        for (int i = 0; i < j; ++i) L[(size_t)i * n + j] = 0.0;
    }
    /* J = L^{-T} (upper triangular): solve L' J = I column by column */
    memset(J, 0, (size_t)n * n * sizeof(double));
    for (int col = 0; col < n; ++col) {
        for (int i = col; i >= 0; --i) {
            double v = (i == col) ? 1.0 : 0.0;
            for (int k = i + 1; k <= col; ++k) v -= L[(size_t)k * n + i] * J[(size_t)k * n + col];
            J[(size_t)i * n + col] = v / L[(size_t)i * n + i];
        }
    }
    /* unconstrained minimum x = -J J' g0 */
    for (int c = 0; c < n; ++c) {
        double v = 0.0;
        for (int k = 0; k < n; ++k) v += J[(size_t)k * n + c] * g0[k];
        d[c] = v;
    }
    for (int i = 0; i < n; ++i) {
        double v = 0.0;
        for (int c = i; c < n; ++c) v += J[(size_t)i * n + c] * d[c];
        x[i] = -v;
    }
    memset(R, 0, (size_t)n * n * sizeof(double));
    int q = 0;
    for (int i = 0; i < m; ++i) inact[i] = 1;

    double xnorm = 0.0;
    const int max_iter = 50 * (n + m) + 100;
    int iter = 0;
    for (;;) {
        if (++iter > max_iter) return -3;
        /* step 1: most violated constraint */
        xnorm = 0.0;
        for (int i = 0; i < n; ++i) xnorm = fmax(xnorm, fabs(x[i]));
        const double tol = 1e-11 * (1.0 + xnorm);
        int p = -1;
        double smin = -tol;
        for (int i = 0; i < m; ++i) {
            if (!inact[i]) continue;
            s[i] = gi_dot(C, i, x);
            if (s[i] < smin) { smin = s[i]; p = i; }
        }
        if (p < 0) break;
        double sp = s[p];
        for (int k = 0; k < q; ++k) uu[k] = lambda[act[k]];
        uu[q] = 0.0;
        for (;;) {
            if (++iter > max_iter) return -3;
            /* step 2a: directions */
            gi_Jt_n(n, J, C, p, d);
            double dd = 0.0, dd2 = 0.0;
            for (int c = 0; c < n; ++c) dd += d[c] * d[c];
            for (int c = q; c < n; ++c) dd2 += d[c] * d[c];
            for (int i = 0; i < n; ++i) {
                double v = 0.0;
                for (int c = q; c < n; ++c) v += J[(size_t)i * n + c] * d[c];
                z[i] = v;
            }
            for (int k = q - 1; k >= 0; --k) {
                double v = d[k];
                for (int c = k + 1; c < q; ++c) v -= R[(size_t)k * n + c] * r[c];
                r[k] = v / R[(size_t)k * n + k];
            }
            /* step 2b: step lengths */
            double t1 = INFINITY;
            int lpos = -1;
            for (int k = 0; k < q; ++k) {
                if (r[k] > 0.0) {
                    const double tk = uu[k] / r[k];
                    if (tk < t1) { t1 = tk; lpos = k; }
                }
            }
            const int zfree = dd2 > 1e-24 * dd; /* n_p not in span of active normals */
            const double t2 = zfree ? -sp / dd2 : INFINITY; /* z'n_p = ||J2' n_p||^2 */
            const double t = fmin(t1, t2);
            if (!isfinite(t)) return -2;
            if (!zfree) {
                /* dual step only, drop constraint lpos */
                for (int k = 0; k < q; ++k) uu[k] -= t * r[k];
                uu[q] += t;
                inact[act[lpos]] = 1;
                lambda[act[lpos]] = 0.0;
                goto drop;
            }
            for (int i = 0; i < n; ++i) x[i] += t * z[i];
            for (int k = 0; k < q; ++k) uu[k] -= t * r[k];
            uu[q] += t;
            if (t == t2) {
                /* full step: add constraint p  (Givens-reduce d, append column to R) */
                for (int j = n - 1; j >= q + 1; --j) {
                    if (d[j] == 0.0) continue;
                    double cg, sg, h;
                    gi_givens(d[j - 1], d[j], &cg, &sg, &h);
                    d[j - 1] = h;
                    d[j] = 0.0;
                    for (int k = 0; k < n; ++k) {
                        const double a = J[(size_t)k * n + j - 1], b = J[(size_t)k * n + j];
                        J[(size_t)k * n + j - 1] = cg * a + sg * b;
                        J[(size_t)k * n + j] = -sg * a + cg * b;
                    }
                }
                for (int k = 0; k <= q; ++k) R[(size_t)k * n + q] = d[k];
                act[q] = p;
                inact[p] = 0;
                ++q;
                for (int k = 0; k < q; ++k) lambda[act[k]] = uu[k];
                break; /* back to step 1 */
            }
            /* partial step: drop constraint lpos */
            inact[act[lpos]] = 1;
            lambda[act[lpos]] = 0.0;
        drop:
            for (int k = lpos; k < q - 1; ++k) {
                act[k] = act[k + 1];
                uu[k] = uu[k + 1];
                for (int rr = 0; rr < n; ++rr) R[(size_t)rr * n + k] = R[(size_t)rr * n + k + 1];
            }
            uu[q - 1] = uu[q];
            for (int rr = 0; rr < n; ++rr) R[(size_t)rr * n + q - 1] = 0.0;
            for (int j = lpos; j < q - 1; ++j) {
                const double b = R[(size_t)(j + 1) * n + j];
                if (b == 0.0) continue;
                double cg, sg, h;
                gi_givens(R[(size_t)j * n + j], b, &cg, &sg, &h);
                R[(size_t)j * n + j] = h;
                R[(size_t)(j + 1) * n + j] = 0.0;
                for (int k = j + 1; k < q - 1; ++k) {
                    const double a1 = R[(size_t)j * n + k], a2 = R[(size_t)(j + 1) * n + k];
                    R[(size_t)j * n + k] = cg * a1 + sg * a2;
                    R[(size_t)(j + 1) * n + k] = -sg * a1 + cg * a2;
                }
                for (int k = 0; k < n; ++k) {
                    const double a1 = J[(size_t)k * n + j], a2 = J[(size_t)k * n + j + 1];
                    J[(size_t)k * n + j] = cg * a1 + sg * a2;
                    J[(size_t)k * n + j + 1] = -sg * a1 + cg * a2;
                }
            }
            --q;
            sp = gi_dot(C, p, x); /* still < 0 after a partial step: retry step 2a */
        }
    }
    for (int i = 0; i < m; ++i)
        if (inact[i]) lambda[i] = 0.0;
    if (n_active) *n_active = q;
    return 0;
}

static size_t gi_work_bytes(int n, int m) {
    return (size_t)(3 * n * n + 4 * n + 1 + m) * sizeof(double) + (size_t)(n + 1) * sizeof(int) +
           (size_t)m + 64;
}

int oracle_gi_solve(int n, const double* G, const double* g0, int m, const double* CI,
                    const double* ci0, double* x, double* lambda, int* n_active) {
    int* ptr = (int*)malloc((size_t)(m + 1) * sizeof(int));
    int* idx = (int*)malloc((size_t)n * m * sizeof(int) + 1);
    double* val = (double*)malloc((size_t)n * m * sizeof(double) + 1);
    void* work = malloc(gi_work_bytes(n, m));
    int nnz = 0, rc;
    ptr[0] = 0;
    for (int i = 0; i < m; ++i) {
        for (int k = 0; k < n; ++k) {
            const double v = CI[(size_t)i * n + k];
            if (v != 0.0) { idx[nnz] = k; val[nnz] = v; ++nnz; }
        }
        ptr[i + 1] = nnz;
    }
    gi_cons C = {m, ptr, idx, val, ci0};
    memset(lambda, 0, (size_t)m * sizeof(double));
    rc = gi_solve_sparse(n, G, g0, &C, x, lambda, n_active, (double*)work);
    free(ptr); free(idx); free(val); free(work);
    return rc;
}

/* ---------------------------------------------------------------------------
 * Full instance solve
 * ------------------------------------------------------------------------- */
int oracle_solve(const oracle_params* p, int H, const double* rec, const uint8_t* contact,
                 double* grf, double* kkt, int* n_active) {
    return oracle_solve_ex(p, H, rec, contact, NULL, grf, kkt, n_active);
}

int oracle_solve_ex(const oracle_params* p, int H, const double* rec, const uint8_t* contact,
                    const double* normals, double* grf, double* kkt, int* n_active) {
    const int n = 24 * H, m = 32 * H, N = 12 * H;
    const int dyn = 12 * H, fric = 16 * H;
    int rc = 0;
    double* P = (double*)malloc((size_t)n * sizeof(double));
    double* q = (double*)malloc((size_t)n * sizeof(double));
    double* A = (double*)malloc((size_t)m * n * sizeof(double));
    double* l = (double*)malloc((size_t)m * sizeof(double));
    double* u = (double*)malloc((size_t)m * sizeof(double));
    double* Hc = (double*)malloc((size_t)N * N * sizeof(double));
    double* g = (double*)malloc((size_t)N * sizeof(double));
    int* fidx = (int*)malloc((size_t)N * sizeof(int));   /* free variable -> U index */
    int* umap = (int*)malloc((size_t)N * sizeof(int));   /* U index -> free index or -1 */
    const int max_ineq = 2 * (m - dyn);
    int* cptr = (int*)malloc((size_t)(max_ineq + 1) * sizeof(int));
    int* cidx = (int*)malloc((size_t)max_ineq * 3 * sizeof(int));   /* <= 3 nonzeros per row */
    double* cval = (double*)malloc((size_t)max_ineq * 3 * sizeof(double));
    double* c0 = (double*)malloc((size_t)max_ineq * sizeof(double));
    double *Hf = NULL, *gf = NULL, *xf = NULL, *lam = NULL;
    void* work = NULL;
    if (!P || !q || !A || !l || !u || !Hc || !g || !fidx || !umap || !cptr || !cidx || !cval || !c0) {
        rc = -10;
        goto out;
    }
    oracle_build_sparse_qp_ex(p, H, rec, contact, normals, P, q, A, l, u);
    if (oracle_condense(H, P, q, A, l, Hc, g, NULL, NULL) != 0) { rc = -11; goto out; }

    /* swing leg-steps: bound row u == l == 0 and the friction rows force
     * fx = fy = 0, so the three forces are exactly zero -> eliminate. */
    int nf = 0;
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < 4; ++j) {
            const int brow = dyn + fric + 4 * i + j;
            const int swing = (u[brow] == 0.0 && l[brow] == 0.0);
            for (int k = 0; k < 3; ++k) {
                const int ui = 12 * i + 3 * j + k;
                if (swing) umap[ui] = -1;
                else { umap[ui] = nf; fidx[nf++] = ui; }
            }
        }
    /* inequality rows (friction + bounds) in condensed, reduced coordinates */
    int mi = 0, nnz = 0;
    cptr[0] = 0;
    for (int row = dyn; row < m; ++row) {
        int cnt = 0, ids[4];
        double vs[4];
        int touches_fixed = 0;
        const int blk = (row < dyn + fric) ? (row - dyn) / 16 : (row - dyn - fric) / 4;
        for (int col = 24 * blk; col < 24 * blk + 12; ++col) {
            const double v = A[(size_t)row * n + col];
            if (v == 0.0) continue;
            const int ui = 12 * blk + (col - 24 * blk);
            if (umap[ui] < 0) { touches_fixed = 1; continue; }
            ids[cnt] = umap[ui]; vs[cnt] = v; ++cnt;
        }
        if (touches_fixed) {
            if (cnt != 0 || l[row] > 0.0 || u[row] < 0.0) { rc = -12; goto out; }
            continue;
        }
        if (l[row] > -ORACLE_INF * 0.5) { /* a'x - l >= 0 */
            for (int k = 0; k < cnt; ++k) { cidx[nnz] = ids[k]; cval[nnz] = vs[k]; ++nnz; }
            c0[mi] = -l[row];
            cptr[++mi] = nnz;
        }
        if (u[row] < ORACLE_INF * 0.5) { /* -a'x + u >= 0 */
            for (int k = 0; k < cnt; ++k) { cidx[nnz] = ids[k]; cval[nnz] = -vs[k]; ++nnz; }
            c0[mi] = u[row];
            cptr[++mi] = nnz;
        }
    }
    memset(grf, 0, (size_t)N * sizeof(double));
    if (nf == 0) {
        if (kkt) kkt[0] = kkt[1] = kkt[2] = kkt[3] = 0.0;
        if (n_active) *n_active = 0;
        goto out;
    }
    Hf = (double*)malloc((size_t)nf * nf * sizeof(double));
    gf = (double*)malloc((size_t)nf * sizeof(double));
    xf = (double*)malloc((size_t)nf * sizeof(double));
    lam = (double*)calloc((size_t)(mi + 1), sizeof(double));
    work = malloc(gi_work_bytes(nf, mi));
    if (!Hf || !gf || !xf || !lam || !work) { rc = -10; goto out; }
    for (int a = 0; a < nf; ++a) {
        gf[a] = g[fidx[a]];
        for (int b = 0; b < nf; ++b) Hf[(size_t)a * nf + b] = Hc[(size_t)fidx[a] * N + fidx[b]];
    }
    {
        gi_cons C = {mi, cptr, cidx, cval, c0};
        rc = gi_solve_sparse(nf, Hf, gf, &C, xf, lam, n_active, (double*)work);
        if (rc == 0 && kkt) {
            /* KKT certificate in reduced coordinates */
            double stat = 0.0, scale = 1.0, pv = 0.0, dv = 0.0, comp = 0.0, xn = 1.0;
            double* res = (double*)calloc((size_t)nf, sizeof(double));
            for (int a = 0; a < nf; ++a) {
                double v = gf[a];
                for (int b = 0; b < nf; ++b) v += Hf[(size_t)a * nf + b] * xf[b];
                res[a] = v;
                scale = fmax(scale, fabs(gf[a]));
                xn = fmax(xn, fabs(xf[a]));
            }
            for (int i = 0; i < mi; ++i) {
                const double si = gi_dot(&C, i, xf);
                for (int k = cptr[i]; k < cptr[i + 1]; ++k) res[cidx[k]] -= lam[i] * cval[k];
                pv = fmax(pv, -si);
                dv = fmax(dv, -lam[i]);
                comp = fmax(comp, fabs(lam[i] * si));
                scale = fmax(scale, fabs(lam[i]));
            }
            for (int a = 0; a < nf; ++a) stat = fmax(stat, fabs(res[a]));
            kkt[0] = stat / scale;
            kkt[1] = fmax(pv, 0.0) / xn;
            kkt[2] = fmax(dv, 0.0) / scale;
            kkt[3] = comp / (scale * xn);
            free(res);
        }
    }
    for (int a = 0; a < nf; ++a) grf[fidx[a]] = xf[a];
out:
    free(P); free(q); free(A); free(l); free(u); free(Hc); free(g); free(fidx); free(umap);
    free(cptr); free(cidx); free(cval); free(c0); free(Hf); free(gf); free(xf); free(lam);
    free(work);
    return rc;
}

typedef struct batch_job {
    const oracle_params* p;
    int H, b0, b1;
    const double* rec;
    const uint8_t* contact;
    const double* normals;
    double* grf;
    int32_t* status;
    int fails;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    const int rl = 33 + 12 * j->H;
    for (int b = j->b0; b < j->b1; ++b) {
        const int rc = oracle_solve_ex(j->p, j->H, j->rec + (size_t)b * rl, j->contact + (size_t)b * 4 * j->H,
                                       j->normals ? j->normals + (size_t)b * 12 : NULL,
                                       j->grf + (size_t)b * 12 * j->H, NULL, NULL);
        if (j->status) j->status[b] = rc;
        if (rc != 0) j->fails++;
    }
    return NULL;
}

int oracle_solve_batch(const oracle_params* p, int H, int batch, const double* rec,
                       const uint8_t* contact, double* grf, int32_t* status, int n_threads) {
    return oracle_solve_batch_ex(p, H, batch, rec, contact, NULL, grf, status, n_threads);
}

int oracle_solve_batch_ex(const oracle_params* p, int H, int batch, const double* rec,
                          const uint8_t* contact, const double* normals, double* grf,
                          int32_t* status, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > batch) n_threads = batch > 0 ? batch : 1;
    pthread_t* th = (pthread_t*)malloc((size_t)n_threads * sizeof(pthread_t));
    batch_job* jobs = (batch_job*)calloc((size_t)n_threads, sizeof(batch_job));
    int fails = 0;
    for (int t = 0; t < n_threads; ++t) {
        jobs[t].p = p; jobs[t].H = H; jobs[t].rec = rec; jobs[t].contact = contact; jobs[t].normals = normals;
        jobs[t].grf = grf; jobs[t].status = status;
        jobs[t].b0 = (int)((long long)batch * t / n_threads);
        jobs[t].b1 = (int)((long long)batch * (t + 1) / n_threads);
        if (n_threads == 1) batch_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    for (int t = 0; t < n_threads; ++t) {
        if (n_threads > 1) pthread_join(th[t], NULL);
        fails += jobs[t].fails;
    }
    free(th);
    free(jobs);
    return fails;
}

/* ---------------------------------------------------------------------------
 * LeggedContactFSM restatement
 * ------------------------------------------------------------------------- */
typedef struct gait_tab {
    int size;
    int state[3];
    double sw[3];
} gait_tab;

static gait_tab gait_table(int gait, int leg) {
    gait_tab t;
    memset(&t, 0, sizeof(t));
    switch (gait) {
    case 1: /* crawl  LeggedContactFSM.cpp:158-199 */
        if (leg == 0) { t.size = 2; t.state[0] = 0; t.state[1] = 1; t.sw[0] = 0.25; t.sw[1] = 1.0; }
        else if (leg == 1) { t.size = 3; t.state[0] = 1; t.state[1] = 0; t.state[2] = 1; t.sw[0] = 0.25; t.sw[1] = 0.5; t.sw[2] = 1.0; }
        else if (leg == 2) { t.size = 3; t.state[0] = 1; t.state[1] = 0; t.state[2] = 1; t.sw[0] = 0.5; t.sw[1] = 0.75; t.sw[2] = 1.0; }
        else { t.size = 2; t.state[0] = 1; t.state[1] = 0; t.sw[0] = 0.75; t.sw[1] = 1.0; }
        break;
    case 2: /* trot with stand  LeggedContactFSM.cpp:116-156 */
        if (leg == 0 || leg == 3) { t.size = 2; t.state[0] = 1; t.state[1] = 0; t.sw[0] = 0.6; t.sw[1] = 1.0; }
        else { t.size = 3; t.state[0] = 1; t.state[1] = 0; t.state[2] = 1; t.sw[0] = 0.1; t.sw[1] = 0.5; t.sw[2] = 1.0; }
        break;
    case 3: /* stand  LeggedContactFSM.cpp:201-212 */
        t.size = 1; t.state[0] = 1; t.sw[0] = 1.0;
        break;
    default: /* trot  LeggedContactFSM.cpp:93-114 */
        t.size = 2;
        if (leg == 0 || leg == 3) { t.state[0] = 1; t.state[1] = 0; }
        else { t.state[0] = 0; t.state[1] = 1; }
        t.sw[0] = 0.5; t.sw[1] = 1.0;
        break;
    }
    return t;
}

int oracle_predict_contact(int gait, int leg, double gait_phase, double gait_speed, double dt) {
    const gait_tab t = gait_table(gait, leg);
    double ph = gait_phase + gait_speed * dt;
    while (ph > 1.0) ph -= 1.0;
    for (int i = 0; i < t.size; ++i)
        if (ph <= t.sw[i]) return t.state[i];
    return 1;
}

int oracle_current_contact(int gait, int leg, double gait_phase) {
    const gait_tab t = gait_table(gait, leg);
    for (int i = 0; i < t.size; ++i)
        if (gait_phase < t.sw[i]) return t.state[i];
    return t.state[t.size - 1];
}

/* ---------------------------------------------------------------------------
 * GRF -> joint torque (BaseInterface.cpp:451-459)
 * ------------------------------------------------------------------------- */
/* A1Kinematics::fk (A1Kinematics.cpp:38-72): foot position in the body frame, written out term by
 * term as the reference's expanded expression, for complex joint angles (complex-step derivative). */
static void fk_complex(const double complex q[3], const double ro[3], const double rf[5], double complex p[3]) {
    const double complex c0 = ccos(q[0]), c1 = ccos(q[1]), c2 = ccos(q[2]);
    const double complex s0 = csin(q[0]), s1 = csin(q[1]), s2 = csin(q[2]);
    const double complex s12 = csin(q[1] + q[2]), c12 = ccos(q[1] + q[2]);
    p[0] = rf[0] + ro[2] * s12 - rf[4] * s12 - s1 * rf[3] + ro[0] * c12;
    p[1] = rf[1] + ro[1] * c0 + rf[2] * c0 + c1 * s0 * rf[3] + ro[0] * c1 * s0 * s2 + ro[0] * c2 * s0 * s1
           - ro[2] * c1 * c2 * s0 + ro[2] * s0 * s1 * s2 + rf[4] * c1 * c2 * s0 - rf[4] * s0 * s1 * s2;
    p[2] = ro[1] * s0 + rf[2] * s0 - c0 * c1 * rf[3] - ro[0] * c0 * c1 * s2 - ro[0] * c0 * c2 * s1
           + ro[2] * c0 * c1 * c2 - ro[2] * c0 * s1 * s2 - rf[4] * c0 * c1 * c2 + rf[4] * c0 * s1 * s2;
}

void oracle_foot_position(const double rho_fix[5], const double rho_opt[3], const double q[3], double p[3]) {
    double complex qc[3] = {q[0], q[1], q[2]}, pc[3];
    fk_complex(qc, rho_opt, rho_fix, pc);
    for (int r = 0; r < 3; ++r) p[r] = creal(pc[r]);
}

/* J[3r+c] = dp_r/dq_c by complex-step differentiation (exact to rounding; no subtraction) */
void oracle_foot_jacobian(const double rho_fix[5], const double rho_opt[3], const double q[3], double J[9]) {
    const double h = 1e-30;
    for (int c = 0; c < 3; ++c) {
        double complex qc[3] = {q[0], q[1], q[2]}, pc[3];
        qc[c] += h * I;
        fk_complex(qc, rho_opt, rho_fix, pc);
        for (int r = 0; r < 3; ++r) J[3 * r + c] = cimag(pc[r]) / h;
    }
}

/* tau_i = -J_i' (R' u0_i) per leg (BaseInterface.cpp:453-458); rho_fix[4][5], rho_opt[4][3] */
void oracle_grf_to_torque(const double* rho_fix, const double* rho_opt, const double rot[9],
                          const double joint_pos[12], const double grf0[12], double tau[12]) {
    for (int i = 0; i < 4; ++i) {
        double J[9], fr[3];
        oracle_foot_jacobian(rho_fix + 5 * i, rho_opt + 3 * i, joint_pos + 3 * i, J);
        for (int r = 0; r < 3; ++r)
            fr[r] = rot[r] * grf0[3 * i] + rot[3 + r] * grf0[3 * i + 1] + rot[6 + r] * grf0[3 * i + 2];
        for (int c = 0; c < 3; ++c)
            tau[3 * i + c] = -(J[c] * fr[0] + J[3 + c] * fr[1] + J[6 + c] * fr[2]);
    }
}

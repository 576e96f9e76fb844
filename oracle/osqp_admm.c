/*
 * osqp_admm.c -- the reference's own QP algorithm, OSQP's ADMM, restated in C on the reference's sparse
 * problem (TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it; tests/ check it against the numpy
 * restatement oracle/osqp_restate.py).  Product code never links or calls it.
 *
 * What it restates: the reference hands its QP to OSQP through OsqpEigen
 * (src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:182-194 settings: eps_abs 1e-3, eps_rel 1e-4,
 * warm start; :314-327 update / solve / getSolution; NaN -> zeros :321-326).  OSQP is a third-party dependency
 * the reference does not vendor (unpinned git HEAD, .devcontainer/Dockerfile:55; image dated 2022-10-03: the
 * v0.6.x line).  Its published algorithm -- Stellato et al., Math. Prog. Comp. 12 (2020), Alg. 1 with the v0.6
 * implementation choices -- is restated step for step from oracle/osqp_restate.py: modified Ruiz equilibration
 * (10 passes, scaling bounds [1e-4, 1e4], cost scaling), per-row rho (x1e3 on equality rows, 1e-6 on free rows),
 * over-relaxation alpha = 1.6, sigma = 1e-6, termination on unscaled residuals every 25 iterations, adaptive rho
 * every 100 iterations (tolerance 5x), max_iter 4000, polish off, cold start (x = z = y = 0: the instances are
 * independent, as on the reference's first tick).
 *
 * Linear algebra: OSQP factors the quasi-definite KKT matrix with QDLDL; this restatement factors the
 * equivalent reduced matrix P + sigma I + A' diag(rho) A by an envelope (skyline) Cholesky -- the time-staged
 * variable order [u_0, x_1, u_1, x_2, ...] of the reference (ConvexQPSolver.cpp:101-128) makes it banded
 * (half-bandwidth < 36) -- so one factorisation is O(n b^2) and one solve O(n b).  Same iterates up to
 * rounding.  A is kept in CSR.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "lmpc_oracle.h"

#define OSQP_INFTY 1e30
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define RHO_TOL 1e-4
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define ADAPTIVE_RHO_TOLERANCE 5.0

void oracle_osqp_settings_default(oracle_osqp_settings* s) {
    s->eps_abs = 1e-3;  /* ConvexQPSolver.cpp:183 */
    s->eps_rel = 1e-4;  /* ConvexQPSolver.cpp:184 */
    s->rho = 0.1;
    s->sigma = 1e-6;
    s->alpha = 1.6;
    s->scaling = 10;
    s->max_iter = 4000;
    s->check_termination = 25;
    s->adaptive_rho_interval = 100;
}

static double limit_scaling(double v) {
    if (v < MIN_SCALING) v = 1.0;
    return v > MAX_SCALING ? MAX_SCALING : v;
}

typedef struct work {
    int n, m, nnz;
    int *rp, *ci;     /* CSR of the scaled A */
    double* av;
    double *Pd, *q;   /* scaled diagonal P, scaled q */
    double *D, *E, c;
    double *ls, *us, *rv;
    int* lo;          /* envelope: first column of row i of the reduced matrix */
    double* K;        /* n x n, row-major; lower triangle within the envelope holds L */
    double *x, *z, *y, *xt, *zt, *r, *w;  /* iterates and temporaries */
} work;

static void rho_vec(work* W, double rho) {
    for (int i = 0; i < W->m; ++i) {
        const int loose = W->ls[i] < -OSQP_INFTY * MIN_SCALING && W->us[i] > OSQP_INFTY * MIN_SCALING;
        const int eq = !loose && W->us[i] - W->ls[i] < RHO_TOL;
        W->rv[i] = loose ? RHO_MIN : eq ? RHO_EQ_OVER_RHO_INEQ * rho : rho;
    }
}

/* K = P + sigma I + A' diag(rv) A within the envelope, then L L' in place */
static int factor(work* W, double sigma) {
    const int n = W->n;
    for (int i = 0; i < n; ++i) {
        double* Ki = W->K + (size_t)i * n;
        for (int j = W->lo[i]; j <= i; ++j) Ki[j] = 0.0;
        Ki[i] = W->Pd[i] + sigma;
    }
    for (int r = 0; r < W->m; ++r)
        for (int a = W->rp[r]; a < W->rp[r + 1]; ++a) {
            const int i = W->ci[a];
            const double v = W->rv[r] * W->av[a];
            for (int b = W->rp[r]; b < W->rp[r + 1]; ++b) {
                const int j = W->ci[b];
                if (j <= i) W->K[(size_t)i * n + j] += v * W->av[b];
            }
        }
    for (int i = 0; i < n; ++i) {
        double* Li = W->K + (size_t)i * n;
        for (int j = W->lo[i]; j <= i; ++j) {
            const double* Lj = W->K + (size_t)j * n;
            const int k0 = W->lo[i] > W->lo[j] ? W->lo[i] : W->lo[j];
            double s = Li[j];
            for (int k = k0; k < j; ++k) s -= Li[k] * Lj[k];
            if (j < i) {
                Li[j] = s / Lj[j];
            } else {
                if (!(s > 0.0)) return -1;
                Li[i] = sqrt(s);
            }
        }
    }
    return 0;
}

static void solve_factored(const work* W, double* v) {
    const int n = W->n;
    for (int i = 0; i < n; ++i) {  /* L w = v */
        const double* Li = W->K + (size_t)i * n;
        double s = v[i];
        for (int k = W->lo[i]; k < i; ++k) s -= Li[k] * v[k];
        v[i] = s / Li[i];
    }
    for (int i = n - 1; i >= 0; --i) {  /* L' v = w (column sweep) */
        const double* Li = W->K + (size_t)i * n;
        v[i] /= Li[i];
        for (int k = W->lo[i]; k < i; ++k) v[k] -= Li[k] * v[i];
    }
}

static void amul(const work* W, const double* x, double* out) {
    for (int r = 0; r < W->m; ++r) {
        double s = 0.0;
        for (int a = W->rp[r]; a < W->rp[r + 1]; ++a) s += W->av[a] * x[W->ci[a]];
        out[r] = s;
    }
}

static void atmul(const work* W, const double* y, double* out) {
    memset(out, 0, sizeof(double) * (size_t)W->n);
    for (int r = 0; r < W->m; ++r)
        for (int a = W->rp[r]; a < W->rp[r + 1]; ++a) out[W->ci[a]] += W->av[a] * y[r];
}

static double maxabs(const double* v, int n) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
    return m;
}

static void work_free(work* W) {
    free(W->rp); free(W->ci); free(W->av); free(W->Pd); free(W->q); free(W->D); free(W->E);
    free(W->ls); free(W->us); free(W->rv); free(W->lo); free(W->K);
    free(W->x); free(W->z); free(W->y); free(W->xt); free(W->zt); free(W->r); free(W->w);
}

int oracle_osqp_solve(int n, int m, const double* P_diag, const double* q, const double* A, const double* l,
                      const double* u, const oracle_osqp_settings* s, double* x_out, int* iters, int* converged,
                      double info[3]) {
    work W;
    memset(&W, 0, sizeof(W));
    W.n = n;
    W.m = m;
    int nnz = 0;
    for (size_t e = 0; e < (size_t)n * m; ++e) nnz += A[e] != 0.0;
    W.nnz = nnz;
    W.rp = (int*)malloc(sizeof(int) * (size_t)(m + 1));
    W.ci = (int*)malloc(sizeof(int) * (size_t)(nnz > 0 ? nnz : 1));
    W.av = (double*)malloc(sizeof(double) * (size_t)(nnz > 0 ? nnz : 1));
    W.Pd = (double*)malloc(sizeof(double) * (size_t)n);
    W.q = (double*)malloc(sizeof(double) * (size_t)n);
    W.D = (double*)malloc(sizeof(double) * (size_t)n);
    W.E = (double*)malloc(sizeof(double) * (size_t)m);
    W.ls = (double*)malloc(sizeof(double) * (size_t)m);
    W.us = (double*)malloc(sizeof(double) * (size_t)m);
    W.rv = (double*)malloc(sizeof(double) * (size_t)m);
    W.lo = (int*)malloc(sizeof(int) * (size_t)n);
    W.K = (double*)malloc(sizeof(double) * (size_t)n * n);
    W.x = (double*)calloc((size_t)n, sizeof(double));
    W.z = (double*)calloc((size_t)m, sizeof(double));
    W.y = (double*)calloc((size_t)m, sizeof(double));
    W.xt = (double*)malloc(sizeof(double) * (size_t)n);
    W.zt = (double*)malloc(sizeof(double) * (size_t)m);
    W.r = (double*)malloc(sizeof(double) * (size_t)n);
    W.w = (double*)malloc(sizeof(double) * (size_t)(n > m ? n : m));
    if (!W.rp || !W.ci || !W.av || !W.Pd || !W.q || !W.D || !W.E || !W.ls || !W.us || !W.rv || !W.lo || !W.K ||
        !W.x || !W.z || !W.y || !W.xt || !W.zt || !W.r || !W.w) {
        work_free(&W);
        return -1;
    }
    nnz = 0;
    for (int r = 0; r < m; ++r) {
        W.rp[r] = nnz;
        for (int j = 0; j < n; ++j)
            if (A[(size_t)r * n + j] != 0.0) {
                W.ci[nnz] = j;
                W.av[nnz++] = A[(size_t)r * n + j];
            }
    }
    W.rp[m] = nnz;
    /* envelope of P + A' R A: row i starts at the smallest column sharing a row of A with column i */
    for (int i = 0; i < n; ++i) W.lo[i] = i;
    for (int r = 0; r < m; ++r) {
        if (W.rp[r] == W.rp[r + 1]) continue;
        const int c0 = W.ci[W.rp[r]];  /* CSR columns ascend */
        for (int a = W.rp[r]; a < W.rp[r + 1]; ++a)
            if (c0 < W.lo[W.ci[a]]) W.lo[W.ci[a]] = c0;
    }
    /* modified Ruiz equilibration (OSQP scale_data) */
    for (int j = 0; j < n; ++j) {
        W.Pd[j] = P_diag[j];
        W.q[j] = q[j];
        W.D[j] = 1.0;
    }
    for (int i = 0; i < m; ++i) W.E[i] = 1.0;
    W.c = 1.0;
    double* col = W.xt;  /* temporaries during scaling */
    double* row = W.zt;
    for (int pass = 0; pass < s->scaling; ++pass) {
        for (int j = 0; j < n; ++j) col[j] = fabs(W.Pd[j]);
        for (int r = 0; r < m; ++r) {
            double mx = 0.0;
            for (int a = W.rp[r]; a < W.rp[r + 1]; ++a) {
                const double v = fabs(W.av[a]);
                mx = fmax(mx, v);
                col[W.ci[a]] = fmax(col[W.ci[a]], v);
            }
            row[r] = mx;
        }
        for (int j = 0; j < n; ++j) col[j] = 1.0 / sqrt(limit_scaling(col[j]));
        for (int r = 0; r < m; ++r) row[r] = 1.0 / sqrt(limit_scaling(row[r]));
        for (int j = 0; j < n; ++j) {
            W.Pd[j] *= col[j] * col[j];
            W.q[j] *= col[j];
            W.D[j] *= col[j];
        }
        for (int r = 0; r < m; ++r) {
            for (int a = W.rp[r]; a < W.rp[r + 1]; ++a) W.av[a] *= row[r] * col[W.ci[a]];
            W.E[r] *= row[r];
        }
        double mean = 0.0;
        for (int j = 0; j < n; ++j) mean += fabs(W.Pd[j]);
        mean /= n;
        const double cost = fmax(mean, maxabs(W.q, n));
        const double ct = 1.0 / limit_scaling(cost);
        for (int j = 0; j < n; ++j) {
            W.Pd[j] *= ct;
            W.q[j] *= ct;
        }
        W.c *= ct;
    }
    for (int i = 0; i < m; ++i) {
        const double li = fmin(fmax(l[i], -OSQP_INFTY), OSQP_INFTY), ui = fmin(fmax(u[i], -OSQP_INFTY), OSQP_INFTY);
        W.ls[i] = li <= -OSQP_INFTY ? -OSQP_INFTY : W.E[i] * li;
        W.us[i] = ui >= OSQP_INFTY ? OSQP_INFTY : W.E[i] * ui;
    }
    double rho = s->rho;
    rho_vec(&W, rho);
    if (factor(&W, s->sigma) != 0) {
        work_free(&W);
        return -2;
    }
    int it_done = s->max_iter, conv = 0;
    double prim = INFINITY, dual = INFINITY;
    double* Ax = W.zt;
    double* Aty = W.w;
    for (int it = 1; it <= s->max_iter; ++it) {
        /* r = sigma x - q + A'(rho z - y) */
        for (int i = 0; i < m; ++i) W.w[i] = W.rv[i] * W.z[i] - W.y[i];
        atmul(&W, W.w, W.r);
        for (int j = 0; j < n; ++j) W.r[j] += s->sigma * W.x[j] - W.q[j];
        memcpy(W.xt, W.r, sizeof(double) * (size_t)n);
        solve_factored(&W, W.xt);
        amul(&W, W.xt, W.zt);
        for (int j = 0; j < n; ++j) W.x[j] = s->alpha * W.xt[j] + (1.0 - s->alpha) * W.x[j];
        for (int i = 0; i < m; ++i) {
            const double zr = s->alpha * W.zt[i] + (1.0 - s->alpha) * W.z[i];
            const double zn = fmin(fmax(zr + W.y[i] / W.rv[i], W.ls[i]), W.us[i]);
            W.y[i] += W.rv[i] * (zr - zn);
            W.z[i] = zn;
        }
        const int check = (it % s->check_termination == 0) || it == s->max_iter;
        const int adapt = s->adaptive_rho_interval > 0 && it % s->adaptive_rho_interval == 0;
        if (!check && !adapt) continue;
        amul(&W, W.x, Ax);
        atmul(&W, W.y, Aty);
        if (check) {
            double pr = 0.0, ax = 0.0, zz = 0.0, du = 0.0, px = 0.0, at = 0.0, qq = 0.0;
            for (int i = 0; i < m; ++i) {
                const double ei = 1.0 / W.E[i];
                pr = fmax(pr, fabs(ei * (Ax[i] - W.z[i])));
                ax = fmax(ax, fabs(ei * Ax[i]));
                zz = fmax(zz, fabs(ei * W.z[i]));
            }
            for (int j = 0; j < n; ++j) {
                const double di = 1.0 / W.D[j], pxj = W.Pd[j] * W.x[j];
                du = fmax(du, fabs(di * (pxj + W.q[j] + Aty[j])));
                px = fmax(px, fabs(di * pxj));
                at = fmax(at, fabs(di * Aty[j]));
                qq = fmax(qq, fabs(di * W.q[j]));
            }
            prim = m ? pr : 0.0;
            dual = du / W.c;
            const double ptol = s->eps_abs + s->eps_rel * fmax(ax, zz);
            const double dtol = s->eps_abs + s->eps_rel / W.c * fmax(px, fmax(at, qq));
            if (prim <= ptol && dual <= dtol) {
                it_done = it;
                conv = 1;
                break;
            }
        }
        if (adapt) {
            double pn = 0.0, an = 0.0, zn = 0.0, dn = 0.0, pxn = 0.0, atn = 0.0;
            for (int i = 0; i < m; ++i) {
                pn = fmax(pn, fabs(Ax[i] - W.z[i]));
                an = fmax(an, fabs(Ax[i]));
                zn = fmax(zn, fabs(W.z[i]));
            }
            for (int j = 0; j < n; ++j) {
                const double pxj = W.Pd[j] * W.x[j];
                dn = fmax(dn, fabs(pxj + W.q[j] + Aty[j]));
                pxn = fmax(pxn, fabs(pxj));
                atn = fmax(atn, fabs(Aty[j]));
            }
            pn /= fmax(an, zn) + 1e-10;
            dn /= fmax(pxn, fmax(atn, maxabs(W.q, n))) + 1e-10;
            double est = rho * sqrt(pn / (dn + 1e-10));
            est = fmin(fmax(est, RHO_MIN), RHO_MAX);
            if (est > rho * ADAPTIVE_RHO_TOLERANCE || est < rho / ADAPTIVE_RHO_TOLERANCE) {
                rho = est;
                rho_vec(&W, rho);
                if (factor(&W, s->sigma) != 0) {
                    work_free(&W);
                    return -2;
                }
            }
        }
    }
    for (int j = 0; j < n; ++j) x_out[j] = W.D[j] * W.x[j];
    if (iters) *iters = it_done;
    if (converged) *converged = conv;
    if (info) {
        info[0] = prim;
        info[1] = dual;
        info[2] = rho;
    }
    work_free(&W);
    return 0;
}

/* ---- the reference's compute_grfs restated over a batch (bench.py cpu_baseline) ---- */
typedef struct admm_job {
    const oracle_params* p;
    const oracle_osqp_settings* s;
    int H, b0, b1;
    const double *rec, *normals;
    const uint8_t* contact;
    double* grf;
    int32_t *iters, *converged;
} admm_job;

static void* admm_worker(void* arg) {
    admm_job* J = (admm_job*)arg;
    const int H = J->H, n = 24 * H, m = 32 * H, RL = 33 + 12 * H;
    double* P = (double*)malloc(sizeof(double) * (size_t)n);
    double* q = (double*)malloc(sizeof(double) * (size_t)n);
    double* A = (double*)malloc(sizeof(double) * (size_t)m * n);
    double* l = (double*)malloc(sizeof(double) * (size_t)m);
    double* u = (double*)malloc(sizeof(double) * (size_t)m);
    double* x = (double*)malloc(sizeof(double) * (size_t)n);
    for (int b = J->b0; b < J->b1 && P && q && A && l && u && x; ++b) {
        oracle_build_sparse_qp_ex(J->p, H, J->rec + (size_t)b * RL, J->contact + (size_t)b * 4 * H,
                                  J->normals ? J->normals + (size_t)b * 12 : NULL, P, q, A, l, u);
        int it = 0, cv = 0;
        const int rc = oracle_osqp_solve(n, m, P, q, A, l, u, J->s, x, &it, &cv, NULL);
        int finite = rc == 0;
        for (int j = 0; j < n && finite; ++j) finite = isfinite(x[j]);
        double* g = J->grf + (size_t)b * 12 * H;
        for (int i = 0; i < H; ++i)
            for (int k = 0; k < 12; ++k) g[12 * i + k] = finite ? x[24 * i + k] : 0.0;  /* NaN -> zeros, QPS:321-326 */
        if (J->iters) J->iters[b] = it;
        if (J->converged) J->converged[b] = cv;
    }
    free(P); free(q); free(A); free(l); free(u); free(x);
    return NULL;
}

int oracle_osqp_grf_batch(const oracle_params* p, int H, int batch, const double* rec, const uint8_t* contact,
                          const double* normals, const oracle_osqp_settings* s, double* grf, int32_t* iters,
                          int32_t* converged, int n_threads) {
    oracle_osqp_settings def;
    if (!s) {
        oracle_osqp_settings_default(&def);
        s = &def;
    }
    if (n_threads < 1) n_threads = 1;
    if (n_threads > batch) n_threads = batch > 0 ? batch : 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    admm_job* jobs = (admm_job*)calloc((size_t)n_threads, sizeof(admm_job));
    if (!th || !jobs) {
        free(th);
        free(jobs);
        return -1;
    }
    for (int t = 0; t < n_threads; ++t) {
        admm_job* J = &jobs[t];
        J->p = p; J->s = s; J->H = H; J->rec = rec; J->contact = contact; J->normals = normals;
        J->grf = grf; J->iters = iters; J->converged = converged;
        J->b0 = (int)((long long)batch * t / n_threads);
        J->b1 = (int)((long long)batch * (t + 1) / n_threads);
        if (n_threads == 1) admm_worker(J);
        else pthread_create(&th[t], NULL, admm_worker, J);
    }
    if (n_threads > 1)
        for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

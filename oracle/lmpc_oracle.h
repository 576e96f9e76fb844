/*
 * lmpc_oracle.h -- CPU oracle for the convex-MPC GRF QP (TEST INFRASTRUCTURE ONLY).
 *
 * This is a plain-C restatement of the reference's hot path, used only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * CHECKER.  Product code never links or calls it.
 *
 * What it restates (paths relative to /root/reference/src/legged_ctrl):
 *   - sparse QP layout, Hessian, friction/bound rows, gravity RHS
 *       src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:16-196
 *   - update_B_matrix / update_A_matrix      ConvexQPSolver.cpp:198-228
 *   - calc_mpc_reference (x0, RHS, gradient)  ConvexQPSolver.cpp:254-313
 *   - update_bound_constraints               ConvexQPSolver.cpp:329-346
 *   - update_cons_matrix (values of the dynamics rows) ConvexQPSolver.cpp:230-239
 *   - LeggedContactFSM::predict_contact_state  src/utils/LeggedContactFSM.cpp:280-294
 *     and the gait tables                      LeggedContactFSM.cpp:93-212
 *   - Utils::skew                              src/utils/Utils.cpp:89-95
 *
 * The reference hands the QP to OSQP (third-party, unpinned git HEAD, not
 * vendored; ConvexQPSolver.cpp:182-194,315-320) which only reaches
 * eps_abs=1e-3 / eps_rel=1e-4.  The QP is strictly convex after state
 * elimination (R = 1e-4 I > 0), so its optimum is unique; the oracle returns
 * that exact optimum with a dense dual active-set method (Goldfarb-Idnani),
 * i.e. what a qpOASES-class solver returns, and certifies it by KKT.
 *
 * PARITY STATUS: parity unpinned -- the reference ships no test, fixture or
 * golden vector for this path and cannot be built here (Eigen3, OsqpEigen,
 * OSQP and ROS are absent).  The restatement is cross-checked against an
 * independent numpy restatement + KKT certificate (tests/golden/make_golden.py).
 */
#ifndef LMPC_ORACLE_H
#define LMPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Shared physical / weight parameters (LeggedParam fields read by the path,
 * LeggedState.h:156-165, plus the constants hard-coded in ConvexQPSolver.cpp). */
typedef struct oracle_params {
    double q_weights[12];
    double r_weights[12];
    double robot_mass;
    double trunk_inertia[9]; /* row-major body-frame inertia */
    double mu;               /* 0.3  ConvexQPSolver.cpp:25  */
    double f_max;            /* 180  ConvexQPSolver.cpp:171,336,342 */
    double gravity;          /* 9.8  ConvexQPSolver.cpp:175,296 */
    double dt;               /* MPC_UPDATE_FREQUENCY/1000 = 0.01, ConvexQPSolver.cpp:26 */
} oracle_params;

/* Per-instance record (doubles):  [x0(12) | rot(9,row-major) | feet(4x3 leg-major) | x_ref(H x 12)]
 * contact: H x 4 bytes (1 = stance). */
#define ORACLE_REC_X0   0
#define ORACLE_REC_ROT  12
#define ORACLE_REC_FEET 21
#define ORACLE_REC_XREF 33
#define ORACLE_INF 1e30

/* Build the reference's OSQP problem exactly as ConvexQPSolver leaves it right
 * before solver.solve() (ConvexQPSolver.cpp:315-318), n = 24H, m = 32H:
 *   P_diag[n], q[n], A[m*n] (dense row-major), l[m], u[m].
 * Infinite bounds are written as +/-ORACLE_INF (OsqpEigen::INFTY). */
void oracle_build_sparse_qp(const oracle_params* p, int H, const double* rec,
                            const uint8_t* contact, double* P_diag, double* q,
                            double* A, double* l, double* u);

/* Terrain extension (beyond the reference, which is
 * flat-ground only).  normals[4][3] = per-leg ground normal (need not be unit,
 * n_z > 0), constant over the horizon; NULL = flat ground = the reference.
 * The reference's pyramid and f_max bound act on g = R'f, R = oracle_terrain_frame(n)
 * (columns t1, t2, n; R = I exactly for n = e_z). */
void oracle_terrain_frame(const double n[3], double R[9]);
void oracle_build_sparse_qp_ex(const oracle_params* p, int H, const double* rec,
                               const uint8_t* contact, const double* normals, double* P_diag,
                               double* q, double* A, double* l, double* u);
int oracle_solve_ex(const oracle_params* p, int H, const double* rec, const uint8_t* contact,
                    const double* normals, double* grf, double* kkt, int* n_active);
/* normals[batch][4][3] or NULL */
int oracle_solve_batch_ex(const oracle_params* p, int H, int batch, const double* rec,
                          const uint8_t* contact, const double* normals, double* grf,
                          int32_t* status, int n_threads);

/* GRF -> joint torque, the step after the QP (BaseInterface.cpp:451-459; A1Kinematics.cpp:8-72).
 * Foot position restated from the reference's expanded fk expression; its Jacobian by
 * complex-step differentiation (independent of the product's closed-form Jacobian). */
void oracle_foot_position(const double rho_fix[5], const double rho_opt[3], const double q[3], double p[3]);
void oracle_foot_jacobian(const double rho_fix[5], const double rho_opt[3], const double q[3], double J[9]);
void oracle_grf_to_torque(const double* rho_fix /*[4][5]*/, const double* rho_opt /*[4][3]*/,
                          const double rot[9], const double joint_pos[12], const double grf0[12],
                          double tau[12]);

/* Reference helper restatements (for unit tests). Row-major 12x12. */
void oracle_update_A(double dt, double yaw, double Ad[144]);
void oracle_update_B(const oracle_params* p, const double rot[9], const double feet[12],
                     double Bd[144]);

/* Eliminate the states from the sparse QP (generic dense elimination of the
 * dynamics rows) giving  min 1/2 U'Hc U + g'U  on U = [u_0..u_{H-1}] (N = 12H).
 * Hc[N*N] row-major, g[N].  X = T U + c with T[(12H)*N], c[12H] (may be NULL). */
int oracle_condense(int H, const double* P_diag, const double* q, const double* A,
                    const double* l, double* Hc, double* g, double* T, double* c);

/* Full oracle solve of one instance: build -> condense -> exact dual active set.
 * grf[H*12] receives u_0..u_{H-1} (world-frame forces FL,FR,RL,RR x xyz).
 * kkt[4] (optional) receives the scaled certificate
 * [stationarity, primal violation, dual violation, complementarity].
 * Returns 0 on success, <0 on failure. */
int oracle_solve(const oracle_params* p, int H, const double* rec, const uint8_t* contact,
                 double* grf, double* kkt, int* n_active);

/* oracle_solve over a batch, statically split over n_threads host threads
 * (bench.py's cpu_baseline leg).  status[b] = oracle_solve's return code.
 * Returns the number of failed instances. */
int oracle_solve_batch(const oracle_params* p, int H, int batch, const double* rec,
                       const uint8_t* contact, double* grf, int32_t* status, int n_threads);

/* Dense Goldfarb-Idnani solver:  min 1/2 x'Gx + g0'x  s.t.  CI' x + ci0 >= 0.
 * G[n*n] row-major SPD (not modified), CI[n*m] column-major (column k = constraint k).
 * lambda[m] receives multipliers (0 for inactive).
 * Returns 0 ok, -1 not SPD, -2 infeasible, -3 iteration limit. */
int oracle_gi_solve(int n, const double* G, const double* g0, int m, const double* CI,
                    const double* ci0, double* x, double* lambda, int* n_active);

/* LeggedContactFSM restatement (LeggedContactFSM.cpp:93-212,280-294).
 * gait: 0 trot (default), 1 crawl, 2 trot-with-stand, 3 stand.
 * Returns 1 = STANCE, 0 = SWING. */
int oracle_predict_contact(int gait, int leg, double gait_phase, double gait_speed, double dt);
/* FSM state at gait_phase (what get_contact_state() returns once the FSM has
 * advanced to that phase: first pattern entry whose switch time is > phase). */
int oracle_current_contact(int gait, int leg, double gait_phase);

/* The reference's own algorithm, OSQP's ADMM (osqp_admm.c; restated from its published algorithm, see there),
 * with the reference's settings by default (ConvexQPSolver.cpp:182-194).  Dense row-major A in, CSR inside. */
typedef struct oracle_osqp_settings {
    double eps_abs, eps_rel, rho, sigma, alpha;
    int scaling, max_iter, check_termination, adaptive_rho_interval;
} oracle_osqp_settings;
void oracle_osqp_settings_default(oracle_osqp_settings* s);
/* min 1/2 x'diag(P)x + q'x  s.t. l <= A x <= u; info[3] (optional) = final primal / dual residual, rho.
 * Returns 0 ok, -1 allocation, -2 factorisation failed. */
int oracle_osqp_solve(int n, int m, const double* P_diag, const double* q, const double* A, const double* l,
                      const double* u, const oracle_osqp_settings* s, double* x, int* iters, int* converged,
                      double info[3]);
/* compute_grfs over a batch: the reference's sparse QP (oracle_build_sparse_qp_ex) -> ADMM -> u_0..u_{H-1}
 * (grf[b][H][12]; NaN -> zeros); iters / converged may be NULL; s NULL = the reference's settings. */
int oracle_osqp_grf_batch(const oracle_params* p, int H, int batch, const double* rec, const uint8_t* contact,
                          const double* normals, const oracle_osqp_settings* s, double* grf, int32_t* iters,
                          int32_t* converged, int n_threads);

#ifdef __cplusplus
}
#endif
#endif

/* lmpc_hoqp.h -- C-ABI of the batched hierarchical QP (whole-body control), SURVEY.md 8f row 4.
 *
 * Replaces, for a batch of robots, the reference's chain of priority levels
 *     HoQp ho_qp(task_2, make_shared<HoQp>(task_1, make_shared<HoQp>(task_0)));   (wbc.cpp:93-99)
 * where each level (src/legged_ctrl/src/wbc_ctrl/HoQp.cpp:15-27) minimises, over its coordinates y in the
 * null space Z of every higher level's equalities and its own slacks w,
 *     1/2 |A (x_prev + Z y) - b|^2 + 1/2 |w|^2 + 1/2 1e-12 |y|^2                         (HoQp.cpp:73-107)
 *     s.t. w >= 0,  D (x_prev + Z y) - w <= f,  every higher level's rows D_h x <= f_h + w_h   (:109-145)
 * with qpOASES (:158-174), then x = x_prev + Z y (HoQp.h:41-45) and Z <- Z ker(A Z) by Eigen's FullPivLU
 * kernel basis (:147-156).  The tasks are the reference's Task (include/wbc_ctrl/task.h:16-35): a x = b,
 * d x <= f.  One instance = one chain of `num_levels` tasks over `num_vars` variables; every instance of a
 * batch has the same row counts (pad with zero rows: a zero equality row changes nothing, a zero
 * inequality row gets the slack 0).  Level 0 has the highest priority.
 *
 * Record of one instance (doubles), level after level: a_l [eq_rows][num_vars] row-major, b_l [eq_rows],
 * d_l [ineq_rows][num_vars] row-major, f_l [ineq_rows].
 * Outputs: x [batch][num_levels][num_vars] -- level l's getSolutions(); slack [batch][total ineq rows] --
 * the last level's getStackedSlackSolutions() = [w_0; w_1; ...] (HoQp.cpp:176-182), whose first
 * sum_{k<=l} ineq_rows entries are level l's.  Higher levels' frozen rows are paired with the stacked
 * slacks exactly as the reference pairs them (tasks stacked current-first, HoQp.cpp:58; slacks
 * current-last), which differs from row-by-row pairing only when two higher levels carry inequalities.
 *
 * Numerics: fp64.  Each level's QP is strictly convex (1e-12 regulariser), its optimum unique, but along
 * ker(A Z) the 1e-12 term sits below the rounding of A'A: there the optimum is not resolvable in double
 * (qpOASES included), and a level's x is determined only up to those directions.  Quantities that do not
 * depend on them -- A_l x_l, every slack, and the last level's x when the hierarchy pins every variable
 * (e.g. the WBC) -- are what the parity tests compare.  Levels without equality rows get the same 1e-12
 * term (the reference hands qpOASES a zero Hessian block there; its regularisation picks the point).
 */
#ifndef LMPC_HOQP_H
#define LMPC_HOQP_H

#include <stddef.h>
#include <stdint.h>

#include "lmpc/lmpc.h" /* LMPC_OK / LMPC_ERR_*, LMPC_QP_* status codes */

#ifdef __cplusplus
extern "C" {
#endif

#define LMPC_HOQP_MAX_LEVELS 4
#define LMPC_HOQP_MAX_VARS 64
#define LMPC_HOQP_MAX_ROWS 64      /* equality or inequality rows of one level */
#define LMPC_HOQP_MAX_STACKED 128  /* frozen + own inequality rows at any level */
#define LMPC_HOQP_MAX_LDS_BYTES 65536 /* one chain's LDS block (lmpc_hoqp_lds_bytes) must fit one workgroup */

typedef struct {
    int32_t num_vars;                          /* n (wbc.h:18: 18 + 12 + 12 = 42 for the WBC) */
    int32_t num_levels;                        /* 1..LMPC_HOQP_MAX_LEVELS */
    int32_t eq_rows[LMPC_HOQP_MAX_LEVELS];     /* rows of a_l; 0 = no equality task */
    int32_t ineq_rows[LMPC_HOQP_MAX_LEVELS];   /* rows of d_l; 0 = no inequality task */
} lmpc_hoqp_dims;

typedef struct {
    int32_t max_iter;   /* interior-point iterations per level (default 60) */
    double tol_mu;      /* stop: mean complementarity <= tol_mu * scale (default 1e-13) */
    double tol_res;     /* stop: max primal / dual residual <= tol_res * scale (default 1e-7) */
    int32_t crossover;  /* round 3: 1 (default) = after each level's interior point, the exact active-set crossover
                           (taken when it verifies; bits 16-17 of that level's iteration word: 1 tried, 3 taken):
                           each level's answer is the active-set optimum qpOASES returns, to rounding;
                           0 = the interior-point iterate as is (about 13 % faster on the WBC; ~1e-9 instead of
                           ~1e-12 there, ~1e-4 on degenerate levels) */
} lmpc_hoqp_options;

typedef struct lmpc_hoqp_ctx lmpc_hoqp_ctx;

/* Fills the WBC's dimensions (wbc.cpp:93-96 with the padded row counts of legged_mpc_control_amd/wbc.py):
 * n = 42, levels (30 eq, 44 ineq), (18 eq), (12 eq). */
void lmpc_hoqp_dims_wbc(lmpc_hoqp_dims* d);
void lmpc_hoqp_options_default(lmpc_hoqp_options* o);
/* doubles per instance record; < 0 (LMPC_ERR_ARG) if the dimensions are outside the limits above, including
 * an LDS block over LMPC_HOQP_MAX_LDS_BYTES */
int64_t lmpc_hoqp_record_len(const lmpc_hoqp_dims* d);
/* LDS bytes one chain occupies: (max stacked rows + max(np, max eq rows)) * (np + 1) doubles + vectors, np = n
 * rounded up to 16 (the WBC: 40 448 B, four chains per CU); sets how many chains share a CU */
int64_t lmpc_hoqp_lds_bytes(const lmpc_hoqp_dims* d);
int lmpc_hoqp_slack_len(const lmpc_hoqp_dims* d); /* total inequality rows */

int lmpc_hoqp_create(const lmpc_hoqp_dims* d, int max_batch, int device, lmpc_hoqp_ctx** out);
void lmpc_hoqp_destroy(lmpc_hoqp_ctx* ctx);
int lmpc_hoqp_set_options(lmpc_hoqp_ctx* ctx, const lmpc_hoqp_options* o);

/* Host buffers, synchronous.  status [batch] and iters [batch][num_levels] may be NULL.
 *   LMPC_QP_CONVERGED: every level stopped on its clean criterion (complementarity <= tol_mu * scale and
 *     residuals <= tol_res * scale), or its exact active-set crossover verified (a level that stopped short of
 *     the clean criterion -- degenerate rows whose slack and multiplier both vanish -- is re-solved on the active
 *     set its iterate identifies, and that answer is kept when its multipliers, inactive rows and slacks check
 *     to 1e-9 of the level's scale), or -- the relaxed degenerate stop -- complementarity 1e3 below tol_mu with
 *     the residuals within 1e3 of tol_res when the crossover did not verify;
 *   LMPC_QP_MAX_ITER: some level stopped at max_iter, or on a non-finite Newton direction short of the relaxed
 *     criterion, without a verified crossover (best iterate kept);
 *   LMPC_QP_NAN: a non-finite record entry, residual or result; zeros returned, and the levels after the failing
 *     one report 0 iterations. */
int lmpc_hoqp_solve_batch(lmpc_hoqp_ctx* ctx, const double* tasks, int batch, double* x, double* slack,
                          int32_t* status, int32_t* iters);
/* Device buffers (resident in HBM), asynchronous on `stream` (hipStream_t; NULL = the null stream, as in
 * lmpc.h).  status / iters may be NULL.  Calls on one context are ordered as issued across streams, as in lmpc.h:
 * the event is recorded on the last call's stream when the next device-path call comes on another one, so that
 * stream must still exist then (host-pointer calls, lmpc_hoqp_sync and lmpc_hoqp_destroy wait for the device). */
int lmpc_hoqp_solve_device(lmpc_hoqp_ctx* ctx, const double* d_tasks, int batch, double* d_x, double* d_slack,
                           int32_t* d_status, int32_t* d_iters, void* stream);
int lmpc_hoqp_sync(lmpc_hoqp_ctx* ctx);

/* Round 3: the same solves, also returning every level's getStackedZMatrix() (HoQp.h:26-29: the null-space basis
 * the levels below work in, Z_{l+1} = Z_l ker(A_l Z_l) by Eigen's FullPivLU kernel basis, HoQp.cpp:147-156; Z_l
 * itself for a level without equalities).  z [batch][num_levels][num_vars][num_vars] row-major: level l's basis
 * in its first zcols[b][l] columns, the rest zero (a trivial kernel is Eigen's single zero column: zcols 1).
 * zcols [batch][num_levels] may be NULL; z NULL = the calls above.  LMPC_QP_NAN chains: zeros, zcols 0.
 * The host path allocates its staging for z on first use (max_batch x num_levels x num_vars^2 doubles). */
int lmpc_hoqp_solve_batch_z(lmpc_hoqp_ctx* ctx, const double* tasks, int batch, double* x, double* slack,
                            int32_t* status, int32_t* iters, double* z, int32_t* zcols);
int lmpc_hoqp_solve_device_z(lmpc_hoqp_ctx* ctx, const double* d_tasks, int batch, double* d_x, double* d_slack,
                             int32_t* d_status, int32_t* d_iters, double* d_z, int32_t* d_zcols, void* stream);

/* ---- WBC task formulation (wbc.cpp:102-259), the step before the hierarchical QP ----------------------------
 * Per robot, the dynamics terms the reference takes from Pinocchio (wbc.cpp:59-91) and the task targets; the
 * output is one record of the WBC layout (lmpc_hoqp_dims_wbc, 4472 doubles): level 0 = [M, -J', -S'] x = -h
 * (EoM), swing feet's forces = 0, stance feet's J qdd = -dJ v; +-tau <= limits, friction pyramids of the stance
 * feet (then zero rows); level 1 = base acceleration, swing feet's J qdd = accel - dJ v (then zero rows);
 * level 2 = contact forces = desired.  Rows in the reference's order (legged_mpc_control_amd/wbc.py). */
typedef struct {
    double M[18 * 18];      /* mass matrix, row-major */
    double nle[18];         /* nonlinear effects h(q, v) */
    double J[12 * 18];      /* foot translation Jacobians, foot-major rows (LOCAL_WORLD_ALIGNED) */
    double dJv[12];         /* dJ v per foot */
    double base_accel[6];   /* formulateBaseAccelTask's b (wbc.cpp:195-203) */
    double swing_acc[12];   /* kp (p_des - p) + kd (v_des - v) per foot (wbc.cpp:239) */
    double forces_des[12];  /* input_desired.head(12) */
    double torque_limits[3];/* HAA HFE KFE (config/task.info:226-231: 33.5 each) */
    double mu;              /* friction coefficient (config/task.info:233-236: 0.3) */
    int32_t contact[4];     /* stance flags, FL FR RL RR */
} lmpc_wbc_input;
/* one robot, host */
int lmpc_wbc_tasks(const lmpc_wbc_input* in, double* record);
/* a batch on the device (inputs and records resident in HBM), asynchronous on `stream` */
int lmpc_wbc_tasks_device(const lmpc_wbc_input* d_in, int batch, double* d_records, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LMPC_HOQP_H */

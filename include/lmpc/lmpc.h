/*
 * lmpc.h -- C-ABI of the MI355X-native batched convex-MPC GRF QP solver.
 *
 * This is the drop-in boundary for the reference's convex-MPC QP path
 * (zha0ming1e/legged_mpc_control, src/legged_ctrl):
 *
 *   reference interface (file:line, relative to src/legged_ctrl)        replaced by
 *   ---------------------------------------------------------------     -----------------------
 *   ConvexQPSolver(q_weights, r_weights)  ConvexQPSolver.h:25 /         lmpc_create
 *       ConvexQPSolver.cpp:16-196 (OSQP setup, constants mu/f_max/g)
 *   ~ConvexQPSolver / OSQP workspace       ConvexQPSolver.h:62          lmpc_destroy
 *   calc_mpc_reference(state, leg_FSM)     ConvexQPSolver.cpp:254-313   lmpc_pack_record +
 *                                                                       lmpc_contact_schedule
 *   update_bound_constraints(...)          ConvexQPSolver.cpp:329-346   lmpc_contact_schedule
 *   LeggedContactFSM::predict_contact_state LeggedContactFSM.cpp:280-294 lmpc_predict_contact
 *   update_cons_matrix()                   ConvexQPSolver.cpp:230-239   (no-op: matrices are
 *                                                                        built on the device)
 *   compute_grfs(state) -> u_0 (12)        ConvexQPSolver.cpp:314-327   lmpc_solve_batch (host
 *                                                                        buffers, batch >= 1) /
 *                                                                        lmpc_solve_batch_device
 *
 * All arithmetic is fp64, as in the reference (Eigen double).  Plain C types
 * only; no exceptions cross this boundary.  A context is NOT thread-safe
 * (like the reference solver object): use one context per host thread.
 * Every entry point runs on the context's device and restores the caller's
 * current HIP device before it returns; a stream passed in must belong to the
 * context's device (LMPC_ERR_ARG otherwise).  Calls on one context are
 * ordered as issued even when they use different streams (the context's
 * factor workspace, hand-over flags and staging blocks are shared by every
 * entry point): an asynchronous device-path call on stream A followed by a
 * call on stream B or a host-pointer call makes B / the host wait for A.
 * The wait is set up when the stream changes (an event recorded on A at the
 * call on B), so back-to-back calls on one stream pay no event at all; stream
 * A must therefore still exist at the context's next device-path call on
 * another stream (a host-pointer call, lmpc_sync and lmpc_destroy wait for the
 * device instead and have no such requirement).
 *
 * Per-instance record layout (doubles, see lmpc_record_len):
 *   [ x0(12) | rot(9, row-major body->world) | feet(4 legs x xyz, world-aligned,
 *     body-centred = foot_pos_abs) | x_ref(H x 12) ]
 *   x0    = [euler(3), pos(3), omega_world(3), v_world(3)]  (ConvexQPSolver.cpp:256-259)
 *   x_ref = reference state of step i (ConvexQPSolver.cpp:264-276)
 * contact[H][4] (uint8, 1 = stance): step 0 = plan_contacts, step i>=1 =
 *   predict_contact_state(i*dt) (ConvexQPSolver.cpp:329-346).
 * Output grf[H][12]: u_0..u_{H-1}, FL,FR,RL,RR x (fx,fy,fz) in the world frame;
 *   grf[0..11] is exactly what compute_grfs returns.
 */
#ifndef LMPC_LMPC_H
#define LMPC_LMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LMPC_ABI_VERSION 7 /* 2: terrain-normal extension (_ex entry points); 3: dense-path selection;
                              4: warm start (lmpc_solve_batch_warm, lmpc_shift_active_set);
                              5: dense-path caps in lmpc_options, no environment overrides;
                              6: Riccati-kernel selection (lmpc_set_riccati_path);
                              7: per-leg gait phases in lmpc_command (lmpc_contact_schedule_legs), the polish's
                                 KKT certificate (lmpc_options.tol_x) */
#define LMPC_MAX_HORIZON 32

/* return codes (API level) */
#define LMPC_OK 0
#define LMPC_ERR_ARG (-1)
#define LMPC_ERR_DEVICE (-2)
#define LMPC_ERR_ALLOC (-3)
#define LMPC_ERR_LAUNCH (-4)
#define LMPC_ERR_NOT_BUILT (-5)

/* per-QP status codes (status[b]).  LMPC_QP_CONVERGED is a KKT certificate (ABI 7): the returned forces are primal
 * feasible (pyramid and bound rows within tol_p * f_max), the gradient has no component on any stance leg-step's free
 * directions (within tol_d of the gradient scale) and the multipliers of its active faces are non-negative -- i.e. the
 * exact optimum of the reference's QP to those tolerances.  Which gradient depends on the kernel that solved the QP:
 *   - the Riccati kernels (LMPC_DENSE_OFF, and every QP the dense paths leave) take it from the adjoint of the state
 *     trajectory they swept, so they also check that this trajectory is the dynamics of the returned forces
 *     (x_{k+1} = A_k x_k + B u_k - g dt e11 within tol_x of the state scale);
 *   - the condensed dense paths (LMPC_DENSE_IPM, LMPC_DENSE_GI) take it as H u + g of the condensed QP, where the
 *     dynamics hold by the construction of H and g (there is no trajectory to check): tol_x does not apply to them. */
#define LMPC_QP_CONVERGED 0
#define LMPC_QP_MAX_ITER 1 /* no certified optimum: the best (feasible) interior-point iterate returned */
#define LMPC_QP_NAN 2      /* zeros returned, as the reference does (ConvexQPSolver.cpp:321-326) */

#define LMPC_REC_X0 0
#define LMPC_REC_ROT 12
#define LMPC_REC_FEET 21
#define LMPC_REC_XREF 33

/* Shared parameters: LeggedParam fields read by the path (LeggedState.h:156-165)
 * plus the constants the reference hard-codes (ConvexQPSolver.cpp:25,26,171,175). */
typedef struct lmpc_params {
    double q_weights[12];
    double r_weights[12];
    double robot_mass;
    double trunk_inertia[9]; /* row-major, body frame */
    double mu;               /* friction coefficient, reference 0.3 */
    double f_max;            /* normal-force bound, reference 180 N */
    double gravity;          /* reference 9.8 */
    double dt;               /* MPC step, reference MPC_UPDATE_FREQUENCY/1000 = 0.01 s */
} lmpc_params;

/* Solver options (defaults via lmpc_options_default).  The device solve is a
 * Mehrotra interior point whose Newton step is a Riccati (LQR) recursion over
 * the horizon, followed by an active-set polish (equality-constrained LQR on
 * the identified active set, verified by primal feasibility and multiplier
 * signs).  A verified polish is the exact optimum of the reference's QP. */
typedef struct lmpc_options {
    int max_iter;     /* IPM iterations cap per attempt (default 40) */
    int max_rounds;   /* active-set polish rounds per attempt (default 8) */
    int max_attempts; /* IPM+polish attempts (default 3); each retry stops the IPM 1e-3 tighter, at most
                         1e-8 on the second attempt and 1e-12 on the third (1e-4 lower each further one) */
    double tol_mu;    /* IPM stop: mean complementarity, then the polish (default 2e-4; 1e-4 until round 6) */
    double tol_p;     /* polish primal feasibility, relative to f_max (default 1e-9) */
    double tol_d;     /* polish multiplier sign, relative to gradient scale (default 1e-9) */
    /* ABI 5: the dense paths' caps and the warm-start budget (were environment hooks).  None of them
     * changes the answer: a QP a dense kernel leaves is solved by the Riccati kernel in the same call. */
    int gi_max_steps;      /* dual active set: steps before the hand-over (default 240) */
    int dense_iter_cap;    /* condensed interior point: iterations before the hand-over (default 0 = none) */
    int dense_polish_iter; /* condensed interior point: first-attempt iterations before the polish (default 40) */
    int warm_rounds;       /* warm start: polish rounds before the cold fallback (default 12) */
    /* ABI 7: the certificate's dynamics check -- the Riccati kernels' state trajectory against the dynamics of the
     * forces they return, relative to max(1, max |x|) (default 1e-8; the measured rounding level is <= 2e-10,
     * DESIGN.md 2.6).  The Riccati kernels only: the condensed dense paths have no trajectory (LMPC_QP_CONVERGED). */
    double tol_x;
} lmpc_options;

/* Robot presets: gazebo_go1_convex.yaml:39-71 (+ LeggedState.cpp:146,155-160
 * defaults for mass/inertia) and gazebo_a1_convex.yaml:40-72,133-140. */
void lmpc_params_go1(lmpc_params* p);
void lmpc_params_a1(lmpc_params* p);
void lmpc_options_default(lmpc_options* o);

int lmpc_record_len(int horizon); /* doubles per record: 33 + 12*H */
int lmpc_abi_version(void);
const char* lmpc_strerror(int code);

/* ---- device solver ---------------------------------------------------- */
typedef struct lmpc_ctx lmpc_ctx;

/* Creates a solver context on HIP device `device` for horizon H (1..LMPC_MAX_HORIZON)
 * and batches up to max_batch (host-pointer path staging buffers). */
int lmpc_create(const lmpc_params* p, int horizon, int max_batch, int device, lmpc_ctx** out);
void lmpc_destroy(lmpc_ctx* ctx);
int lmpc_set_options(lmpc_ctx* ctx, const lmpc_options* o);
int lmpc_set_params(lmpc_ctx* ctx, const lmpc_params* p);

/* Dense path (ABI 3).  QPs with 1..20 stance leg-steps at H <= 16 are solved on the condensed QP by
 * LMPC_DENSE_IPM (interior point + active-set polish; the default and, since round 3, the faster kernel
 * both for large batches and for one QP per call, e.g. the per-tick drop-in) or LMPC_DENSE_GI (dual active
 * set: one factorisation, then rank-one steps; a long tail of many-step QPs);
 * LMPC_DENSE_OFF sends every QP to the Riccati kernel.  All return the same optimum: a dense QP left
 * without a verified optimum (iteration or step cap, non-finite iterate) is solved by the Riccati
 * kernel in the same call, so its status is the Riccati kernel's.  Set it before
 * solving; no environment variable changes it (ABI 5).
 * lmpc_get_dense_path returns the path in effect (LMPC_DENSE_OFF when H > 16). */
#define LMPC_DENSE_OFF 0
#define LMPC_DENSE_IPM 1
#define LMPC_DENSE_GI 2
int lmpc_set_dense_path(lmpc_ctx* ctx, int path);
int lmpc_get_dense_path(const lmpc_ctx* ctx);

/* Riccati path (ABI 6).  The QPs no dense kernel takes (more than 20 stance leg-steps, H > 16, or a dense QP
 * left without a verified optimum) run on LMPC_RICCATI_LDS (the default since round 4: every per-stage factor
 * in LDS, no global workspace, the interior point's Newton systems in reduced inputs) or LMPC_RICCATI_SCRATCH (the
 * round-1..3 kernel: factors in a per-QP global workspace).  Both return the same verified optimum (DESIGN.md 4d
 * has the measurements).  Warm-started solves (lmpc_solve_batch_warm) always run on LMPC_RICCATI_SCRATCH.  Fixed
 * per context, never per launch. */
#define LMPC_RICCATI_SCRATCH 0
#define LMPC_RICCATI_LDS 1
int lmpc_set_riccati_path(lmpc_ctx* ctx, int path);
int lmpc_get_riccati_path(const lmpc_ctx* ctx);

/* Pre-allocates the per-QP device workspace of the context's paths for batches up to `batch`: the dense
 * path's hand-over flags and, with LMPC_RICCATI_SCRATCH, the factor workspace (the device path grows them on
 * demand; call this after lmpc_set_riccati_path and before capturing a HIP graph). */
int lmpc_reserve(lmpc_ctx* ctx, int batch);
/* ABI 7: also the warm-start workspace (warm-started solves, lmpc_solve_batch_warm, always run on the scratch kernel):
 * a host that warm-starts calls this once at set-up, so the first warm solve does not allocate (hipMalloc and a
 * device-wide synchronisation) inside the control loop.  The drop-in classes do it in their constructors. */
int lmpc_reserve_warm(lmpc_ctx* ctx, int batch);

/* Host buffers in/out, synchronous.  rec[batch][33+12H], contact[batch][H][4],
 * grf[batch][H][12]; status[batch] and iters[batch] may be NULL. */
int lmpc_solve_batch(lmpc_ctx* ctx, const double* rec, const uint8_t* contact, int batch,
                     double* grf, int32_t* status, int32_t* iters);

/* Device buffers (already resident in HBM), asynchronous on `stream`
 * (a hipStream_t; NULL = HIP's null stream, which is ordered with every blocking stream, e.g.
 * PyTorch's default stream -- the context's own stream is non-blocking and is used only by the
 * host-pointer entry points). Every `void* stream` of this header has this meaning.
 * status/iters may be NULL. */
int lmpc_solve_batch_device(lmpc_ctx* ctx, const double* d_rec, const uint8_t* d_contact,
                            int batch, double* d_grf, int32_t* d_status, int32_t* d_iters,
                            void* stream);

/* Wait for everything the context has issued: its own stream and the last
 * device-path launch on a caller's stream. */
int lmpc_sync(lmpc_ctx* ctx);

/* ---- terrain extension (ABI 2) -------------
 * Beyond the reference, which is flat-ground only (ConvexQPSolver.cpp:131-172).
 * normals[batch][4][3]: per-instance, per-leg ground normal (FL,FR,RL,RR; need
 * not be unit length; n_z > 0), constant over the horizon.  The reference's
 * friction pyramid and 0 <= f_n <= f_max*contact bound then act on the
 * contact-frame force g = R'f, R = lmpc_terrain_frame(n): columns t1, t2, n, the
 * minimal rotation taking e_z to n.  n = e_z gives R = I exactly, so flat
 * normals pose the reference's problem and agree with lmpc_solve_batch to
 * rounding; normals == NULL is the flat (reference) problem itself.  GRFs are
 * returned in the world frame, as always. */
void lmpc_terrain_frame(const double normal[3], double R[9] /* row-major */);
/* host buffers; returns LMPC_ERR_ARG if some normal has n_z <= 0 or is not finite */
int lmpc_solve_batch_ex(lmpc_ctx* ctx, const double* rec, const uint8_t* contact,
                        const double* normals, int batch, double* grf, int32_t* status,
                        int32_t* iters);
/* Warm start across MPC ticks (the reference's OSQP runs with warm_start = true,
 * ConvexQPSolver.cpp:185).  act_in / act_out: [batch][H][4] u8 per leg-step (layout of
 * `contact`): bits 0-3 the active pyramid faces (+fx, -fx, +fy, -fy rows of QPS:131-158),
 * bit 4 the f_max bound, 15 a lift-off leg (f = 0).  The Riccati kernel starts each QP in
 * its active-set polish from act_in (NULL: cold), which verifies the KKT conditions; a set
 * that does not verify within 12 polish rounds falls back to the cold interior point, so the
 * answer is the same exact optimum either way.  act_out (may be NULL) receives the verified
 * set, 0 for swing legs.  Every QP of a warm call runs on the Riccati kernel (the condensed
 * dense kernels are not warm-started).  Host buffers, synchronous. */
int lmpc_solve_batch_warm(lmpc_ctx* ctx, const double* rec, const uint8_t* contact,
                          const double* normals, int batch, const uint8_t* act_in,
                          uint8_t* act_out, double* grf, int32_t* status, int32_t* iters);
/* One MPC step later: stage k takes stage k+1's set, the last stage keeps its own
 * (shifted may alias act). */
void lmpc_shift_active_set(const uint8_t* act, int batch, int H, uint8_t* shifted);
/* device buffers, asynchronous (normals unchecked: the caller guarantees n_z > 0) */
int lmpc_solve_batch_device_ex(lmpc_ctx* ctx, const double* d_rec, const uint8_t* d_contact,
                               const double* d_normals, int batch, double* d_grf,
                               int32_t* d_status, int32_t* d_iters, void* stream);

/* ---- host-side path helpers (exact restatements of the reference) ------ */

/* LeggedContactFSM gait tables (LeggedContactFSM.cpp:93-212). */
#define LMPC_GAIT_TROT 0
#define LMPC_GAIT_CRAWL 1
#define LMPC_GAIT_TROT_WITH_STAND 2
#define LMPC_GAIT_STAND 3

/* predict_contact_state (LeggedContactFSM.cpp:280-294): 1 = STANCE, 0 = SWING */
int lmpc_predict_contact(int gait, int leg, double gait_phase, double gait_speed, double dt);
/* FSM state once it has advanced to gait_phase (get_contact_state()). */
int lmpc_current_contact(int gait, int leg, double gait_phase);

/* update_bound_constraints schedule (ConvexQPSolver.cpp:329-346):
 * contact[0][j] = plan_contacts[j]; contact[i][j] = predict(gait, j, phase, speed, i*dt). */
int lmpc_contact_schedule(int gait, double gait_phase, double gait_speed, double dt, int horizon,
                          const uint8_t plan_contacts[4], uint8_t* contact);
/* ABI 7: the same with one phase per leg, as the reference's four leg FSMs keep them (LeggedContactFSM.h:64; each
 * leg advances on its own in ConvexMpc::foot_update, ConvexMpc.cpp:94-104, and an early touchdown wraps that leg's
 * phase by -1, LeggedContactFSM.cpp:61-66,214-221): contact[i][j] = predict(gait, j, gait_phase[j], speed, i*dt)
 * (ConvexQPSolver.cpp:341-342). */
int lmpc_contact_schedule_legs(int gait, const double gait_phase[4], double gait_speed, double dt, int horizon,
                               const uint8_t plan_contacts[4], uint8_t* contact);

/* calc_mpc_reference input packing (ConvexQPSolver.cpp:256-276). */
typedef struct lmpc_state_in {
    double root_euler[3];
    double root_pos[3];
    double root_ang_vel[3];   /* world frame */
    double root_lin_vel[3];   /* world frame */
    double root_rot_mat[9];   /* row-major */
    double foot_pos_abs[12];  /* leg-major xyz */
    double root_euler_d[3];
    double root_pos_d[3];
    double root_lin_vel_d_rel[3];
    double root_ang_vel_d_rel[3];
} lmpc_state_in;
/* Writes the record; also returns v_d_world = R * v_d_rel (reference writes it
 * back into state.ctrl.root_lin_vel_d_world, ConvexQPSolver.cpp:260). */
int lmpc_pack_record(const lmpc_params* p, int horizon, const lmpc_state_in* st, double* rec,
                     double lin_vel_d_world[3]);

/* ---- the step before the QP, on the device --------------
 * One command per instance = what calc_mpc_reference and update_bound_constraints
 * read (ConvexQPSolver.cpp:254-313,329-346) plus the contact FSM state
 * (LeggedContactFSM.cpp:280-294).  The device expands commands into records and
 * contact schedules in HBM: 408 B in per instance instead of 33+12H doubles and
 * 4H bytes, and no host preprocessing.  The expansion is bit-identical to
 * lmpc_pack_record + lmpc_contact_schedule_legs on the host. */
typedef struct lmpc_command {
    lmpc_state_in state;
    double gait_phase[4];     /* per-leg FSM phase (FL, FR, RL, RR; ABI 7), nominally in [0, 1); a leg that touched
                                 down early carries its wrapped phase (below 0), as LeggedContactFSM::common_enter
                                 leaves it (LeggedContactFSM.cpp:214-221) */
    double gait_speed;        /* phase per second */
    int32_t gait;             /* LMPC_GAIT_* */
    uint8_t plan_contacts[4]; /* step-0 contacts (ctrl.plan_contacts) */
} lmpc_command;

/* host: one command -> rec[33+12H], contact[H][4] */
int lmpc_command_to_record(const lmpc_params* p, int horizon, const lmpc_command* cmd, double* rec,
                           uint8_t* contact);
/* device: d_cmd[batch] -> d_rec[batch][33+12H], d_contact[batch][H][4] (async on stream) */
int lmpc_build_records_device(lmpc_ctx* ctx, const lmpc_command* d_cmd, int batch, double* d_rec,
                              uint8_t* d_contact, void* stream);
/* device: expand into the context's own buffers, then solve (one call per control tick) */
int lmpc_solve_commands_device(lmpc_ctx* ctx, const lmpc_command* d_cmd, const double* d_normals,
                               int batch, double* d_grf, int32_t* d_status, int32_t* d_iters,
                               void* stream);

/* ---- the step after the QP: GRF -> joint torque --------
 * BaseInterface::tau_ctrl_update (BaseInterface.cpp:451-459): per leg i,
 *   f_rel = R' u0_i (world -> body),  tau_i = -J_i' f_rel,
 * J_i = A1Kinematics::jac(q_i, rho_opt_i, rho_fix_i) (A1Kinematics.cpp:14-18): the body-frame
 * foot Jacobian of the hip-abduction / hip / knee chain.  rho_fix = [leg_offset_x, leg_offset_y,
 * motor_offset, upper_leg_length, lower_leg_length], rho_opt = foot offset (BaseInterface.cpp:76-97). */
typedef struct lmpc_leg_kin {
    double rho_fix[4][5];
    double rho_opt[4][3];
} lmpc_leg_kin;
/* the reference's constants (BaseInterface.cpp:76-97, LeggedParams.h:24), FL FR RL RR */
void lmpc_leg_kin_default(lmpc_leg_kin* k);
/* J row-major: J[3*r + c] = d p_r / d q_c */
void lmpc_foot_jacobian(const lmpc_leg_kin* k, int leg, const double q[3], double J[9]);
/* one instance, host: rot[9] row-major, joint_pos[12], grf0[12] (u_0, world) -> tau[12] */
int lmpc_grf_to_torque(const lmpc_leg_kin* k, const double rot[9], const double joint_pos[12],
                       const double grf0[12], double tau[12]);
/* batch, device: R from d_rec[b] (LMPC_REC_ROT), u_0 = d_grf[b][0][:], d_joint_pos[b][12] -> d_tau[b][12] */
int lmpc_grf_to_torque_device(lmpc_ctx* ctx, const lmpc_leg_kin* k, const double* d_rec,
                              const double* d_joint_pos, const double* d_grf, int batch, double* d_tau,
                              void* stream);

/* ---- synthetic batches, counter-based (Philox4x32-10) ---- */
typedef struct lmpc_synth_cfg {
    int gait;             /* LMPC_GAIT_*, or -1 = mixed (uniform over the four) */
    double gait_speed;    /* phase per second (Go1 4.0, A1 3.5) */
    double default_feet[12]; /* default_foot_pos_rel, leg-major */
    int standing;         /* 1 = config-1 nominal standing instance (no randomness) */
} lmpc_synth_cfg;
void lmpc_synth_cfg_go1(lmpc_synth_cfg* c);
void lmpc_synth_cfg_a1_standing(lmpc_synth_cfg* c);
/* Instance b of the batch is global index first_index+b; identical on every rank. */
int lmpc_synth_fill(const lmpc_params* p, const lmpc_synth_cfg* cfg, int horizon, uint64_t seed,
                    int64_t first_index, int count, double* rec, uint8_t* contact);
/* Terrain normals for instances first_index..first_index+count-1 (config 4):
 * per leg, tilt theta ~ U(0, theta_max) about a direction phi ~ U(-pi, pi),
 * n = (sin theta cos phi, sin theta sin phi, cos theta).  A Philox stream separate
 * from lmpc_synth_fill's, so records are identical with and without normals. */
int lmpc_synth_normals(uint64_t seed, int64_t first_index, int count, double theta_max,
                       double* normals /* [count][4][3] */);
/* Synthetic commands (lmpc_synth_fill == lmpc_synth_commands + lmpc_command_to_record).  The
 * device variants generate the same instances from (seed, global index) in HBM, so no input
 * bytes cross PCIe or xGMI; they agree with the host generator to a few ulp
 * (the device math library's sin/cos/log). */
int lmpc_synth_commands(const lmpc_synth_cfg* cfg, uint64_t seed, int64_t first_index, int count,
                        lmpc_command* cmd);
int lmpc_synth_commands_device(lmpc_ctx* ctx, const lmpc_synth_cfg* cfg, uint64_t seed,
                               int64_t first_index, int count, lmpc_command* d_cmd, void* stream);
int lmpc_synth_normals_device(lmpc_ctx* ctx, uint64_t seed, int64_t first_index, int count,
                              double theta_max, double* d_normals, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LMPC_LMPC_H */

// ConvexQPSolver.cpp -- C++ host mirror of legged::ConvexQPSolver over the C-ABI.
// Reference: src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp
#include "lmpc/ConvexQPSolver.hpp"

#include <cstring>
#include <utility>

namespace legged {

ConvexQPSolver::ConvexQPSolver(const double* q_weights, const double* r_weights, int horizon, int device,
                               double robot_mass, const double* trunk_inertia) {
    lmpc_params_go1(&params_);  // mu, f_max, g, dt, inertia defaults (ConvexQPSolver.cpp:25-26,171,175)
    for (int i = 0; i < 12; ++i) {
        params_.q_weights[i] = q_weights[i];
        params_.r_weights[i] = r_weights[i];
    }
    params_.robot_mass = robot_mass;
    if (trunk_inertia) std::memcpy(params_.trunk_inertia, trunk_inertia, 9 * sizeof(double));
    H_ = horizon;
    rec_.assign((size_t)lmpc_record_len(H_), 0.0);
    contact_.assign((size_t)4 * H_, 1);
    grf_.assign((size_t)12 * H_, 0.0);
    act_.assign((size_t)4 * H_, 0);
    act_in_.assign((size_t)4 * H_, 0);
    error_ = lmpc_create(&params_, H_, 1, device, &ctx_);
    // Warm start is on by default (set_warm_start): every tick then runs on the Riccati kernel, from the
    // previous tick's verified active set (the first tick from the cold interior point).  Cold solves
    // (set_warm_start(false)) take the condensed interior point, since round 3 the lower-latency dense kernel
    // for one QP per call too (0.146 ms mean / 0.183 ms p99 per call at H = 10 against 0.166 / 0.303 on the dual
    // active set, tools/single_qp_latency.py).  The Python drop-in (legged_mpc_control_amd.ConvexQPSolver) has
    // the same defaults.
    if (error_ == LMPC_OK) error_ = lmpc_set_dense_path(ctx_, LMPC_DENSE_IPM);
    // the warm-start workspace now, not inside the first tick (hipMalloc + a device-wide synchronisation)
    if (error_ == LMPC_OK) error_ = lmpc_reserve_warm(ctx_, 1);
}

ConvexQPSolver::~ConvexQPSolver() { lmpc_destroy(ctx_); }

ConvexQPSolver::ConvexQPSolver(ConvexQPSolver&& o) noexcept { *this = std::move(o); }

ConvexQPSolver& ConvexQPSolver::operator=(ConvexQPSolver&& o) noexcept {
    if (this != &o) {
        lmpc_destroy(ctx_);
        ctx_ = o.ctx_;
        o.ctx_ = nullptr;
        params_ = o.params_;
        H_ = o.H_;
        rec_ = std::move(o.rec_);
        contact_ = std::move(o.contact_);
        grf_ = std::move(o.grf_);
        act_ = std::move(o.act_);
        act_in_ = std::move(o.act_in_);
        warm_ = o.warm_;
        have_act_ = o.have_act_;
        status_ = o.status_;
        error_ = o.error_;
        iters_ = o.iters_;
    }
    return *this;
}

// ConvexQPSolver::calc_mpc_reference (ConvexQPSolver.cpp:254-313) incl. update_bound_constraints (:329-346)
void ConvexQPSolver::calc_mpc_reference(LeggedState& state, LeggedContactFSM leg_FSM[NUM_LEG]) {
    lmpc_state_in st;
    std::memcpy(st.root_euler, state.fbk.root_euler, sizeof(st.root_euler));
    std::memcpy(st.root_pos, state.fbk.root_pos, sizeof(st.root_pos));
    std::memcpy(st.root_ang_vel, state.fbk.root_ang_vel, sizeof(st.root_ang_vel));
    std::memcpy(st.root_lin_vel, state.fbk.root_lin_vel, sizeof(st.root_lin_vel));
    std::memcpy(st.root_rot_mat, state.fbk.root_rot_mat, sizeof(st.root_rot_mat));
    std::memcpy(st.foot_pos_abs, state.fbk.foot_pos_abs, sizeof(st.foot_pos_abs));
    std::memcpy(st.root_euler_d, state.ctrl.root_euler_d, sizeof(st.root_euler_d));
    std::memcpy(st.root_pos_d, state.ctrl.root_pos_d, sizeof(st.root_pos_d));
    std::memcpy(st.root_lin_vel_d_rel, state.ctrl.root_lin_vel_d_rel, sizeof(st.root_lin_vel_d_rel));
    std::memcpy(st.root_ang_vel_d_rel, state.ctrl.root_ang_vel_d_rel, sizeof(st.root_ang_vel_d_rel));
    lmpc_pack_record(&params_, H_, &st, rec_.data(), state.ctrl.root_lin_vel_d_world);
    for (int j = 0; j < NUM_LEG; ++j) contact_[j] = state.ctrl.plan_contacts[j] ? 1 : 0;
    for (int i = 1; i < H_; ++i)
        for (int j = 0; j < NUM_LEG; ++j)
            contact_[4 * i + j] = leg_FSM[j].predict_contact_state(i * params_.dt) == STANCE ? 1 : 0;
}

// ConvexQPSolver::compute_grfs (ConvexQPSolver.cpp:314-327): returns u_0; NaN -> zeros
std::array<double, DIM_GRF> ConvexQPSolver::compute_grfs(LeggedState& /*state*/) {
    std::array<double, DIM_GRF> out{};
    int32_t st = 0, it = 0;
    if (!ctx_) {
        error_ = LMPC_ERR_DEVICE;
    } else if (warm_ && have_act_) {
        // previous tick's verified set, one step on; a set that no longer verifies falls back to the cold
        // interior point inside the kernel, so the answer is the exact optimum either way
        lmpc_shift_active_set(act_.data(), 1, H_, act_in_.data());
        error_ = lmpc_solve_batch_warm(ctx_, rec_.data(), contact_.data(), nullptr, 1, act_in_.data(), act_.data(),
                                       grf_.data(), &st, &it);
    } else if (warm_) {
        error_ = lmpc_solve_batch_warm(ctx_, rec_.data(), contact_.data(), nullptr, 1, nullptr, act_.data(),
                                       grf_.data(), &st, &it);
    } else {
        error_ = lmpc_solve_batch(ctx_, rec_.data(), contact_.data(), 1, grf_.data(), &st, &it);
    }
    have_act_ = warm_ && error_ == LMPC_OK && st == LMPC_QP_CONVERGED;
    status_ = st;
    iters_ = it;
    if (error_ != LMPC_OK) return out;  // zeros, as the reference returns on a failed solve
    for (int i = 0; i < DIM_GRF; ++i) out[i] = grf_[i];
    return out;
}

}  // namespace legged

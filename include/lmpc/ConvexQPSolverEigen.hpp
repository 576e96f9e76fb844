// ConvexQPSolverEigen.hpp -- the reference's ConvexQPSolver with its own signatures, for a ROS build.
//
// A ROS build of src/legged_ctrl swaps ONE include and links liblmpc.so:
//     ConvexMpc.h:   #include "mpc_ctrl/convex_mpc/ConvexQPSolver.h"   ->   #include "lmpc/ConvexQPSolverEigen.hpp"
// Everything else compiles unchanged, because this class keeps the reference's declarations
// (src/legged_ctrl/include/mpc_ctrl/convex_mpc/ConvexQPSolver.h:23-40):
//     ConvexQPSolver();  ConvexQPSolver(Eigen::VectorXd& q_weights_, Eigen::VectorXd& r_weights_);
//     void calc_mpc_reference(LeggedState& state, LeggedContactFSM leg_FSM[NUM_LEG]);
//     void update_cons_matrix();
//     Eigen::Matrix<double, DIM_GRF, 1> compute_grfs(LeggedState& state);
//     void update_bound_constraints(bool contacts[NUM_LEG], LeggedContactFSM leg_FSM[NUM_LEG]);
// and ConvexMpc's use of it (ConvexMpc.cpp:13-14 assignment from a temporary, :70-72 the tick) reads as is.
// The state and the FSMs are the reference's own types (LeggedState.h, utils/LeggedContactFSM.h): the contact
// schedule is built by calling the reference FSM's predict_contact_state exactly as update_bound_constraints
// does (ConvexQPSolver.cpp:329-346), so no second, phase-synced FSM is kept.  PLAN_HORIZON and
// MPC_UPDATE_FREQUENCY come from the reference's LeggedParams.h, mu / f_max / g from lmpc_params_go1 (the
// reference's constants, ConvexQPSolver.cpp:25-26,171,175).
//
// Header-only; needs Eigen and the reference headers, so it is compiled only inside that build.  The non-Eigen
// mirror (ConvexQPSolver.hpp) is what this repository's tests exercise; both call the same C-ABI (lmpc.h) with
// the same defaults (warm start on, the condensed interior point LMPC_DENSE_IPM for cold solves).
// tests/cpp/eigen_dropin_test.cpp compiles this header against a minimal test stand-in of the few Eigen and
// reference members it touches; it has not been compiled against real Eigen (absent from this image).
#pragma once

#include <Eigen/Dense>

#include <cstring>
#include <utility>
#include <vector>

#include "LeggedParams.h"
#include "LeggedState.h"
#include "utils/LeggedContactFSM.h"
#include "lmpc/lmpc.h"

namespace legged {

class ConvexQPSolver {
public:
    ConvexQPSolver() = default;

    // ConvexQPSolver.cpp:16-196: the weights from the YAML (state.param.q_weights / r_weights)
    ConvexQPSolver(Eigen::VectorXd& q_weights_, Eigen::VectorXd& r_weights_, int device = 0) {
        lmpc_params_go1(&params_);  // mu 0.3, f_max 180, g 9.8; mass / inertia are read per tick from the state
        for (int i = 0; i < 12; ++i) {
            params_.q_weights[i] = q_weights_[i];
            params_.r_weights[i] = r_weights_[i];
        }
        params_.dt = MPC_UPDATE_FREQUENCY / 1000.0;  // ConvexQPSolver.cpp:26
        H_ = PLAN_HORIZON;
        device_ = device;
        rec_.assign((size_t)lmpc_record_len(H_), 0.0);
        contact_.assign((size_t)4 * H_, 1);
        grf_.assign((size_t)12 * H_, 0.0);
        act_.assign((size_t)4 * H_, 0);
        act_in_.assign((size_t)4 * H_, 0);
        error_ = lmpc_create(&params_, H_, 1, device_, &ctx_);
        if (error_ == LMPC_OK) error_ = lmpc_set_dense_path(ctx_, LMPC_DENSE_IPM);
        // warm start is on by default: its workspace now, not at the first tick
        if (error_ == LMPC_OK) error_ = lmpc_reserve_warm(ctx_, 1);
    }
    ~ConvexQPSolver() { lmpc_destroy(ctx_); }
    ConvexQPSolver(const ConvexQPSolver&) = delete;
    ConvexQPSolver& operator=(const ConvexQPSolver&) = delete;
    ConvexQPSolver(ConvexQPSolver&& o) noexcept { *this = std::move(o); }
    ConvexQPSolver& operator=(ConvexQPSolver&& o) noexcept {  // fastConvex = ConvexQPSolver(q, r) (ConvexMpc.cpp:13)
        if (this != &o) {
            lmpc_destroy(ctx_);
            ctx_ = o.ctx_;
            o.ctx_ = nullptr;
            params_ = o.params_;
            H_ = o.H_;
            device_ = o.device_;
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

    // ConvexQPSolver.cpp:254-313 (x0, x_ref, v_d_world written back at :260) + :329-346 (bounds)
    void calc_mpc_reference(LeggedState& state, LeggedContactFSM leg_FSM[NUM_LEG]) {
        if (!ctx_ || H_ == 0) {  // default-constructed (or moved-from) solver: no buffers to write into
            error_ = LMPC_ERR_ARG;
            return;
        }
        lmpc_state_in st;
        for (int i = 0; i < 3; ++i) {
            st.root_euler[i] = state.fbk.root_euler[i];
            st.root_pos[i] = state.fbk.root_pos[i];
            st.root_ang_vel[i] = state.fbk.root_ang_vel[i];
            st.root_lin_vel[i] = state.fbk.root_lin_vel[i];
            st.root_euler_d[i] = state.ctrl.root_euler_d[i];
            st.root_pos_d[i] = state.ctrl.root_pos_d[i];
            st.root_lin_vel_d_rel[i] = state.ctrl.root_lin_vel_d_rel[i];
            st.root_ang_vel_d_rel[i] = state.ctrl.root_ang_vel_d_rel[i];
            for (int j = 0; j < 3; ++j) st.root_rot_mat[3 * i + j] = state.fbk.root_rot_mat(i, j);
        }
        for (int leg = 0; leg < NUM_LEG; ++leg)
            for (int k = 0; k < 3; ++k) st.foot_pos_abs[3 * leg + k] = state.fbk.foot_pos_abs(k, leg);
        // B is built from the state's mass and inertia every tick (update_B_matrix, ConvexQPSolver.cpp:280-283)
        params_.robot_mass = state.param.robot_mass;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) params_.trunk_inertia[3 * i + j] = state.param.a1_trunk_inertia(i, j);
        (void)lmpc_set_params(ctx_, &params_);
        double vdw[3];
        lmpc_pack_record(&params_, H_, &st, rec_.data(), vdw);
        for (int i = 0; i < 3; ++i) state.ctrl.root_lin_vel_d_world[i] = vdw[i];
        update_bound_constraints(state.ctrl.plan_contacts, leg_FSM);
    }

    // ConvexQPSolver.cpp:230-239: the constraint values are generated on the device inside the solve
    void update_cons_matrix() {}

    // ConvexQPSolver.cpp:329-346: step 0 from plan_contacts, step i from the reference FSM's own prediction
    void update_bound_constraints(bool contacts[NUM_LEG], LeggedContactFSM leg_FSM[NUM_LEG]) {
        if (!ctx_ || H_ == 0 || contact_.size() < (size_t)4 * H_) {
            error_ = LMPC_ERR_ARG;
            return;
        }
        for (int j = 0; j < NUM_LEG; ++j) contact_[j] = contacts[j] ? 1 : 0;
        for (int i = 1; i < H_; ++i)
            for (int j = 0; j < NUM_LEG; ++j)
                contact_[4 * i + j] = leg_FSM[j].predict_contact_state(i * params_.dt) == STANCE ? 1 : 0;
    }

    // ConvexQPSolver.cpp:314-327: u_0 (FL, FR, RL, RR x xyz, world frame); NaN or a failed solve -> zeros
    Eigen::Matrix<double, DIM_GRF, 1> compute_grfs(LeggedState& /*state*/) {
        Eigen::Matrix<double, DIM_GRF, 1> out;
        for (int i = 0; i < DIM_GRF; ++i) out(i) = 0.0;
        int32_t st = 0, it = 0;
        if (!ctx_) {
            error_ = LMPC_ERR_DEVICE;
        } else if (warm_) {
            // OSQP's warm_start (ConvexQPSolver.cpp:185): the previous tick's verified active set, one step on
            if (have_act_) lmpc_shift_active_set(act_.data(), 1, H_, act_in_.data());
            error_ = lmpc_solve_batch_warm(ctx_, rec_.data(), contact_.data(), nullptr, 1,
                                           have_act_ ? act_in_.data() : nullptr, act_.data(), grf_.data(), &st, &it);
        } else {
            error_ = lmpc_solve_batch(ctx_, rec_.data(), contact_.data(), 1, grf_.data(), &st, &it);
        }
        have_act_ = warm_ && error_ == LMPC_OK && st == LMPC_QP_CONVERGED;
        status_ = st;
        iters_ = it;
        if (error_ != LMPC_OK) return out;
        for (int i = 0; i < DIM_GRF; ++i) out(i) = grf_[(size_t)i];
        return out;
    }

    // extras (not in the reference)
    const std::vector<double>& last_solution() const { return grf_; }  // u_0 .. u_{H-1}
    int last_status() const { return status_; }
    int last_error() const { return error_; }
    int last_iterations() const { return iters_; }
    void set_warm_start(bool on) {
        warm_ = on;
        have_act_ = false;
    }

private:
    lmpc_ctx* ctx_ = nullptr;
    lmpc_params params_{};
    int H_ = 0;
    int device_ = 0;
    std::vector<double> rec_;
    std::vector<uint8_t> contact_;
    std::vector<double> grf_;
    std::vector<uint8_t> act_, act_in_;
    bool warm_ = true;
    bool have_act_ = false;
    int status_ = 0;
    int error_ = 0;
    int iters_ = 0;
};

}  // namespace legged

// ConvexQPSolver.hpp -- C++ host mirror of the reference's convex-MPC solver
// component, running on the MI355X through the C-ABI in lmpc.h.
//
// Same class and method names, argument meaning and call sequence as
//   src/legged_ctrl/include/mpc_ctrl/convex_mpc/ConvexQPSolver.h:23-40
//   src/legged_ctrl/include/utils/LeggedContactFSM.h:13-50
// so ConvexMpc::grf_update (ConvexMpc.cpp:64-78) reads unchanged:
//     fastConvex.calc_mpc_reference(state, leg_FSM);
//     fastConvex.update_cons_matrix();
//     auto qp_solution = fastConvex.compute_grfs(state);
// The state record below carries exactly the LeggedState fields the QP path
// reads (LeggedState.h:29-34,52,79-96,156-165) as plain arrays (row-major
// rotation, leg-major foot positions) instead of Eigen types; INTEGRATION.md
// shows the Eigen adapter a ROS build adds.
#pragma once

#include <array>
#include <vector>

#include "lmpc/lmpc.h"

namespace legged {

constexpr int NUM_LEG = 4;
constexpr int DIM_GRF = 12;
constexpr int MPC_STATE_DIM_SPARSE = 12;
constexpr double MPC_UPDATE_FREQUENCY = 10.0;  // ms (LeggedParams.h:7)
constexpr int PLAN_HORIZON = 30;              // LeggedParams.h:13 (runtime here)

enum LeggedContactState { SWING, STANCE };

struct LeggedFeedback {
    double root_euler[3] = {0, 0, 0};
    double root_pos[3] = {0, 0, 0};
    double root_ang_vel[3] = {0, 0, 0};   // world frame
    double root_lin_vel[3] = {0, 0, 0};   // world frame
    double root_rot_mat[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};  // row-major
    double foot_pos_abs[12] = {0};        // leg-major xyz (column i of the reference's 3x4)
};

struct LeggedCtrl {
    double root_euler_d[3] = {0, 0, 0};
    double root_pos_d[3] = {0, 0, 0};
    double root_lin_vel_d_rel[3] = {0, 0, 0};
    double root_lin_vel_d_world[3] = {0, 0, 0};
    double root_ang_vel_d_rel[3] = {0, 0, 0};
    bool plan_contacts[NUM_LEG] = {true, true, true, true};
};

struct LeggedParam {
    double q_weights[12] = {0};
    double r_weights[12] = {0};
    double robot_mass = 13.0;
    double a1_trunk_inertia[9] = {0.0158533, 0, 0, 0, 0.0377999, 0, 0, 0, 0.0456542};
    double gait_counter_speed = 4.0;
};

struct LeggedState {
    LeggedFeedback fbk;
    LeggedCtrl ctrl;
    LeggedParam param;
};

// Gait-phase part of the reference FSM (swing-trajectory generation is not on the QP path).
class LeggedContactFSM {
public:
    LeggedContactFSM() = default;
    void reset_params(LeggedState& legged_state, int leg_id) {
        leg_id_ = leg_id;
        gait_speed_ = legged_state.param.gait_counter_speed;
        set_default_gait_pattern();
    }
    void set_default_gait_pattern() { gait_ = LMPC_GAIT_TROT; }
    void set_crawl_gait_pattern() { gait_ = LMPC_GAIT_CRAWL; }
    void set_trot_with_stand_gait_pattern() { gait_ = LMPC_GAIT_TROT_WITH_STAND; }
    void set_default_stand_pattern() { gait_ = LMPC_GAIT_STAND; }
    void reset() { gait_phase_ = 0.0; }
    // phase progression of LeggedContactFSM::update (LeggedContactFSM.cpp:50,214-221)
    double advance(double dt) {
        gait_phase_ += gait_speed_ * dt;
        while (gait_phase_ >= 1.0) gait_phase_ -= 1.0;
        return gait_phase_;
    }
    void set_gait_phase(double ph) { gait_phase_ = ph; }
    double gait_phase() const { return gait_phase_; }
    int gait() const { return gait_; }
    double gait_speed() const { return gait_speed_; }
    LeggedContactState get_contact_state() const {
        return lmpc_current_contact(gait_, leg_id_, gait_phase_) ? STANCE : SWING;
    }
    LeggedContactState predict_contact_state(double dt) const {
        return lmpc_predict_contact(gait_, leg_id_, gait_phase_, gait_speed_, dt) ? STANCE : SWING;
    }

private:
    int leg_id_ = 0;
    int gait_ = LMPC_GAIT_TROT;
    double gait_phase_ = 0.0;
    double gait_speed_ = 4.0;
};

class ConvexQPSolver {
public:
    ConvexQPSolver() = default;
    // ConvexQPSolver.cpp:16 ; horizon/device are runtime here (PLAN_HORIZON macro in the reference)
    ConvexQPSolver(const double* q_weights, const double* r_weights, int horizon = PLAN_HORIZON,
                   int device = 0, double robot_mass = 13.0, const double* trunk_inertia = nullptr);
    ~ConvexQPSolver();
    ConvexQPSolver(const ConvexQPSolver&) = delete;
    ConvexQPSolver& operator=(const ConvexQPSolver&) = delete;
    ConvexQPSolver(ConvexQPSolver&& o) noexcept;
    ConvexQPSolver& operator=(ConvexQPSolver&& o) noexcept;

    void calc_mpc_reference(LeggedState& state, LeggedContactFSM leg_FSM[NUM_LEG]);
    void update_cons_matrix() {}  // values are assembled on the device inside the solve
    std::array<double, DIM_GRF> compute_grfs(LeggedState& state);

    // extras (not in the reference): whole-horizon solution and per-QP status
    const std::vector<double>& last_solution() const { return grf_; }
    int last_status() const { return status_; }
    int last_error() const { return error_; }
    int horizon() const { return H_; }
    // warm start across ticks (the reference's OSQP runs with warm_start = true, ConvexQPSolver.cpp:185):
    // each tick starts from the previous tick's verified active set, shifted one step (default on)
    void set_warm_start(bool on) {
        warm_ = on;
        have_act_ = false;
    }
    bool warm_start() const { return warm_; }
    int last_iterations() const { return iters_; }  // interior-point iterations | polish rounds << 16

private:
    lmpc_ctx* ctx_ = nullptr;
    lmpc_params params_{};
    int H_ = 0;
    std::vector<double> rec_;
    std::vector<uint8_t> contact_;
    std::vector<double> grf_;
    std::vector<uint8_t> act_, act_in_;  // last verified active set [H][4]; its one-step shift
    bool warm_ = true;
    bool have_act_ = false;
    int status_ = 0;
    int error_ = 0;
    int iters_ = 0;
};

}  // namespace legged

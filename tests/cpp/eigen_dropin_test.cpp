// The reference's ConvexMpc (src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexMpc.cpp:6-22,64-78) over
// include/lmpc/ConvexQPSolverEigen.hpp: the constructor and grf_update lines below are the reference's, verbatim;
// only the include of the solver header differs.  Compiled against the test stand-ins in tests/cpp/eigen_dropin/
// (this image has neither Eigen nor ROS).  Prints, per tick, the status, the contact schedule the solver built, the
// packed record the checker rebuilds and u_0, for tests/test_gpu_parity.py to compare with the oracle.
//   eigen_dropin_test <ticks>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "lmpc/ConvexQPSolverEigen.hpp"

namespace legged {
class ConvexMpc {
public:
    explicit ConvexMpc(LeggedState& state) {
        for (int i = 0; i < NUM_LEG; i++) {
            leg_FSM[i].reset_params(state, i);
        }
        // notice we scale weights by control dt
        fastConvex = ConvexQPSolver(state.param.q_weights,
                                    state.param.r_weights);
    }
    bool grf_update(LeggedState& state, double t, double dt) {
        fastConvex.calc_mpc_reference(state, leg_FSM);
        fastConvex.update_cons_matrix();
        Eigen::Matrix<double, DIM_GRF, 1> qp_solution = fastConvex.compute_grfs(state);
        for (int i = 0; i < NUM_LEG; ++i) {
            foot_forces_grf_world.block<3, 1>(0, i) = qp_solution.segment<3>(i * 3);
        }
        return true;
    }
    LeggedContactFSM leg_FSM[NUM_LEG];
    ConvexQPSolver fastConvex;
    Eigen::Matrix<double, 3, NUM_LEG> foot_forces_grf_world;
};
}  // namespace legged

using namespace legged;

int main(int argc, char** argv) {
    const int ticks = argc > 1 ? std::atoi(argv[1]) : 3;
    LeggedState state;
    const double q[12] = {50.0, 100.0, 0.0, 0.0, 0.0, 3500.0, 0.01, 0.01, 10.0, 15.0, 15.0, 20.0};  // Go1 sim YAML
    for (int i = 0; i < 12; ++i) {
        state.param.q_weights[i] = q[i];
        state.param.r_weights[i] = 1e-4;
    }
    const double I[3] = {0.0158533, 0.0377999, 0.0456542};
    for (int i = 0; i < 3; ++i) state.param.a1_trunk_inertia(i, i) = I[i];
    const double feet[4][3] = {{0.17, 0.12, -0.3}, {0.17, -0.17, -0.3}, {-0.17, 0.17, -0.3}, {-0.17, -0.12, -0.3}};
    for (int leg = 0; leg < 4; ++leg)
        for (int k = 0; k < 3; ++k) state.fbk.foot_pos_abs(k, leg) = feet[leg][k];
    state.fbk.root_pos[2] = 0.28;
    state.ctrl.root_pos_d[2] = 0.28;
    ConvexMpc mpc(state);
    for (int tick = 0; tick < ticks; ++tick) {
        for (int i = 0; i < NUM_LEG; ++i) {
            mpc.leg_FSM[i].set_phase(std::fmod(0.1 + 0.04 * tick, 1.0));
            state.ctrl.plan_contacts[i] = mpc.leg_FSM[i].get_contact_state();
        }
        state.fbk.root_pos[0] = 0.004 * tick;
        state.fbk.root_lin_vel[0] = 0.4;
        state.ctrl.root_lin_vel_d_rel[0] = 0.4;
        state.ctrl.root_ang_vel_d_rel[2] = 0.1;
        state.fbk.root_euler[2] = 0.02 * tick;
        const double c = std::cos(state.fbk.root_euler[2]), s = std::sin(state.fbk.root_euler[2]);
        state.fbk.root_rot_mat(0, 0) = c; state.fbk.root_rot_mat(0, 1) = -s;
        state.fbk.root_rot_mat(1, 0) = s; state.fbk.root_rot_mat(1, 1) = c;
        state.fbk.root_rot_mat(2, 2) = 1.0;
        mpc.grf_update(state, 0.01 * tick, 0.01);
        if (mpc.fastConvex.last_error() != LMPC_OK) {
            std::fprintf(stderr, "solve failed: %s\n", lmpc_strerror(mpc.fastConvex.last_error()));
            return 3;
        }
        // the checker's copy of the record (the same restatement the adapter called)
        lmpc_params p;
        lmpc_params_go1(&p);
        for (int i = 0; i < 12; ++i) {
            p.q_weights[i] = q[i];
            p.r_weights[i] = 1e-4;
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
        for (int leg = 0; leg < 4; ++leg)
            for (int k = 0; k < 3; ++k) st.foot_pos_abs[3 * leg + k] = state.fbk.foot_pos_abs(k, leg);
        const int H = PLAN_HORIZON, rl = lmpc_record_len(H);
        double* rec = new double[rl];
        double vdw[3];
        lmpc_pack_record(&p, H, &st, rec, vdw);
        std::printf("tick %d status %d\nrec", tick, mpc.fastConvex.last_status());
        for (int i = 0; i < rl; ++i) std::printf(" %.17g", rec[i]);
        std::printf("\ncontact");
        for (int i = 0; i < H; ++i)
            for (int j = 0; j < NUM_LEG; ++j)
                std::printf(" %d", i == 0 ? (int)state.ctrl.plan_contacts[j]
                                          : (int)(mpc.leg_FSM[j].predict_contact_state(i * 0.01) == STANCE));
        std::printf("\nvdw %.17g %.17g %.17g", state.ctrl.root_lin_vel_d_world[0], state.ctrl.root_lin_vel_d_world[1],
                    state.ctrl.root_lin_vel_d_world[2]);
        std::printf("\nu0");
        for (int leg = 0; leg < NUM_LEG; ++leg)
            for (int k = 0; k < 3; ++k) std::printf(" %.17g", mpc.foot_forces_grf_world(k, leg));
        std::printf("\n");
        delete[] rec;
    }
    return 0;
}

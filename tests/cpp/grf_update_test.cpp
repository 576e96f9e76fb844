// Drives legged::ConvexQPSolver the way ConvexMpc::grf_update does
// (src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexMpc.cpp:6-22,64-108) for a few
// ticks, printing the packed record, the contact schedule and the solution so
// tests/test_gpu_parity.py can check them against the CPU oracle.
// Usage: grf_update_test <horizon> <ticks>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "lmpc/ConvexQPSolver.hpp"

using namespace legged;

int main(int argc, char** argv) {
    const int H = argc > 1 ? std::atoi(argv[1]) : 10;
    const int ticks = argc > 2 ? std::atoi(argv[2]) : 3;
    LeggedState state;
    // A1 sim weights (gazebo_a1_convex.yaml:40-72)
    const double q[12] = {60.0, 100.0, 0.0, 0.0, 0.0, 450.0, 0.15, 0.15, 100.0, 3.0, 3.0, 5.0};
    for (int i = 0; i < 12; ++i) {
        state.param.q_weights[i] = q[i];
        state.param.r_weights[i] = 1e-4;
    }
    state.param.gait_counter_speed = 3.5;
    const double feet[12] = {0.17, 0.17, -0.3, 0.17, -0.17, -0.3, -0.17, 0.17, -0.3, -0.17, -0.17, -0.3};
    for (int i = 0; i < 12; ++i) state.fbk.foot_pos_abs[i] = feet[i];
    state.fbk.root_pos[2] = 0.30;
    state.ctrl.root_pos_d[2] = 0.30;

    // ConvexMpc ctor
    LeggedContactFSM leg_FSM[NUM_LEG];
    for (int i = 0; i < NUM_LEG; ++i) leg_FSM[i].reset_params(state, i);
    ConvexQPSolver fastConvex;
    fastConvex = ConvexQPSolver(state.param.q_weights, state.param.r_weights, H);
    if (fastConvex.last_error() != LMPC_OK) {
        std::fprintf(stderr, "create failed: %s\n", lmpc_strerror(fastConvex.last_error()));
        return 2;
    }
    const int rl = lmpc_record_len(H);
    for (int tick = 0; tick < ticks; ++tick) {
        // movement_mode 0 -> reset FSMs, all plan_contacts true (ConvexMpc.cpp:86-92);
        // later ticks: trotting with perturbed state
        if (tick == 0) {
            for (int i = 0; i < NUM_LEG; ++i) {
                leg_FSM[i].reset();
                state.ctrl.plan_contacts[i] = true;
            }
        } else {
            for (int i = 0; i < NUM_LEG; ++i) {
                leg_FSM[i].advance(0.01 * 7 * tick);
                state.ctrl.plan_contacts[i] = leg_FSM[i].get_contact_state() == STANCE;
            }
            state.fbk.root_lin_vel[0] = 0.1 * tick;
            state.ctrl.root_lin_vel_d_rel[0] = 0.5;
            state.ctrl.root_ang_vel_d_rel[2] = 0.2;
            state.fbk.root_euler[2] = 0.05 * tick;
            const double c = std::cos(state.fbk.root_euler[2]), s = std::sin(state.fbk.root_euler[2]);
            const double R[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
            for (int i = 0; i < 9; ++i) state.fbk.root_rot_mat[i] = R[i];
        }
        // ConvexMpc::grf_update
        fastConvex.calc_mpc_reference(state, leg_FSM);
        fastConvex.update_cons_matrix();
        std::array<double, DIM_GRF> qp_solution = fastConvex.compute_grfs(state);
        if (fastConvex.last_error() != LMPC_OK) {
            std::fprintf(stderr, "solve failed: %s\n", lmpc_strerror(fastConvex.last_error()));
            return 3;
        }
        // re-pack the record exactly as the solver did, for the checker
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
        }
        for (int i = 0; i < 9; ++i) st.root_rot_mat[i] = state.fbk.root_rot_mat[i];
        for (int i = 0; i < 12; ++i) st.foot_pos_abs[i] = state.fbk.foot_pos_abs[i];
        double* rec = new double[rl];
        lmpc_pack_record(&p, H, &st, rec, nullptr);
        std::printf("tick %d status %d\nrec", tick, fastConvex.last_status());
        for (int i = 0; i < rl; ++i) std::printf(" %.17g", rec[i]);
        std::printf("\ncontact");
        for (int i = 0; i < H; ++i)
            for (int j = 0; j < NUM_LEG; ++j)
                std::printf(" %d", i == 0 ? (int)state.ctrl.plan_contacts[j]
                                          : (int)(leg_FSM[j].predict_contact_state(i * 0.01) == STANCE));
        std::printf("\ngrf");
        for (double v : fastConvex.last_solution()) std::printf(" %.17g", v);
        std::printf("\nu0");
        for (double v : qp_solution) std::printf(" %.17g", v);
        std::printf("\n");
        delete[] rec;
    }
    return 0;
}

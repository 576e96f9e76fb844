// Dev tool (GPU): wall-clock latency of one MPC tick through the C++ drop-in, exactly the reference's call
// sequence (ConvexMpc.cpp:70-72): calc_mpc_reference -> update_cons_matrix -> compute_grfs, one QP per tick
// (host state in, u0 out: H2D + kernels + D2H).  Usage: tick_latency <horizon> <ticks>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "lmpc/ConvexQPSolver.hpp"

using namespace legged;

int main(int argc, char** argv) {
    const int H = argc > 1 ? std::atoi(argv[1]) : 10;
    const int ticks = argc > 2 ? std::atoi(argv[2]) : 2000;
    const bool warm = !(argc > 3 && std::string(argv[3]) == "cold");  // default: warm start across ticks
    LeggedState state;
    const double q[12] = {50.0, 100.0, 0.0, 0.0, 0.0, 3500.0, 0.01, 0.01, 10.0, 15.0, 15.0, 20.0};  // Go1 sim
    for (int i = 0; i < 12; ++i) {
        state.param.q_weights[i] = q[i];
        state.param.r_weights[i] = 1e-4;
    }
    state.param.gait_counter_speed = 4.0;
    const double feet[12] = {0.17, 0.12, -0.3, 0.17, -0.17, -0.3, -0.17, 0.17, -0.3, -0.17, -0.12, -0.3};
    for (int i = 0; i < 12; ++i) state.fbk.foot_pos_abs[i] = feet[i];
    state.fbk.root_pos[2] = 0.28;
    state.ctrl.root_pos_d[2] = 0.28;
    LeggedContactFSM leg_FSM[NUM_LEG];
    for (int i = 0; i < NUM_LEG; ++i) leg_FSM[i].reset_params(state, i);
    ConvexQPSolver fastConvex(state.param.q_weights, state.param.r_weights, H);
    if (fastConvex.last_error() != LMPC_OK) {
        std::fprintf(stderr, "create failed: %s\n", lmpc_strerror(fastConvex.last_error()));
        return 2;
    }
    fastConvex.set_warm_start(warm);
    std::vector<double> ms;
    double solves = 0.0;
    int bad = 0;
    for (int tick = 0; tick < ticks + 50; ++tick) {
        for (int i = 0; i < NUM_LEG; ++i) {
            leg_FSM[i].advance(0.01);
            state.ctrl.plan_contacts[i] = leg_FSM[i].get_contact_state() == STANCE;
        }
        state.fbk.root_lin_vel[0] = 0.3 + 0.1 * std::sin(0.05 * tick);
        state.ctrl.root_lin_vel_d_rel[0] = 0.5;
        state.ctrl.root_ang_vel_d_rel[2] = 0.2;
        state.fbk.root_euler[2] = 0.002 * tick;
        const double c = std::cos(state.fbk.root_euler[2]), s = std::sin(state.fbk.root_euler[2]);
        const double R[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
        for (int i = 0; i < 9; ++i) state.fbk.root_rot_mat[i] = R[i];
        const auto t0 = std::chrono::steady_clock::now();
        fastConvex.calc_mpc_reference(state, leg_FSM);
        fastConvex.update_cons_matrix();
        std::array<double, DIM_GRF> u0 = fastConvex.compute_grfs(state);
        const auto t1 = std::chrono::steady_clock::now();
        bad += fastConvex.last_error() != LMPC_OK || fastConvex.last_status() != 0 || !std::isfinite(u0[2]);
        if (tick >= 50) {
            ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            const int it = fastConvex.last_iterations();
            solves += 2 * (it & 0xFFFF) + (it >> 16);  // Riccati solves (cold dual active set: 0 + steps)
        }
    }
    std::sort(ms.begin(), ms.end());
    double mean = 0.0;
    for (double v : ms) mean += v;
    mean /= ms.size();
    std::printf("{\"horizon\": %d, \"warm_start\": %s, \"ticks\": %zu, \"mean_ms\": %.4f, \"median_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"max_ms\": %.4f, \"failed_ticks\": %d, \"mean_riccati_solves\": %.2f}\n",
                H, warm ? "true" : "false", ms.size(), mean, ms[ms.size() / 2], ms[(size_t)(0.99 * ms.size())],
                ms.back(), bad, solves / ms.size());
    return bad ? 3 : 0;
}

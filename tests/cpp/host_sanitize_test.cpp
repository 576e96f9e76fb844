// host_sanitize_test.cpp -- the host-side code of the path under the sanitizers ("ASan/UBSan on
// CPU oracle tests"; race detection of the threaded batch oracle under TSan).  Built and run by
// tests/test_sanitizers.py with g++ -fsanitize=address,undefined (mode "asan") or -fsanitize=thread ("tsan").
//
// asan: the product's host helpers (lmpc_host.cpp: presets, gait FSM, contact schedule, record packing,
//       commands, synthetic generator, terrain frame, GRF -> torque) across every horizon 1..LMPC_MAX_HORIZON,
//       cross-checked against the CPU checker (oracle/lmpc_oracle.c), and the checker's solve on flat and
//       terrain instances with its KKT certificate;
// tsan: the checker's threaded batch solve (bench.py's cpu_baseline leg) against the sequential solve, bitwise.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "lmpc/lmpc.h"
#include "lmpc_oracle.h"

static int g_fail = 0;
#define CHECK(cond, ...)                          \
    do {                                          \
        if (!(cond)) {                            \
            std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);             \
            std::printf("\n");                    \
            ++g_fail;                             \
        }                                         \
    } while (0)

static oracle_params to_oracle(const lmpc_params& p) {
    oracle_params o;
    std::memcpy(o.q_weights, p.q_weights, sizeof(o.q_weights));
    std::memcpy(o.r_weights, p.r_weights, sizeof(o.r_weights));
    o.robot_mass = p.robot_mass;
    std::memcpy(o.trunk_inertia, p.trunk_inertia, sizeof(o.trunk_inertia));
    o.mu = p.mu;
    o.f_max = p.f_max;
    o.gravity = p.gravity;
    o.dt = p.dt;
    return o;
}

static void host_helpers(const lmpc_params& p) {
    // gait FSM: product restatement == checker restatement on a phase grid, every gait and leg
    for (int gait = 0; gait < 4; ++gait)
        for (int leg = 0; leg < 4; ++leg)
            for (int k = 0; k < 200; ++k) {
                const double ph = k / 200.0;
                CHECK(lmpc_current_contact(gait, leg, ph) == oracle_current_contact(gait, leg, ph), "current %d %d", gait, leg);
                for (int i = 0; i < 12; ++i)
                    CHECK(lmpc_predict_contact(gait, leg, ph, 4.0, i * p.dt) ==
                              oracle_predict_contact(gait, leg, ph, 4.0, i * p.dt),
                          "predict %d %d %d", gait, leg, i);
            }
    // records, schedules, commands and the synthetic generator at every horizon the ABI accepts
    lmpc_synth_cfg cfg;
    lmpc_synth_cfg_go1(&cfg);
    for (int H = 1; H <= LMPC_MAX_HORIZON; ++H) {
        const int n = 6, RL = lmpc_record_len(H);
        std::vector<double> rec((size_t)n * RL), rec2((size_t)n * RL);
        std::vector<uint8_t> con((size_t)n * 4 * H), con2((size_t)n * 4 * H);
        std::vector<lmpc_command> cmd(n);
        CHECK(lmpc_synth_fill(&p, &cfg, H, 99, 1000, n, rec.data(), con.data()) == LMPC_OK, "synth H=%d", H);
        CHECK(lmpc_synth_commands(&cfg, 99, 1000, n, cmd.data()) == LMPC_OK, "commands H=%d", H);
        for (int b = 0; b < n; ++b) {
            CHECK(lmpc_command_to_record(&p, H, &cmd[b], rec2.data() + (size_t)b * RL, con2.data() + (size_t)b * 4 * H) ==
                      LMPC_OK, "cmd->rec");
            std::vector<uint8_t> sched(4 * H);
            lmpc_contact_schedule_legs(cmd[b].gait, cmd[b].gait_phase, cmd[b].gait_speed, p.dt, H, cmd[b].plan_contacts,
                                       sched.data());
            CHECK(std::memcmp(sched.data(), con.data() + (size_t)b * 4 * H, 4 * H) == 0, "schedule H=%d b=%d", H, b);
            double vdw[3];
            std::vector<double> r3(RL);
            CHECK(lmpc_pack_record(&p, H, &cmd[b].state, r3.data(), vdw) == LMPC_OK, "pack");
            CHECK(std::memcmp(r3.data(), rec.data() + (size_t)b * RL, RL * sizeof(double)) == 0, "pack != synth");
        }
        CHECK(rec == rec2 && con == con2, "commands -> records != synth_fill at H=%d", H);
        std::vector<double> nrm((size_t)n * 12);
        CHECK(lmpc_synth_normals(7, 0, n, 0.3, nrm.data()) == LMPC_OK, "normals");
        for (int i = 0; i < 4 * n; ++i) {
            double R[9], Ro[9];
            lmpc_terrain_frame(&nrm[3 * i], R);
            oracle_terrain_frame(&nrm[3 * i], Ro);
            for (int e = 0; e < 9; ++e) CHECK(std::fabs(R[e] - Ro[e]) <= 1e-15, "terrain frame");
        }
    }
    // GRF -> joint torque: product (closed-form Jacobian) vs checker (complex-step derivative of fk)
    lmpc_leg_kin kin;
    lmpc_leg_kin_default(&kin);
    for (int t = 0; t < 50; ++t) {
        double rot[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, q[12], f[12], tau[12], tau_o[12];
        const double yaw = 0.1 * t;
        rot[0] = rot[4] = std::cos(yaw);
        rot[1] = -std::sin(yaw);
        rot[3] = std::sin(yaw);
        for (int i = 0; i < 12; ++i) {
            q[i] = 0.3 * std::sin(0.7 * t + i);
            f[i] = 40.0 * std::cos(0.3 * t + 2 * i);
        }
        CHECK(lmpc_grf_to_torque(&kin, rot, q, f, tau) == LMPC_OK, "torque");
        oracle_grf_to_torque(&kin.rho_fix[0][0], &kin.rho_opt[0][0], rot, q, f, tau_o);
        for (int i = 0; i < 12; ++i) CHECK(std::fabs(tau[i] - tau_o[i]) <= 1e-9 * (1 + std::fabs(tau_o[i])), "tau %d", i);
    }
}

static void checker_solves(const lmpc_params& p) {
    const oracle_params op = to_oracle(p);
    lmpc_synth_cfg cfg;
    lmpc_synth_cfg_go1(&cfg);
    for (int H : {10, 30}) {
        const int n = 3, RL = lmpc_record_len(H);
        std::vector<double> rec((size_t)n * RL), grf((size_t)12 * H), nrm((size_t)n * 12);
        std::vector<uint8_t> con((size_t)n * 4 * H);
        lmpc_synth_fill(&p, &cfg, H, 5, 0, n, rec.data(), con.data());
        lmpc_synth_normals(5, 0, n, 0.3, nrm.data());
        for (int b = 0; b < n; ++b) {
            double kkt[4];
            int na = 0;
            CHECK(oracle_solve(&op, H, rec.data() + (size_t)b * RL, con.data() + (size_t)b * 4 * H, grf.data(), kkt, &na) ==
                      0, "solve H=%d", H);
            CHECK(kkt[0] <= 1e-8 && kkt[1] <= 1e-8 && kkt[2] <= 1e-8 && kkt[3] <= 1e-8, "kkt H=%d", H);
            CHECK(oracle_solve_ex(&op, H, rec.data() + (size_t)b * RL, con.data() + (size_t)b * 4 * H, nrm.data() + 12 * b,
                                  grf.data(), kkt, &na) == 0, "terrain solve H=%d", H);
            CHECK(kkt[0] <= 1e-8 && kkt[1] <= 1e-8, "terrain kkt H=%d", H);
        }
    }
}

static void threaded_batch(const lmpc_params& p) {
    const oracle_params op = to_oracle(p);
    lmpc_synth_cfg cfg;
    lmpc_synth_cfg_go1(&cfg);
    cfg.gait = -1;  // mixed gaits
    const int H = 10, n = 48, RL = lmpc_record_len(H);
    std::vector<double> rec((size_t)n * RL), g1((size_t)n * 12 * H), g8((size_t)n * 12 * H), nrm((size_t)n * 12);
    std::vector<uint8_t> con((size_t)n * 4 * H);
    std::vector<int32_t> s1(n), s8(n);
    lmpc_synth_fill(&p, &cfg, H, 11, 0, n, rec.data(), con.data());
    lmpc_synth_normals(11, 0, n, 0.3, nrm.data());
    CHECK(oracle_solve_batch_ex(&op, H, n, rec.data(), con.data(), nrm.data(), g1.data(), s1.data(), 1) == 0, "batch 1");
    CHECK(oracle_solve_batch_ex(&op, H, n, rec.data(), con.data(), nrm.data(), g8.data(), s8.data(), 8) == 0, "batch 8");
    CHECK(g1 == g8 && s1 == s8, "threaded batch differs from the sequential one");
}

int main(int argc, char** argv) {
    const bool tsan = argc > 1 && std::strcmp(argv[1], "tsan") == 0;
    lmpc_params p;
    lmpc_params_go1(&p);
    if (tsan) {
        threaded_batch(p);
    } else {
        lmpc_params a1;
        lmpc_params_a1(&a1);
        lmpc_options o;
        lmpc_options_default(&o);
        CHECK(o.max_iter > 0 && a1.robot_mass > 0.0, "presets");
        host_helpers(p);
        checker_solves(p);
        threaded_batch(p);
    }
    std::printf("%s %s\n", tsan ? "tsan" : "asan+ubsan", g_fail ? "FAILED" : "OK");
    return g_fail ? 1 : 0;
}

// lmpc_host.cpp -- host-side pieces of the convex-MPC QP path that sit either
// side of the device solve: robot presets, the gait-FSM contact schedule, the
// calc_mpc_reference record packing and the synthetic batch generator.
//
// Reference anchors (relative to src/legged_ctrl):
//   presets              config/gazebo_go1_convex.yaml:39-71, config/gazebo_a1_convex.yaml:40-72,133-140,
//                        src/LeggedState.cpp:146,155-160 (mass / inertia defaults)
//   gait tables          src/utils/LeggedContactFSM.cpp:93-212
//   predict_contact      src/utils/LeggedContactFSM.cpp:280-294
//   bound schedule       src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:329-346
//   reference trajectory src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:256-276
#include <cmath>
#include <cstring>

#include "lmpc/lmpc.h"

namespace {

struct GaitTab {
    int size;
    int state[3];
    double sw[3];
};

GaitTab gait_table(int gait, int leg) {
    GaitTab t{};
    switch (gait) {
    case LMPC_GAIT_CRAWL:  // LeggedContactFSM.cpp:158-199
        if (leg == 0) t = {2, {0, 1, 0}, {0.25, 1.0, 0.0}};
        else if (leg == 1) t = {3, {1, 0, 1}, {0.25, 0.5, 1.0}};
        else if (leg == 2) t = {3, {1, 0, 1}, {0.5, 0.75, 1.0}};
        else t = {2, {1, 0, 0}, {0.75, 1.0, 0.0}};
        break;
    case LMPC_GAIT_TROT_WITH_STAND:  // LeggedContactFSM.cpp:116-156
        if (leg == 0 || leg == 3) t = {2, {1, 0, 0}, {0.6, 1.0, 0.0}};
        else t = {3, {1, 0, 1}, {0.1, 0.5, 1.0}};
        break;
    case LMPC_GAIT_STAND:  // LeggedContactFSM.cpp:201-212
        t = {1, {1, 0, 0}, {1.0, 0.0, 0.0}};
        break;
    default:  // trot, LeggedContactFSM.cpp:93-114
        if (leg == 0 || leg == 3) t = {2, {1, 0, 0}, {0.5, 1.0, 0.0}};
        else t = {2, {0, 1, 0}, {0.5, 1.0, 0.0}};
        break;
    }
    return t;
}

// ---- Philox4x32-10 counter-based generator --------------------------------
struct Philox {
    uint32_t key[2];
    uint32_t ctr[4];
    uint32_t out[4];
    int used;

    Philox(uint64_t seed, uint64_t index, uint32_t stream = 0x4c4d5043u /* "LMPC" */) {
        key[0] = (uint32_t)seed;
        key[1] = (uint32_t)(seed >> 32);
        ctr[0] = (uint32_t)index;
        ctr[1] = (uint32_t)(index >> 32);
        ctr[2] = 0;
        ctr[3] = stream;
        used = 4;
    }
    void block() {
        uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
        uint32_t k0 = key[0], k1 = key[1];
        for (int r = 0; r < 10; ++r) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
            const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
            const uint32_t n1 = (uint32_t)p1;
            const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
            const uint32_t n3 = (uint32_t)p0;
            c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        for (int i = 0; i < 4; ++i) out[i] = c[i];
        ctr[2]++;
        used = 0;
    }
    uint32_t next32() {
        if (used >= 4) block();
        return out[used++];
    }
    // uniform in [0,1) with 53 random bits
    double uniform() {
        const uint32_t a = next32() >> 5, b = next32() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    double uniform(double lo, double hi) { return lo + (hi - lo) * uniform(); }
    double normal(double sigma) {
        const double u1 = 1.0 - uniform();  // (0,1]
        const double u2 = uniform();
        return sigma * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

void euler_zyx_to_rot(double roll, double pitch, double yaw, double R[9]) {
    const double cr = std::cos(roll), sr = std::sin(roll);
    const double cp = std::cos(pitch), sp = std::sin(pitch);
    const double cy = std::cos(yaw), sy = std::sin(yaw);
    // R = Rz(yaw) * Ry(pitch) * Rx(roll)
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

}  // namespace

extern "C" {

void lmpc_params_go1(lmpc_params* p) {
    static const double q[12] = {50.0, 100.0, 0.0, 0.0, 0.0, 3500.0, 0.01, 0.01, 10.0, 15.0, 15.0, 20.0};
    std::memset(p, 0, sizeof(*p));
    for (int i = 0; i < 12; ++i) {
        p->q_weights[i] = q[i];
        p->r_weights[i] = 1e-4;
    }
    p->robot_mass = 13.0;  // LeggedState.cpp:146 default (the Go1 sim YAML omits it)
    p->trunk_inertia[0] = 0.0158533;
    p->trunk_inertia[4] = 0.0377999;
    p->trunk_inertia[8] = 0.0456542;
    p->mu = 0.3;
    p->f_max = 180.0;
    p->gravity = 9.8;
    p->dt = 10.0 / 1000.0;
}

void lmpc_params_a1(lmpc_params* p) {
    static const double q[12] = {60.0, 100.0, 0.0, 0.0, 0.0, 450.0, 0.15, 0.15, 100.0, 3.0, 3.0, 5.0};
    lmpc_params_go1(p);
    for (int i = 0; i < 12; ++i) p->q_weights[i] = q[i];
}

void lmpc_options_default(lmpc_options* o) {
    o->max_iter = 40;
    o->max_rounds = 4;
    o->max_attempts = 3;
    o->tol_mu = 1e-8;
    o->tol_p = 1e-9;
    o->tol_d = 1e-9;
}

int lmpc_record_len(int horizon) { return 33 + 12 * horizon; }
int lmpc_abi_version(void) { return LMPC_ABI_VERSION; }

const char* lmpc_strerror(int code) {
    switch (code) {
    case LMPC_OK: return "ok";
    case LMPC_ERR_ARG: return "invalid argument";
    case LMPC_ERR_DEVICE: return "HIP device error";
    case LMPC_ERR_ALLOC: return "device allocation failed";
    case LMPC_ERR_LAUNCH: return "kernel launch failed";
    case LMPC_ERR_NOT_BUILT: return "device code not available for this GPU";
    default: return "unknown error";
    }
}

int lmpc_predict_contact(int gait, int leg, double gait_phase, double gait_speed, double dt) {
    const GaitTab t = gait_table(gait, leg);
    double ph = gait_phase + gait_speed * dt;
    while (ph > 1.0) ph -= 1.0;
    for (int i = 0; i < t.size; ++i)
        if (ph <= t.sw[i]) return t.state[i];
    return 1;  // "should not reach here" -> STANCE
}

int lmpc_current_contact(int gait, int leg, double gait_phase) {
    const GaitTab t = gait_table(gait, leg);
    for (int i = 0; i < t.size; ++i)
        if (gait_phase < t.sw[i]) return t.state[i];
    return t.state[t.size - 1];
}

int lmpc_contact_schedule(int gait, double gait_phase, double gait_speed, double dt, int horizon,
                          const uint8_t plan_contacts[4], uint8_t* contact) {
    if (horizon < 1 || !plan_contacts || !contact) return LMPC_ERR_ARG;
    for (int j = 0; j < 4; ++j) contact[j] = plan_contacts[j] ? 1 : 0;
    for (int i = 1; i < horizon; ++i)
        for (int j = 0; j < 4; ++j)
            contact[4 * i + j] = (uint8_t)lmpc_predict_contact(gait, j, gait_phase, gait_speed, i * dt);
    return LMPC_OK;
}

int lmpc_pack_record(const lmpc_params* p, int horizon, const lmpc_state_in* st, double* rec,
                     double lin_vel_d_world[3]) {
    if (!p || !st || !rec || horizon < 1) return LMPC_ERR_ARG;
    double* x0 = rec + LMPC_REC_X0;
    for (int k = 0; k < 3; ++k) {
        x0[k] = st->root_euler[k];
        x0[3 + k] = st->root_pos[k];
        x0[6 + k] = st->root_ang_vel[k];
        x0[9 + k] = st->root_lin_vel[k];
    }
    std::memcpy(rec + LMPC_REC_ROT, st->root_rot_mat, 9 * sizeof(double));
    std::memcpy(rec + LMPC_REC_FEET, st->foot_pos_abs, 12 * sizeof(double));
    // root_lin_vel_d_world = root_rot_mat * root_lin_vel_d_rel (ConvexQPSolver.cpp:260)
    double vdw[3];
    for (int r = 0; r < 3; ++r)
        vdw[r] = st->root_rot_mat[3 * r + 0] * st->root_lin_vel_d_rel[0] +
                 st->root_rot_mat[3 * r + 1] * st->root_lin_vel_d_rel[1] +
                 st->root_rot_mat[3 * r + 2] * st->root_lin_vel_d_rel[2];
    if (lin_vel_d_world)
        for (int r = 0; r < 3; ++r) lin_vel_d_world[r] = vdw[r];
    const double dt = p->dt;
    for (int i = 0; i < horizon; ++i) {  // ConvexQPSolver.cpp:262-276
        double* xr = rec + LMPC_REC_XREF + 12 * i;
        xr[0] = st->root_euler_d[0];
        xr[1] = st->root_euler_d[1];
        xr[2] = st->root_euler[2] + st->root_ang_vel_d_rel[2] * dt * (i);
        xr[3] = st->root_pos[0] + vdw[0] * dt * (i);
        xr[4] = st->root_pos[1] + vdw[1] * dt * (i);
        xr[5] = st->root_pos_d[2];
        xr[6] = st->root_ang_vel_d_rel[0];
        xr[7] = st->root_ang_vel_d_rel[1];
        xr[8] = st->root_ang_vel_d_rel[2];
        xr[9] = vdw[0];
        xr[10] = vdw[1];
        xr[11] = 0.0;
    }
    return LMPC_OK;
}

void lmpc_synth_cfg_go1(lmpc_synth_cfg* c) {
    // gazebo_go1_convex.yaml:18-35
    static const double feet[12] = {0.17, 0.12, -0.3, 0.17, -0.17, -0.3, -0.17, 0.17, -0.3, -0.17, -0.12, -0.3};
    std::memset(c, 0, sizeof(*c));
    c->gait = LMPC_GAIT_TROT;
    c->gait_speed = 4.0;
    std::memcpy(c->default_feet, feet, sizeof(feet));
    c->standing = 0;
}

void lmpc_synth_cfg_a1_standing(lmpc_synth_cfg* c) {
    // gazebo_a1_convex.yaml:19-36
    static const double feet[12] = {0.17, 0.17, -0.3, 0.17, -0.17, -0.3, -0.17, 0.17, -0.3, -0.17, -0.17, -0.3};
    std::memset(c, 0, sizeof(*c));
    c->gait = LMPC_GAIT_TROT;
    c->gait_speed = 3.5;
    std::memcpy(c->default_feet, feet, sizeof(feet));
    c->standing = 1;
}

int lmpc_synth_fill(const lmpc_params* p, const lmpc_synth_cfg* cfg, int horizon, uint64_t seed,
                    int64_t first_index, int count, double* rec, uint8_t* contact) {
    if (!p || !cfg || !rec || !contact || horizon < 1 || count < 0) return LMPC_ERR_ARG;
    const int rl = lmpc_record_len(horizon);
    for (int b = 0; b < count; ++b) {
        lmpc_state_in st;
        std::memset(&st, 0, sizeof(st));
        double phase = 0.0;
        int gait = cfg->gait < 0 ? LMPC_GAIT_TROT : cfg->gait;
        uint8_t plan[4] = {1, 1, 1, 1};
        if (cfg->standing) {
            // config 1: x0=[0,0,0, 0,0,0.30, 0..], z_d = 0.30, v_d = 0, all plan_contacts = 1,
            // FSM reset (phase 0): ConvexMpc.cpp:86-92 standing mode.
            st.root_pos[2] = 0.30;
            st.root_pos_d[2] = 0.30;
            euler_zyx_to_rot(0.0, 0.0, 0.0, st.root_rot_mat);
            for (int j = 0; j < 12; ++j) st.foot_pos_abs[j] = cfg->default_feet[j];
        } else {
            Philox rng(seed, (uint64_t)(first_index + b));
            const double roll = rng.uniform(-0.2, 0.2);
            const double pitch = rng.uniform(-0.2, 0.2);
            const double yaw = rng.uniform(-M_PI, M_PI);
            st.root_euler[0] = roll;
            st.root_euler[1] = pitch;
            st.root_euler[2] = yaw;
            st.root_pos[0] = rng.uniform(-1.0, 1.0);
            st.root_pos[1] = rng.uniform(-1.0, 1.0);
            st.root_pos[2] = rng.uniform(0.20, 0.35);
            for (int k = 0; k < 3; ++k) st.root_ang_vel[k] = rng.normal(0.3);
            st.root_lin_vel[0] = rng.uniform(-1.0, 1.0);
            st.root_lin_vel[1] = rng.uniform(-1.0, 1.0);
            st.root_lin_vel[2] = rng.normal(0.1);
            st.root_pos_d[2] = rng.uniform(0.25, 0.32);
            st.root_lin_vel_d_rel[0] = rng.uniform(-1.0, 1.0);
            st.root_lin_vel_d_rel[1] = rng.uniform(-0.4, 0.4);
            st.root_ang_vel_d_rel[2] = rng.uniform(-0.8, 0.8);
            euler_zyx_to_rot(roll, pitch, yaw, st.root_rot_mat);
            const double* R = st.root_rot_mat;
            for (int j = 0; j < 4; ++j) {
                double rel[3];
                for (int k = 0; k < 3; ++k) rel[k] = cfg->default_feet[3 * j + k] + rng.uniform(-0.03, 0.03);
                for (int r = 0; r < 3; ++r)
                    st.foot_pos_abs[3 * j + r] = R[3 * r] * rel[0] + R[3 * r + 1] * rel[1] + R[3 * r + 2] * rel[2];
            }
            phase = rng.uniform();
            if (cfg->gait < 0) gait = (int)(rng.uniform() * 4.0) & 3;
            for (int j = 0; j < 4; ++j) plan[j] = (uint8_t)lmpc_current_contact(gait, j, phase);
        }
        double* r = rec + (size_t)b * rl;
        lmpc_pack_record(p, horizon, &st, r, nullptr);
        lmpc_contact_schedule(gait, phase, cfg->gait_speed, p->dt, horizon, plan,
                              contact + (size_t)b * 4 * horizon);
    }
    return LMPC_OK;
}

void lmpc_terrain_frame(const double nin[3], double R[9]) {
    // minimal rotation e_z -> n (Rodrigues about e_z x n, closed form); n = e_z gives I exactly
    const double nn = std::sqrt(nin[0] * nin[0] + nin[1] * nin[1] + nin[2] * nin[2]);
    const double nx = nin[0] / nn, ny = nin[1] / nn, c = nin[2] / nn;
    const double h = 1.0 / (1.0 + c);
    R[0] = 1.0 - nx * nx * h; R[1] = -nx * ny * h;      R[2] = nx;
    R[3] = -nx * ny * h;      R[4] = 1.0 - ny * ny * h; R[5] = ny;
    R[6] = -nx;               R[7] = -ny;               R[8] = c;
}

int lmpc_synth_normals(uint64_t seed, int64_t first_index, int count, double theta_max, double* normals) {
    if (!normals || count < 0 || !(theta_max >= 0.0) || theta_max >= 1.5707963267948966) return LMPC_ERR_ARG;
    for (int b = 0; b < count; ++b) {
        Philox rng(seed, (uint64_t)(first_index + b), 0x54455252u /* "TERR" */);
        for (int j = 0; j < 4; ++j) {
            const double th = rng.uniform(0.0, theta_max);
            const double ph = rng.uniform(-M_PI, M_PI);
            double* n = normals + (size_t)b * 12 + 3 * j;
            n[0] = std::sin(th) * std::cos(ph);
            n[1] = std::sin(th) * std::sin(ph);
            n[2] = std::cos(th);
        }
    }
    return LMPC_OK;
}

}  // extern "C"

// lmpc_common.h -- the pieces of the path that run on BOTH sides of the device solve, written once
// and compiled for the host (lmpc_host.cpp) and for gfx950 (lmpc_prep.hip):
//
//   gait tables + FSM prediction   LeggedContactFSM.cpp:93-212, 280-294
//   bound schedule                 ConvexQPSolver.cpp:329-346
//   reference trajectory / x0      ConvexQPSolver.cpp:256-276
//   synthetic commands             SURVEY.md 8d (Philox4x32-10 keyed by (seed, global index))
//
// Floating-point contraction is switched off in every function of this header (LMPC_NO_FMA) so the host (x86-64, no FMA) and the
// device (FMA-capable) evaluate every non-transcendental expression identically: a command expands
// to a bit-identical record on either side.  Only the synthetic generator's sin/cos/log/sqrt come
// from different libraries (glibc vs the device math library), so device-generated commands match
// the host generator to a few ulp.
#pragma once
#include <cmath>
#include <cstdint>

#include "lmpc/lmpc.h"

#if defined(__HIPCC__)
#define LMPC_HD __host__ __device__
#else
#define LMPC_HD
#endif
// first statement of every function body below that does arithmetic: no a*b+c fusion in this block
#define LMPC_NO_FMA _Pragma("clang fp contract(off)")

static_assert(sizeof(lmpc_command) == 408, "lmpc_command layout (mirrored by _native.LmpcCommand)");

namespace lmpc_common {

struct GaitTab {
    int size;
    int state[3];
    double sw[3];
};

// LeggedContactFSM gait patterns: per leg, `size` phases, each (state, switch time)
LMPC_HD inline GaitTab gait_table(int gait, int leg) {
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

// predict_contact_state (LeggedContactFSM.cpp:280-294): 1 = STANCE, 0 = SWING
LMPC_HD inline int predict_contact(int gait, int leg, double gait_phase, double gait_speed, double dt) {
    LMPC_NO_FMA
    const GaitTab t = gait_table(gait, leg);
    double ph = gait_phase + gait_speed * dt;
    while (ph > 1.0) ph -= 1.0;
    for (int i = 0; i < t.size; ++i)
        if (ph <= t.sw[i]) return t.state[i];
    return 1;  // "should not reach here" -> STANCE
}

// FSM state once it has advanced to gait_phase (get_contact_state())
LMPC_HD inline int current_contact(int gait, int leg, double gait_phase) {
    const GaitTab t = gait_table(gait, leg);
    for (int i = 0; i < t.size; ++i)
        if (gait_phase < t.sw[i]) return t.state[i];
    return t.state[t.size - 1];
}

// contact[i][j] of the bound schedule (ConvexQPSolver.cpp:329-346): leg j predicted from its own FSM's phase
// (ConvexQPSolver.cpp:341-342, LeggedContactFSM.h:64)
LMPC_HD inline uint8_t contact_element(const lmpc_command& c, double dt, int i, int j) {
    LMPC_NO_FMA
    if (i == 0) return c.plan_contacts[j] ? 1 : 0;
    return (uint8_t)predict_contact(c.gait, j, c.gait_phase[j], c.gait_speed, i * dt);
}

// root_lin_vel_d_world = root_rot_mat * root_lin_vel_d_rel, component r (ConvexQPSolver.cpp:260)
LMPC_HD inline double vd_world(const lmpc_state_in& st, int r) {
    LMPC_NO_FMA
    return st.root_rot_mat[3 * r + 0] * st.root_lin_vel_d_rel[0] + st.root_rot_mat[3 * r + 1] * st.root_lin_vel_d_rel[1] +
           st.root_rot_mat[3 * r + 2] * st.root_lin_vel_d_rel[2];
}

// element e of the packed record [x0(12) | R(9) | feet(12) | x_ref(H x 12)] (ConvexQPSolver.cpp:256-276)
LMPC_HD inline double record_element(const lmpc_state_in& st, double dt, int e) {
    LMPC_NO_FMA
    if (e < 12) {
        const int k = e % 3;
        switch (e / 3) {
        case 0: return st.root_euler[k];
        case 1: return st.root_pos[k];
        case 2: return st.root_ang_vel[k];
        default: return st.root_lin_vel[k];
        }
    }
    if (e < LMPC_REC_FEET) return st.root_rot_mat[e - LMPC_REC_ROT];
    if (e < LMPC_REC_XREF) return st.foot_pos_abs[e - LMPC_REC_FEET];
    const int i = (e - LMPC_REC_XREF) / 12, r = (e - LMPC_REC_XREF) % 12;
    switch (r) {
    case 0: return st.root_euler_d[0];
    case 1: return st.root_euler_d[1];
    case 2: return st.root_euler[2] + st.root_ang_vel_d_rel[2] * dt * (i);
    case 3: return st.root_pos[0] + vd_world(st, 0) * dt * (i);
    case 4: return st.root_pos[1] + vd_world(st, 1) * dt * (i);
    case 5: return st.root_pos_d[2];
    case 6: return st.root_ang_vel_d_rel[0];
    case 7: return st.root_ang_vel_d_rel[1];
    case 8: return st.root_ang_vel_d_rel[2];
    case 9: return vd_world(st, 0);
    case 10: return vd_world(st, 1);
    default: return 0.0;
    }
}

// ---- Philox4x32-10 counter-based generator --------------------------------
struct Philox {
    uint32_t key[2];
    uint32_t ctr[4];
    uint32_t out[4];
    int used;

    LMPC_HD Philox(uint64_t seed, uint64_t index, uint32_t stream = 0x4c4d5043u /* "LMPC" */) {
        key[0] = (uint32_t)seed;
        key[1] = (uint32_t)(seed >> 32);
        ctr[0] = (uint32_t)index;
        ctr[1] = (uint32_t)(index >> 32);
        ctr[2] = 0;
        ctr[3] = stream;
        used = 4;
    }
    LMPC_HD void block() {
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
    LMPC_HD uint32_t next32() {
        if (used >= 4) block();
        return out[used++];
    }
    // uniform in [0,1) with 53 random bits
    LMPC_HD double uniform() {
        LMPC_NO_FMA
        const uint32_t a = next32() >> 5, b = next32() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    LMPC_HD double uniform(double lo, double hi) {
        LMPC_NO_FMA
        return lo + (hi - lo) * uniform();
    }
    LMPC_HD double normal(double sigma) {
        LMPC_NO_FMA
        const double u1 = 1.0 - uniform();  // (0,1]
        const double u2 = uniform();
        return sigma * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    }
};

// R = Rz(yaw) Ry(pitch) Rx(roll), row-major (the ZYX convention Utils::quat_to_euler inverts)
LMPC_HD inline void euler_zyx_to_rot(double roll, double pitch, double yaw, double R[9]) {
    LMPC_NO_FMA
    const double cr = cos(roll), sr = sin(roll);
    const double cp = cos(pitch), sp = sin(pitch);
    const double cy = cos(yaw), sy = sin(yaw);
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

// Synthetic command of global instance `index` (SURVEY.md 8d distributions)
LMPC_HD inline void synth_command(const lmpc_synth_cfg& cfg, uint64_t seed, uint64_t index, lmpc_command& c) {
    LMPC_NO_FMA
    lmpc_state_in& st = c.state;
    for (int k = 0; k < 3; ++k) {
        st.root_euler[k] = st.root_pos[k] = st.root_ang_vel[k] = st.root_lin_vel[k] = 0.0;
        st.root_euler_d[k] = st.root_pos_d[k] = st.root_lin_vel_d_rel[k] = st.root_ang_vel_d_rel[k] = 0.0;
    }
    for (int j = 0; j < 4; ++j) c.gait_phase[j] = 0.0;
    c.gait_speed = cfg.gait_speed;
    c.gait = cfg.gait < 0 ? LMPC_GAIT_TROT : cfg.gait;
    for (int j = 0; j < 4; ++j) c.plan_contacts[j] = 1;
    if (cfg.standing) {
        // config 1: x0=[0,0,0, 0,0,0.30, 0..], z_d = 0.30, v_d = 0, all plan_contacts = 1,
        // FSM reset (phase 0): ConvexMpc.cpp:86-92 standing mode.
        st.root_pos[2] = 0.30;
        st.root_pos_d[2] = 0.30;
        euler_zyx_to_rot(0.0, 0.0, 0.0, st.root_rot_mat);
        for (int j = 0; j < 12; ++j) st.foot_pos_abs[j] = cfg.default_feet[j];
        return;
    }
    Philox rng(seed, index);
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
        for (int k = 0; k < 3; ++k) rel[k] = cfg.default_feet[3 * j + k] + rng.uniform(-0.03, 0.03);
        for (int r = 0; r < 3; ++r)
            st.foot_pos_abs[3 * j + r] = R[3 * r] * rel[0] + R[3 * r + 1] * rel[1] + R[3 * r + 2] * rel[2];
    }
    // one phase for the four legs (the FSMs of a synthetic instance are in step: no early touchdowns)
    const double ph = rng.uniform();
    for (int j = 0; j < 4; ++j) c.gait_phase[j] = ph;
    if (cfg.gait < 0) c.gait = (int)(rng.uniform() * 4.0) & 3;
    for (int j = 0; j < 4; ++j) c.plan_contacts[j] = (uint8_t)current_contact(c.gait, j, c.gait_phase[j]);
}

// Terrain normals of instance `index`, leg j (own Philox stream "TERR")
LMPC_HD inline void synth_normals(uint64_t seed, uint64_t index, double theta_max, double n[12]) {
    LMPC_NO_FMA
    Philox rng(seed, index, 0x54455252u);
    for (int j = 0; j < 4; ++j) {
        const double th = rng.uniform(0.0, theta_max);
        const double ph = rng.uniform(-M_PI, M_PI);
        n[3 * j + 0] = sin(th) * cos(ph);
        n[3 * j + 1] = sin(th) * sin(ph);
        n[3 * j + 2] = cos(th);
    }
}

// ---- GRF -> joint torque (BaseInterface.cpp:451-459) ---------------------
// Foot position of the abduction/hip/knee chain in the body frame, for rho = (rho_fix, rho_opt):
//   h(q1,q2) = L1 cos q1 + b cos(q1+q2) + a sin(q1+q2)   (leg extension in the sagittal plane)
//   p = [ox - L1 sin q1 - b sin(q1+q2) + a cos(q1+q2),  oy + d cos q0 + h sin q0,  d sin q0 - h cos q0]
// with a = rho_opt[0], b = L2 - rho_opt[2], d = motor_offset + rho_opt[1] -- the model
// A1Kinematics::fk (A1Kinematics.cpp:8-12,38-72) evaluates.  J = dp/dq in closed form:
LMPC_HD inline void foot_jacobian(const double rf[5], const double ro[3], const double q[3], double J[9]) {
    LMPC_NO_FMA
    const double L1 = rf[3], a = ro[0], b = rf[4] - ro[2], d = rf[2] + ro[1];
    const double s0 = sin(q[0]), c0 = cos(q[0]);
    const double s1 = sin(q[1]), c1 = cos(q[1]);
    const double s12 = sin(q[1] + q[2]), c12 = cos(q[1] + q[2]);
    const double h2 = b * c12 + a * s12;   // knee part of h
    const double g2 = a * c12 - b * s12;   // d h2 / d q2
    const double h = L1 * c1 + h2;
    const double g = g2 - L1 * s1;         // d h / d q1
    J[0] = 0.0;                 J[1] = -h;       J[2] = -h2;
    J[3] = c0 * h - d * s0;     J[4] = s0 * g;   J[5] = s0 * g2;
    J[6] = d * c0 + s0 * h;     J[7] = -c0 * g;  J[8] = -c0 * g2;
}

// tau_leg = -J' (R' f_world) for one leg (rot row-major)
LMPC_HD inline void leg_torque(const double rf[5], const double ro[3], const double rot[9], const double q[3],
                               const double f[3], double tau[3]) {
    LMPC_NO_FMA
    double fr[3], J[9];
    for (int r = 0; r < 3; ++r) fr[r] = rot[r] * f[0] + rot[3 + r] * f[1] + rot[6 + r] * f[2];
    foot_jacobian(rf, ro, q, J);
    for (int c = 0; c < 3; ++c) tau[c] = -(J[c] * fr[0] + J[3 + c] * fr[1] + J[6 + c] * fr[2]);
}

}  // namespace lmpc_common

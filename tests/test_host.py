"""CPU tests of the product's host-side path helpers: record packing
(calc_mpc_reference), contact schedule (update_bound_constraints + FSM) and the
seeded synthetic generator.  No GPU calls."""
import ctypes

import numpy as np
import pytest

from conftest import fsm_commands, golden_files, load_golden

from legged_mpc_control_amd import _native as N
from legged_mpc_control_amd import synth
from oracle import oracle as O


def _pack_np(p, H, st):
    """numpy restatement of ConvexQPSolver::calc_mpc_reference's state packing (:256-276)."""
    R = np.asarray(st["R"])
    vdw = R @ np.asarray(st["vd_rel"])
    rec = np.zeros(33 + 12 * H)
    rec[0:3], rec[3:6], rec[6:9], rec[9:12] = st["euler"], st["pos"], st["w"], st["v"]
    rec[12:21] = R.reshape(9)
    rec[21:33] = np.asarray(st["feet"]).reshape(12)
    for i in range(H):
        rec[33 + 12 * i:33 + 12 * i + 12] = [
            st["euler_d"][0], st["euler_d"][1], st["euler"][2] + st["wd_rel"][2] * p.dt * i,
            st["pos"][0] + vdw[0] * p.dt * i, st["pos"][1] + vdw[1] * p.dt * i, st["pos_d"][2],
            st["wd_rel"][0], st["wd_rel"][1], st["wd_rel"][2], vdw[0], vdw[1], 0.0]
    return rec, vdw


def test_pack_record_matches_restatement():
    rng = np.random.default_rng(3)
    p = synth.params("go1")
    for H in (1, 10, 30):
        a = rng.uniform(-0.5, 0.5, 3)
        c, s = np.cos(a[2]), np.sin(a[2])
        st = dict(euler=a, pos=rng.normal(size=3), w=rng.normal(size=3), v=rng.normal(size=3),
                  R=np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]]), feet=rng.normal(size=(4, 3)) * 0.2,
                  euler_d=rng.normal(size=3), pos_d=rng.normal(size=3), vd_rel=rng.normal(size=3),
                  wd_rel=rng.normal(size=3))
        si = N.LmpcStateIn()
        si.root_euler[:] = list(st["euler"]); si.root_pos[:] = list(st["pos"])
        si.root_ang_vel[:] = list(st["w"]); si.root_lin_vel[:] = list(st["v"])
        si.root_rot_mat[:] = list(st["R"].reshape(9)); si.foot_pos_abs[:] = list(st["feet"].reshape(12))
        si.root_euler_d[:] = list(st["euler_d"]); si.root_pos_d[:] = list(st["pos_d"])
        si.root_lin_vel_d_rel[:] = list(st["vd_rel"]); si.root_ang_vel_d_rel[:] = list(st["wd_rel"])
        rec = np.zeros(33 + 12 * H)
        vdw = np.zeros(3)
        dp = ctypes.POINTER(ctypes.c_double)
        N.check(N.lib().lmpc_pack_record(ctypes.byref(p), H, ctypes.byref(si), rec.ctypes.data_as(dp),
                                         vdw.ctypes.data_as(dp)))
        want, wv = _pack_np(p, H, st)
        np.testing.assert_allclose(rec, want, rtol=0, atol=1e-15)
        np.testing.assert_allclose(vdw, wv, rtol=0, atol=1e-15)


def test_contact_schedule_matches_fsm():
    L = N.lib()
    for gait in range(4):
        for phase in (0.0, 0.13, 0.5, 0.77, 0.999):
            plan = (np.arange(4) % 2).astype(np.uint8)
            out = np.zeros((12, 4), dtype=np.uint8)
            u8 = ctypes.POINTER(ctypes.c_uint8)
            N.check(L.lmpc_contact_schedule(gait, phase, 4.0, 0.01, 12, plan.ctypes.data_as(u8), out.ctypes.data_as(u8)))
            assert np.array_equal(out[0], plan)
            for i in range(1, 12):
                for j in range(4):
                    assert out[i, j] == O.predict_contact(gait, j, phase, 4.0, 0.01 * i)


def test_per_leg_phases_follow_each_leg_fsm():
    """ABI 7: lmpc_command carries one phase per leg, and the expansion predicts every leg from
    its own phase (ConvexQPSolver.cpp:341-342), bit for bit against an independent restatement of the reference's
    four leg FSMs after early touchdowns (oracle/fsm.py: negative phases included)."""
    from oracle import fsm as F

    H = 10
    p = synth.params("go1")
    cmds, fsms = fsm_commands(400, seed=5, H=H)
    phases = np.array([[c.gait_phase[j] for j in range(4)] for c in cmds])
    assert (phases < 0).any() and (np.ptp(phases, axis=1) > 0.02).any()  # wrapped and diverged legs
    rec_ref, _ = synth.fill(p, synth.config_cfg(4), H, 400, synth.BASE_SEED + 4, first_index=505)
    L = N.lib()
    u8 = ctypes.POINTER(ctypes.c_uint8)
    for b in range(400):
        want = np.array(F.schedule(fsms[b], H, p.dt), dtype=np.uint8)
        r, c = synth.command_to_record(p, H, cmds[b])
        assert np.array_equal(c, want), b
        assert np.array_equal(r, rec_ref[b])  # the record does not depend on the gait state
        out = np.zeros((H, 4), dtype=np.uint8)
        ph = np.array(phases[b])
        plan = np.array([cmds[b].plan_contacts[j] for j in range(4)], dtype=np.uint8)
        N.check(L.lmpc_contact_schedule_legs(cmds[b].gait, ph.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 4.0,
                                             p.dt, H, plan.ctypes.data_as(u8), out.ctypes.data_as(u8)))
        assert np.array_equal(out, want), b
        for i in range(1, H):
            for j in range(4):
                assert want[i, j] == L.lmpc_predict_contact(cmds[b].gait, j, phases[b, j], 4.0, p.dt * i)
    # equal phases reduce to the single-phase schedule (the pre-ABI-7 command)
    for gait in range(4):
        one, legs = np.zeros((H, 4), dtype=np.uint8), np.zeros((H, 4), dtype=np.uint8)
        plan = np.ones(4, dtype=np.uint8)
        ph = np.full(4, 0.37)
        N.check(L.lmpc_contact_schedule(gait, 0.37, 4.0, p.dt, H, plan.ctypes.data_as(u8), one.ctypes.data_as(u8)))
        N.check(L.lmpc_contact_schedule_legs(gait, ph.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 4.0, p.dt, H,
                                             plan.ctypes.data_as(u8), legs.ctypes.data_as(u8)))
        assert np.array_equal(one, legs)


def test_current_contact_is_fsm_state():
    L = N.lib()
    for gait in range(4):
        for leg in range(4):
            for ph in np.linspace(0, 0.999, 50):
                assert L.lmpc_current_contact(gait, leg, ph) == O.current_contact(gait, leg, ph)


def test_generator_deterministic_and_shard_invariant():
    p = synth.params("go1")
    cfg = synth.synth_cfg("go1", -1)
    rec, con = synth.fill(p, cfg, 10, 64, seed=99)
    rec2, con2 = synth.fill(p, cfg, 10, 64, seed=99)
    assert np.array_equal(rec, rec2) and np.array_equal(con, con2)
    # rank-style shards build exactly the same instances as the whole batch
    for r in range(4):
        rs, cs = synth.fill(p, cfg, 10, 16, seed=99, first_index=16 * r)
        assert np.array_equal(rs, rec[16 * r:16 * r + 16]) and np.array_equal(cs, con[16 * r:16 * r + 16])
    rec3, _ = synth.fill(p, cfg, 10, 64, seed=100)
    assert not np.array_equal(rec, rec3)


def test_generator_distributions():
    """SURVEY.md 8d ranges: |roll|,|pitch| <= 0.2, p_z in [0.20, 0.35], z_d in [0.25, 0.32], R orthonormal."""
    p, H, rec, con = synth.config_batch(2, count=2000)
    assert np.all(np.abs(rec[:, 0:2]) <= 0.2)
    assert np.all((rec[:, 5] >= 0.2) & (rec[:, 5] <= 0.35))
    assert np.all((rec[:, 33 + 5] >= 0.25) & (rec[:, 33 + 5] <= 0.32))
    R = rec[:, 12:21].reshape(-1, 3, 3)
    assert np.allclose(R @ np.transpose(R, (0, 2, 1)), np.eye(3), atol=1e-12)
    # trot: diagonal pairs, exactly two stance legs per step
    assert np.all(con.sum(-1) == 2)
    assert np.array_equal(con[..., 0], con[..., 3]) and np.array_equal(con[..., 1], con[..., 2])
    # mixed gaits cover all four patterns (stand -> all four legs in stance for every step)
    _, _, recm, conm = synth.config_batch(4, count=400)
    assert np.any(np.all(conm == 1, axis=(1, 2)))


@pytest.mark.parametrize("path", [p for p in golden_files() if "config" in p])
def test_golden_inputs_pin_the_generator(path):
    """The committed fixtures were generated by this generator; regenerate and compare."""
    g = load_golden(path)
    cid = int(path.split("golden_config")[1][0])
    _, H, rec, con = synth.config_batch(cid, count=g["rec"].shape[0])
    assert np.array_equal(rec, g["rec"]) and np.array_equal(con, g["contact"])


def test_presets_match_reference_yaml():
    p = synth.params("go1")  # gazebo_go1_convex.yaml:39-71
    assert list(p.q_weights) == [50.0, 100.0, 0.0, 0.0, 0.0, 3500.0, 0.01, 0.01, 10.0, 15.0, 15.0, 20.0]
    assert list(p.r_weights) == [1e-4] * 12
    assert p.robot_mass == 13.0 and p.mu == 0.3 and p.f_max == 180.0 and p.gravity == 9.8 and p.dt == 0.01
    a1 = synth.params("a1")  # gazebo_a1_convex.yaml:40-72
    assert list(a1.q_weights) == [60.0, 100.0, 0.0, 0.0, 0.0, 450.0, 0.15, 0.15, 100.0, 3.0, 3.0, 5.0]


def test_synth_normals_deterministic_and_distributed():
    """Config 4 terrain normals: unit, tilt theta in [0, 0.3], shard-invariant, own stream."""
    a = synth.normals(4096, 77)
    b = synth.normals(1000, 77, first_index=3000)
    assert np.array_equal(a[3000:4000], b)
    assert np.allclose(np.linalg.norm(a, axis=2), 1.0, atol=1e-15)
    th = np.arccos(np.clip(a[..., 2], -1, 1))
    assert th.min() >= 0.0 and th.max() <= 0.3 + 1e-12
    assert abs(th.mean() - 0.15) < 0.005  # U(0, 0.3)
    ph = np.arctan2(a[..., 1], a[..., 0])
    assert abs(ph.mean()) < 0.05 and ph.std() > 1.7  # U(-pi, pi): std pi/sqrt(3) = 1.81
    # records do not depend on whether normals are drawn (separate Philox stream)
    _, _, rec1, con1 = synth.config_batch(4, count=8)
    synth.config_normals(4, count=8)
    _, _, rec2, con2 = synth.config_batch(4, count=8)
    assert np.array_equal(rec1, rec2) and np.array_equal(con1, con2)
    assert synth.config_normals(2) is None


@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5])
def test_commands_expand_to_the_generator_records(cid):
    """lmpc_synth_fill == lmpc_synth_commands + lmpc_command_to_record, bit for bit (SURVEY.md 8f-1:
    the command is all the step before the QP needs)."""
    p, H, rec, con = synth.config_batch(cid, count=24, first_index=100)
    cmds = synth.commands(synth.config_cfg(cid), 24, synth.BASE_SEED + cid, first_index=100)
    for b in range(24):
        r, c = synth.command_to_record(p, H, cmds[b])
        assert np.array_equal(r, rec[b]) and np.array_equal(c, con[b])
    if cid == 4:
        assert len({cmds[b].gait for b in range(24)}) > 1  # mixed gaits


def test_foot_jacobian_matches_complex_step_oracle():
    """Closed-form J (product) == complex-step derivative of the restated A1Kinematics::fk (oracle),
    for the reference's constants and for nonzero rho_opt."""
    from legged_mpc_control_amd import foot_jacobian, leg_kin_default

    kin = leg_kin_default()
    assert [list(kin.rho_fix[i]) for i in range(4)] == [
        [0.1805, 0.047, 0.0838, 0.21, 0.21], [0.1805, -0.047, -0.0838, 0.21, 0.21],
        [-0.1805, 0.047, 0.0838, 0.21, 0.21], [-0.1805, -0.047, -0.0838, 0.21, 0.21]]  # BaseInterface.cpp:76-97
    rng = np.random.default_rng(5)
    for trial in range(400):
        leg = trial % 4
        if trial >= 200:
            for k in range(3):
                kin.rho_opt[leg][k] = rng.uniform(-0.03, 0.03)
        q = rng.uniform([-0.8, -1.0, -2.7], [0.8, 2.5, -0.5])
        J = foot_jacobian(kin, leg, q)
        Jo = O.foot_jacobian(list(kin.rho_fix[leg]), list(kin.rho_opt[leg]), q)
        assert np.max(np.abs(J - Jo)) <= 1e-15 * 4


def test_grf_to_torque_matches_oracle():
    from legged_mpc_control_amd import grf_to_torque, leg_kin_default

    kin = leg_kin_default()
    p, H, rec, con = synth.config_batch(2, count=64)
    g = load_golden([q for q in golden_files() if "config2" in q][0])
    rng = np.random.default_rng(9)
    rf = np.array([list(kin.rho_fix[i]) for i in range(4)])
    ro = np.array([list(kin.rho_opt[i]) for i in range(4)])
    for b in range(16):
        q = rng.uniform(np.tile([-0.3, 0.4, -2.4], 4), np.tile([0.3, 1.2, -1.2], 4))
        tau = grf_to_torque(kin, g["rec"][b, 12:21], q, g["grf"][b, 0])
        ref = O.grf_to_torque(rf, ro, g["rec"][b, 12:21], q, g["grf"][b, 0])
        assert np.max(np.abs(tau - ref) / np.maximum(1.0, np.abs(ref))) <= 1e-13
    # swing legs carry no force -> zero torque; standing (R = I, straight legs): tau = -J' f
    tau0 = grf_to_torque(kin, np.eye(3), np.zeros(12), np.zeros(12))
    assert np.array_equal(tau0, np.zeros(12))

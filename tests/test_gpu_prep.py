"""GPU tests of the step before the QP on the device: command -> record
expansion (bit-identical to the host restatement), on-device synthetic generation (== the host
generator to a few ulp), and the fused commands -> solve path against the CPU oracle."""
import ctypes

import numpy as np
import pytest

from conftest import fsm_commands, rel_err

from legged_mpc_control_amd import BatchedConvexQPSolver, _native as N, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


def _host_cmds_tensor(cmds, dev):
    import torch

    raw = np.frombuffer(bytes(cmds), dtype=np.uint8).reshape(len(cmds), N.COMMAND_BYTES)
    return torch.from_numpy(raw.copy()).to(dev)


@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5])
def test_device_expansion_bit_identical(cid, dev):
    import torch

    count = 1 if cid == 1 else 300
    p, H, rec, con = synth.config_batch(cid, count=count, first_index=7)
    cmds = synth.commands(synth.config_cfg(cid), count, synth.BASE_SEED + cid, first_index=7)
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_rec, d_con = s.build_records_device(_host_cmds_tensor(cmds, dev))
    torch.cuda.synchronize()
    assert np.array_equal(d_rec.cpu().numpy(), rec)
    assert np.array_equal(d_con.cpu().numpy(), con)


def test_device_expansion_per_leg_phases(dev):
    """ABI 7: commands whose legs carry diverged FSM phases (early touchdowns, negative phases; oracle/fsm.py) expand
    on the device to the host's records and schedules bit for bit, every leg predicted from its own phase; the
    solve of those QPs matches the oracle."""
    import torch

    from oracle import fsm as F

    p, H = synth.params("go1"), 10
    cmds, fsms = fsm_commands(1024, seed=9, H=H)
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_rec, d_con = s.build_records_device(_host_cmds_tensor(cmds, dev))
    torch.cuda.synchronize()
    con = d_con.cpu().numpy()
    for b in range(len(cmds)):
        r, c = synth.command_to_record(p, H, cmds[b])
        assert np.array_equal(c, con[b]) and np.array_equal(c, np.array(F.schedule(fsms[b], H, p.dt), dtype=np.uint8))
        assert np.array_equal(r, d_rec[b].cpu().numpy())
    grf = torch.empty((len(cmds), H, 12), dtype=torch.float64, device=dev)
    st = torch.empty(len(cmds), dtype=torch.int32, device=dev)
    s.solve_commands_device(_host_cmds_tensor(cmds, dev), grf, st)
    torch.cuda.synchronize()
    ref, _, fails = O.solve_batch(O.params_from(p), H, d_rec.cpu().numpy(), con, n_threads=8)
    assert fails == 0 and np.all(st.cpu().numpy() == 0)
    assert rel_err(grf.cpu().numpy(), ref) <= 1e-7


def test_device_generator_matches_host(dev):
    import torch

    p, H = synth.params("go1"), 10
    cfg = synth.config_cfg(4)
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_cmd = s.synth_commands_device(cfg, 4096, 123, first_index=1000, device=dev)
    torch.cuda.synchronize()
    host = synth.commands(cfg, 4096, 123, first_index=1000)
    hraw = np.frombuffer(bytes(host), dtype=np.uint8).reshape(4096, N.COMMAND_BYTES)
    draw = d_cmd.cpu().numpy()
    # 45 state doubles + 4 per-leg phases + speed
    hd, dd = hraw[:, :400].view(np.float64), draw[:, :400].view(np.float64)
    assert np.max(np.abs(hd - dd) / np.maximum(1.0, np.abs(hd))) <= 1e-14
    assert np.array_equal(hraw[:, 400:], draw[:, 400:])  # gait, plan_contacts (and padding-free tail)
    assert np.array_equal(hd[:, 45:49], dd[:, 45:49])  # gait phases: no transcendental on their path
    # normals
    dn = s.synth_normals_device(4096, 123, first_index=1000, device=dev)
    torch.cuda.synchronize()
    hn = synth.normals(4096, 123, first_index=1000)
    assert np.max(np.abs(dn.cpu().numpy() - hn)) <= 1e-15


@pytest.mark.parametrize("cid", [2, 4])
def test_commands_to_solve_on_device_vs_oracle(cid, dev):
    """Inputs generated on the device from (seed, global index), expanded and solved there; the
    records read back feed the CPU oracle."""
    import torch

    p, H = synth.config_batch(cid, count=1)[:2]
    B = 512
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_cmd = s.synth_commands_device(synth.config_cfg(cid), B, synth.BASE_SEED + cid, first_index=40000, device=dev)
    d_nrm = s.synth_normals_device(B, synth.BASE_SEED + cid, first_index=40000, device=dev) if cid == 4 else None
    grf = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
    st = torch.empty(B, dtype=torch.int32, device=dev)
    s.solve_commands_device(d_cmd, grf, st, normals=d_nrm)
    d_rec, d_con = s.build_records_device(d_cmd)
    torch.cuda.synchronize()
    rec, con = d_rec.cpu().numpy(), d_con.cpu().numpy()
    nrm = None if d_nrm is None else d_nrm.cpu().numpy()
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8, normals=nrm)
    assert fails == 0 and np.all(st.cpu().numpy() == 0)
    assert rel_err(grf.cpu().numpy(), ref) <= 1e-7
    # the fused call equals expand + solve
    grf2 = torch.empty_like(grf)
    s.solve_device(d_rec, d_con, grf2, normals=d_nrm)
    torch.cuda.synchronize()
    assert torch.equal(grf, grf2)


def test_grf_to_torque_device_vs_oracle(dev):
    """State -> commands -> records -> QP -> torques, all on the device; torques against the
    oracle's complex-step Jacobian path on the read-back GRFs."""
    import torch

    from legged_mpc_control_amd import leg_kin_default

    p, H = synth.params("go1"), 10
    B = 2048
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_cmd = s.synth_commands_device(synth.config_cfg(4), B, 99, device=dev)
    d_rec, d_con = s.build_records_device(d_cmd)
    grf = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
    s.solve_device(d_rec, d_con, grf)
    rng = np.random.default_rng(2)
    q = rng.uniform(np.tile([-0.3, 0.4, -2.4], 4), np.tile([0.3, 1.2, -1.2], 4), size=(B, 12))
    kin = leg_kin_default()
    kin.rho_opt[1][2] = 0.02  # exercise the foot-offset terms on one leg
    tau = s.grf_to_torque_device(kin, d_rec, torch.from_numpy(q).to(dev), grf)
    torch.cuda.synchronize()
    tau, g, rec = tau.cpu().numpy(), grf.cpu().numpy(), d_rec.cpu().numpy()
    rf = np.array([list(kin.rho_fix[i]) for i in range(4)])
    ro = np.array([list(kin.rho_opt[i]) for i in range(4)])
    worst = 0.0
    for b in range(0, B, 7):
        ref = O.grf_to_torque(rf, ro, rec[b, 12:21], q[b], g[b, 0])
        worst = max(worst, float(np.max(np.abs(tau[b] - ref) / np.maximum(1.0, np.abs(ref)))))
    assert worst <= 1e-12, worst
    swing = d_con.cpu().numpy()[:, 0, :] == 0  # step-0 swing legs: zero force -> zero torque
    assert np.all(tau.reshape(B, 4, 3)[swing] == 0.0)

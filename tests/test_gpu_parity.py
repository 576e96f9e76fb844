"""GPU parity tests (MI355X): the HIP path, called through the C-ABI, against the
CPU oracle (exact optimum of the reference's QP) on the committed golden
fixtures, on live seeded samples of every BASELINE config, and -- at the full
batch sizes -- through size-independent properties (feasibility, determinism,
permutation and shard invariance, device == host path).

Tolerance (BASELINE.json north star): max over all H x 12 forces of
|f_gpu - f_ref| / max(1, |f_ref|) <= 1e-4.  A tighter 1e-7 regression guard is
also asserted (the kernel reaches ~1e-9: both solve the same QP exactly).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden_files, lmpc_params_from, load_golden, rel_err

from legged_mpc_control_amd import BatchedConvexQPSolver, solver_options, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4          # north-star parity bar
TOL_REGRESS = 1e-7  # regression guard
DENSE = {"ipm": "ipm", "gi": "gi", "0": "off"}  # test ids -> lmpc_set_dense_path


def feasibility_violation(grf, con, mu=0.3, fmax=180.0):
    f = grf.reshape(grf.shape[0], -1, 4, 3)
    c = con.astype(bool)
    fx, fy, fz = f[..., 0], f[..., 1], f[..., 2]
    v = np.maximum.reduce([np.abs(fx) - mu * fz, np.abs(fy) - mu * fz, -fz, fz - fmax * c])
    swing_nonzero = np.any(f[~c] != 0.0)
    return float(np.max(v)), bool(swing_nonzero)


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")


@pytest.mark.parametrize("mode", ["ipm", "gi", "0"])
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p))
def test_golden_fixtures(path, mode):
    """Every certified golden instance on each device path: the condensed interior point (default),
    the condensed dual active set and the Riccati kernel (QPs the dense kernels do not take -- more
    than 20 stance leg-steps, H > 16, all-swing -- run on the Riccati kernel in every mode)."""
    g = load_golden(path)
    s = BatchedConvexQPSolver(lmpc_params_from(g["params"]), g["H"], max_batch=g["rec"].shape[0],
                              dense_path=DENSE[mode])
    grf, status, iters = s.solve(g["rec"], g["contact"], normals=g["normals"])
    assert np.all(status == 0), status
    err = rel_err(grf, g["grf"])
    assert err <= TOL
    assert err <= TOL_REGRESS, f"regression: {err:.2e}"


@pytest.mark.parametrize("cid,count,first", [(2, 256, 5000), (3, 48, 777), (4, 512, 12345), (5, 24, 99)])
def test_live_samples_vs_oracle(cid, count, first):
    p, H, rec, con = synth.config_batch(cid, count=count, first_index=first)
    s = BatchedConvexQPSolver(p, H, max_batch=count)
    grf, status, iters = s.solve(rec, con)
    ref, ost, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    assert fails == 0
    assert np.all(status == 0)
    err = rel_err(grf, ref)
    assert err <= TOL and err <= TOL_REGRESS, err


def test_full_config2_batch_vs_oracle():
    """Config 2 at its full size (1024 QPs): every QP against the oracle."""
    p, H, rec, con = synth.config_batch(2)
    s = BatchedConvexQPSolver(p, H, max_batch=rec.shape[0])
    grf, status, iters = s.solve(rec, con)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    assert fails == 0 and np.all(status == 0)
    assert rel_err(grf, ref) <= TOL_REGRESS


@pytest.mark.parametrize("cid,mode", [(3, "ipm"), (4, "ipm"), (4, "gi"), (5, "ipm")])
def test_full_size_properties(cid, mode, torch_dev):
    """Configs 3/4/5 at full batch: converged, feasible, swing legs exactly zero,
    bitwise deterministic, permutation-invariant and shard-invariant, including a shard small enough
    to change the Riccati kernel instance (config 4 also with the dual active-set kernel on its
    dense-eligible QPs)."""
    import torch

    p, H, rec, con = synth.config_batch(cid)
    B = rec.shape[0]
    s = BatchedConvexQPSolver(p, H, max_batch=0, dense_path=mode)
    d_rec, d_con = torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev)
    out = torch.empty((B, H, 12), dtype=torch.float64, device=torch_dev)
    st = torch.empty(B, dtype=torch.int32, device=torch_dev)
    s.solve_device(d_rec, d_con, out, st)
    torch.cuda.synchronize()
    grf, status = out.cpu().numpy(), st.cpu().numpy()
    assert np.all(status == 0), np.bincount(status)
    viol, swing_nonzero = feasibility_violation(grf, con, p.mu, p.f_max)
    assert viol <= 1e-9 * p.f_max and not swing_nonzero
    # determinism
    out2 = torch.empty_like(out)
    s.solve_device(d_rec, d_con, out2, st)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    # permutation invariance
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(1)).to(torch_dev)
    out3 = torch.empty_like(out)
    s.solve_device(d_rec[perm].contiguous(), d_con[perm].contiguous(), out3, st)
    torch.cuda.synchronize()
    assert torch.equal(out3, out[perm])
    # shard invariance: second half solved on its own
    half = B // 2
    out4 = torch.empty((B - half, H, 12), dtype=torch.float64, device=torch_dev)
    s.solve_device(d_rec[half:].contiguous(), d_con[half:].contiguous(), out4, st[: B - half])
    torch.cuda.synchronize()
    assert torch.equal(out4, out[half:])
    # a shard of at most one QP per SIMD: at H <= 10 the Riccati kernel then runs its one-wave-per-SIMD
    # instance instead of the two-wave one (launch_qp) -- same arithmetic, same bits
    small = 512
    out5 = torch.empty((small, H, 12), dtype=torch.float64, device=torch_dev)
    s.solve_device(d_rec[:small].contiguous(), d_con[:small].contiguous(), out5, st[:small])
    torch.cuda.synchronize()
    assert torch.equal(out5, out[:small])
    # oracle on a sample
    idx = np.random.default_rng(cid).choice(B, 32, replace=False)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec[idx], con[idx], n_threads=8)
    assert rel_err(grf[idx], ref) <= TOL_REGRESS


def test_device_path_equals_host_path(torch_dev):
    import torch

    p, H, rec, con = synth.config_batch(2, count=128)
    s = BatchedConvexQPSolver(p, H, max_batch=128)
    grf_h, st_h, it_h = s.solve(rec, con)
    out = torch.empty((128, H, 12), dtype=torch.float64, device=torch_dev)
    st = torch.empty(128, dtype=torch.int32, device=torch_dev)
    it = torch.empty(128, dtype=torch.int32, device=torch_dev)
    stream = torch.cuda.Stream(torch_dev)
    s.solve_device(torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev), out, st, it, stream)
    stream.synchronize()
    assert np.array_equal(out.cpu().numpy(), grf_h)
    assert np.array_equal(st.cpu().numpy(), st_h) and np.array_equal(it.cpu().numpy(), it_h)


@pytest.mark.parametrize("H", [1, 2, 16, 17, 32])
def test_horizon_range(H):
    p = synth.params("go1")
    rec, con = synth.fill(p, synth.synth_cfg("go1", -1), H, 12, seed=555 + H)
    s = BatchedConvexQPSolver(p, H, max_batch=12)
    grf, status, _ = s.solve(rec, con)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=4)
    assert fails == 0 and np.all(status == 0)
    assert rel_err(grf, ref) <= TOL_REGRESS


@pytest.mark.parametrize("H,mode", [(16, "0"), (16, "ipm"), (12, "gi"), (17, "ipm")])
def test_riccati_instances_large_batch(H, mode):
    """Batches above one QP per SIMD (2048 mixed-gait QPs): at H <= 16 the Riccati kernel runs its two-wave
    instance, at H = 17 the one-wave two-leg-step instance.  Sampled QPs vs the oracle, and a 256-QP shard
    (one-wave instance) bit-identical to the same QPs inside the large batch."""
    p, _, rec, con = synth.config_batch(4, count=2048, first_index=4242, H=H)
    s = BatchedConvexQPSolver(p, H, max_batch=2048, dense_path=DENSE[mode])
    grf, status, _ = s.solve(rec, con)
    assert np.all(status == 0), np.bincount(status)
    viol, swing_nonzero = feasibility_violation(grf, con, p.mu, p.f_max)
    assert viol <= 1e-9 * p.f_max and not swing_nonzero
    g2, st2, _ = s.solve(rec[:256], con[:256])
    assert np.array_equal(g2, grf[:256]) and np.all(st2 == 0)
    idx = np.random.default_rng(H).choice(2048, 24, replace=False)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec[idx], con[idx], n_threads=8)
    assert fails == 0
    assert rel_err(grf[idx], ref) <= TOL_REGRESS


def test_a1_params_and_standing_config():
    p, H, rec, con = synth.config_batch(1)
    s = BatchedConvexQPSolver(p, H, max_batch=1)
    grf, status, _ = s.solve(rec, con)
    ref, _, _ = O.solve(O.params_from(p), H, rec[0], con[0])
    assert status[0] == 0 and rel_err(grf[0], ref) <= TOL_REGRESS
    # standing with zero velocity: u_0 supports the weight (sum fz ~ m g), no lateral force
    u0 = grf[0, 0].reshape(4, 3)
    assert abs(u0[:, 2].sum() - p.robot_mass * p.gravity) < 0.5 * p.robot_mass * p.gravity


def test_nan_input_returns_zeros_and_status():
    p, H, rec, con = synth.config_batch(2, count=4)
    rec = rec.copy()
    rec[1, 5] = np.nan
    s = BatchedConvexQPSolver(p, H, max_batch=4)
    grf, status, _ = s.solve(rec, con)
    assert status[1] == 2 and np.all(grf[1] == 0.0)
    assert np.all(status[[0, 2, 3]] == 0)


def test_empty_batch_and_all_swing():
    p, H, rec, con = synth.config_batch(2, count=3)
    s = BatchedConvexQPSolver(p, H, max_batch=3)
    g0, s0, _ = s.solve(rec[:0], con[:0])
    assert g0.shape == (0, H, 12)
    con = con.copy()
    con[:] = 0
    grf, status, _ = s.solve(rec, con)
    assert np.all(status == 0) and np.all(grf == 0.0)


def test_reference_shaped_python_api():
    """ConvexQPSolver used the way ConvexMpc::grf_update does (ConvexMpc.cpp:64-78)."""
    from legged_mpc_control_amd import ConvexQPSolver, LeggedContactFSM, LeggedState

    p = synth.params("go1")
    st = LeggedState()
    st.param.q_weights = np.array(p.q_weights[:])
    st.param.gait_counter_speed = 4.0
    st.fbk.root_pos = np.array([0.1, -0.2, 0.27])
    st.fbk.root_euler = np.array([0.05, -0.03, 0.4])
    c, s_ = np.cos(0.4), np.sin(0.4)
    st.fbk.root_rot_mat = np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1.0]])
    st.fbk.root_lin_vel = np.array([0.3, 0.0, 0.0])
    st.fbk.foot_pos_abs = (st.fbk.root_rot_mat @ np.array(
        [[0.17, 0.12, -0.3], [0.17, -0.17, -0.3], [-0.17, 0.17, -0.3], [-0.17, -0.12, -0.3]]).T)
    st.ctrl.root_pos_d = np.array([0, 0, 0.28])
    st.ctrl.root_lin_vel_d_rel = np.array([0.5, 0.1, 0.0])
    st.ctrl.root_ang_vel_d_rel = np.array([0.0, 0.0, 0.3])
    fsm = [LeggedContactFSM() for _ in range(4)]
    for i in range(4):
        fsm[i].reset_params(st, i)
        fsm[i].gait_phase = 0.3
        st.ctrl.plan_contacts[i] = bool(fsm[i].get_contact_state())
    solver = ConvexQPSolver(p.q_weights, p.r_weights, horizon=10)
    solver.calc_mpc_reference(st, fsm)
    solver.update_cons_matrix()
    u0 = solver.compute_grfs(st)
    ref, _, _ = O.solve(O.params_from(p), 10, solver._rec[0], solver._con[0])
    assert u0.shape == (12,) and solver.last_status == 0
    assert rel_err(u0, ref[0]) <= TOL_REGRESS
    np.testing.assert_allclose(st.ctrl.root_lin_vel_d_world, st.fbk.root_rot_mat @ st.ctrl.root_lin_vel_d_rel)


def test_cpp_dropin_program_vs_oracle():
    """tests/cpp/grf_update_test.cpp drives legged::ConvexQPSolver like ConvexMpc."""
    from legged_mpc_control_amd import build as B

    exe = B.build_cpp_test()
    out = subprocess.run([exe, "10", "3"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    p = synth.params("a1")
    op = O.params_from(p)
    ticks = 0
    for i in range(0, len(lines), 5):
        assert lines[i].endswith("status 0")
        rec = np.array(lines[i + 1].split()[1:], dtype=np.float64)
        con = np.array(lines[i + 2].split()[1:], dtype=np.uint8).reshape(10, 4)
        grf = np.array(lines[i + 3].split()[1:], dtype=np.float64).reshape(10, 12)
        u0 = np.array(lines[i + 4].split()[1:], dtype=np.float64)
        ref, _, _ = O.solve(op, 10, rec, con)
        assert rel_err(grf, ref) <= TOL_REGRESS
        assert np.array_equal(u0, grf[0])
        ticks += 1
    assert ticks == 3


@pytest.mark.parametrize("mode", ["ipm", "0"])
def test_solve_options_and_status_codes(mode):
    """IPM options (max_iter / attempts) on the two interior-point paths: the condensed dense kernel
    (dense path "ipm") and the Riccati kernel (dense path "off").  The dual active-set kernel has no
    interior-point iterations; its step cap hands a QP to the Riccati kernel."""
    from legged_mpc_control_amd import LmpcOptions
    from legged_mpc_control_amd import _native as N

    p, H, rec, con = synth.config_batch(2, count=32)
    s = BatchedConvexQPSolver(p, H, max_batch=32, dense_path=DENSE[mode])
    o = LmpcOptions()
    N.lib().lmpc_options_default(o)
    o.max_iter, o.max_attempts = 2, 1  # far too few IPM iterations: polish may not verify
    s.set_options(o)
    grf, status, iters = s.solve(rec, con)
    assert set(np.unique(status)) <= {0, 1}
    assert np.all((iters & 0xFFFF) <= 2)
    viol, _ = feasibility_violation(grf, con)
    assert viol <= 1e-6 * p.f_max  # status-1 answers are the feasible interior-point iterate
    N.lib().lmpc_options_default(o)
    s.set_options(o)
    grf, status, iters = s.solve(rec, con)
    assert np.all(status == 0)


# ---------------------------------------------------------------------------
# terrain extension (config 4: per-leg normals, theta ~ U(0, 0.3)); parity vs this build's oracle
# ---------------------------------------------------------------------------
def terrain_violation(grf, con, normals, mu=0.3, fmax=180.0):
    """Max pyramid/bound violation of g = R_j'f in each leg's contact frame."""
    B, H = grf.shape[0], con.shape[1]
    f = grf.reshape(B, H, 4, 3)
    v = -np.inf
    for j in range(4):
        Rs = np.stack([synth.terrain_frame(n) for n in normals[:, j]])   # [B,3,3]
        g = np.einsum("bhp,bpq->bhq", f[:, :, j], Rs)                     # g = R'f (row form)
        c = con[:, :, j].astype(bool)
        v = max(v, float(np.max(np.maximum.reduce([np.abs(g[..., 0]) - mu * g[..., 2],
                                                   np.abs(g[..., 1]) - mu * g[..., 2],
                                                   -g[..., 2], g[..., 2] - fmax * c]))))
    return v


def test_terrain_live_samples_vs_oracle():
    p, H, rec, con = synth.config_batch(4, count=512, first_index=20000)
    nrm = synth.config_normals(4, count=512, first_index=20000)
    s = BatchedConvexQPSolver(p, H, max_batch=512)
    grf, status, iters = s.solve(rec, con, normals=nrm)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8, normals=nrm)
    assert fails == 0 and np.all(status == 0)
    err = rel_err(grf, ref)
    assert err <= TOL and err <= TOL_REGRESS, err
    assert terrain_violation(grf, con, nrm, p.mu, p.f_max) <= 1e-9 * p.f_max


def test_terrain_flat_normals_equal_flat_path():
    """normals = e_z poses the reference's problem: same answer as the flat kernel (to rounding)."""
    p, H, rec, con = synth.config_batch(4, count=256)
    s = BatchedConvexQPSolver(p, H, max_batch=256)
    g0, st0, _ = s.solve(rec, con)
    g1, st1, _ = s.solve(rec, con, normals=np.tile([0.0, 0.0, 1.0], (256, 4, 1)))
    assert np.all(st0 == 0) and np.all(st1 == 0)
    assert rel_err(g1, g0) <= 1e-10  # same QP; G0 R is formed in a different order (rounding only)


def test_terrain_full_size_properties(torch_dev):
    """Config 4 at full batch (65536) with terrain: converged, feasible in every contact frame,
    swing legs exactly zero, device path == host path, sampled against the oracle."""
    import torch

    p, H, rec, con = synth.config_batch(4)
    nrm = synth.config_normals(4)
    B = rec.shape[0]
    s = BatchedConvexQPSolver(p, H, max_batch=1024)
    d_rec, d_con = torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev)
    d_nrm = torch.from_numpy(nrm).to(torch_dev)
    out = torch.empty((B, H, 12), dtype=torch.float64, device=torch_dev)
    st = torch.empty(B, dtype=torch.int32, device=torch_dev)
    s.solve_device(d_rec, d_con, out, st, normals=d_nrm)
    torch.cuda.synchronize()
    grf, status = out.cpu().numpy(), st.cpu().numpy()
    assert np.all(status == 0), np.bincount(status)
    assert terrain_violation(grf, con, nrm, p.mu, p.f_max) <= 1e-9 * p.f_max
    assert not np.any(grf.reshape(B, H, 4, 3)[~con.astype(bool)] != 0.0)
    gh, sh, _ = s.solve(rec[:1024], con[:1024], normals=nrm[:1024])
    assert np.array_equal(gh, grf[:1024]) and np.array_equal(sh, status[:1024])
    idx = np.random.default_rng(4).choice(B, 32, replace=False)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec[idx], con[idx], n_threads=8, normals=nrm[idx])
    assert rel_err(grf[idx], ref) <= TOL_REGRESS


def test_terrain_rejects_bad_normals():
    p, H, rec, con = synth.config_batch(4, count=4)
    s = BatchedConvexQPSolver(p, H, max_batch=4)
    bad = np.tile([0.0, 0.0, 1.0], (4, 4, 1))
    bad[2, 1] = [0.3, 0.0, -0.1]  # n_z <= 0: not a ground normal
    with pytest.raises(RuntimeError):
        s.solve(rec, con, normals=bad)
    bad[2, 1] = [np.nan, 0.0, 1.0]
    with pytest.raises(RuntimeError):
        s.solve(rec, con, normals=bad)
    with pytest.raises(ValueError):
        s.solve(rec, con, normals=np.zeros((4, 3)))


# ---------------------------------------------------------------------------
# the two device paths: condensed dense kernel (<= 20 stance leg-steps, H <= 16) and Riccati kernel
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["ipm", "gi"])
@pytest.mark.parametrize("cid", [2, 4])
def test_dense_and_riccati_paths_agree(cid, mode):
    """Every config-2 QP (and the trot-like config-4 QPs) runs on a condensed dense kernel -- the
    interior point ("ipm") or the dual active set ("gi"); with the dense path "off" the
    same QPs run on the Riccati path.  All must give the oracle's optimum."""
    p, H, rec, con = synth.config_batch(cid, count=512, first_index=777)
    nrm = synth.config_normals(cid, count=512, first_index=777)
    nls = con.sum((1, 2))
    dense = (nls >= 1) & (nls <= 20)
    assert np.any(dense) and (cid == 4 or np.all(dense))
    gd, sd, itd = BatchedConvexQPSolver(p, H, max_batch=512, dense_path=mode).solve(rec, con, normals=nrm)
    gr, sr, itr = BatchedConvexQPSolver(p, H, max_batch=512, dense_path="off").solve(rec, con, normals=nrm)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8, normals=nrm)
    assert fails == 0 and np.all(sd == 0) and np.all(sr == 0)
    assert rel_err(gd, ref) <= TOL_REGRESS and rel_err(gr, ref) <= TOL_REGRESS
    assert rel_err(gd, gr) <= 1e-8
    if mode == "ipm":
        # same Newton systems, so the same iteration counts on both paths
        assert np.mean(np.abs((itd & 0xFFFF) - (itr & 0xFFFF))) < 0.05
    else:
        # dual active set: steps in the low 16 bits (0 when the unconstrained minimiser is feasible),
        # drops in the high bits
        steps, drops = itd[dense] & 0xFFFF, itd[dense] >> 16
        assert np.all(drops <= steps) and steps.mean() > 5
        assert np.array_equal(itd[~dense], itr[~dense])  # the rest ran on the Riccati kernel


@pytest.mark.parametrize("mode", ["ipm", "gi"])
def test_dense_path_edge_cases(mode):
    """Dense-path QPs with fewer than 20 stance leg-steps (partly padded tiles), a single stance
    leg-step, and the all-swing QP (left to the Riccati kernel)."""
    p, H, rec, con = synth.config_batch(2, count=8, first_index=31)
    con = con.copy()
    con[0, :, :] = 0; con[0, 0, 1] = 1          # one stance leg-step
    con[1, 5:, :] = 0                           # 10 stance leg-steps (tiles 2-3 empty)
    con[2, :, :] = 0                            # all swing -> zeros (Riccati kernel)
    con[3, :, 0] = 1; con[3, :, 1:] = 0         # one leg in stance all horizon
    con[4, 0:4, :] = 1                          # 16 + ... stance: > 20 -> Riccati
    s = BatchedConvexQPSolver(p, H, max_batch=8, dense_path=mode)
    g, st, it = s.solve(rec, con)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=4)
    assert fails == 0 and np.all(st == 0), st
    assert rel_err(g, ref) <= TOL_REGRESS
    assert np.all(g[2] == 0.0)


def test_multiround_polish_vs_oracle():
    """A polish round that follows a polish round re-factors only from the tile of the first leg-step whose active set
    changed; the diagonal-tile factors ahead of it are reused (lmpc_dense.hip, keep_tiles).  Every QP of a config-2
    batch that needed two or more polish rounds matches the oracle, and some needed three."""
    p, H, rec, con = synth.config_batch(2, count=1024)
    s = BatchedConvexQPSolver(p, H, max_batch=1024, dense_path="ipm")
    g, st, it = s.solve(rec, con)
    rounds = it >> 16
    multi = np.nonzero(rounds >= 2)[0]
    assert len(multi) >= 16 and np.any(rounds >= 3)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec[multi], con[multi], n_threads=8)
    assert np.all(st[multi] == 0)
    assert rel_err(g[multi], ref) <= TOL_REGRESS


def test_dense_path_api(monkeypatch):
    """lmpc_set_dense_path selects the dense kernel per context (ABI 3); no environment variable changes it
    (ABI 5); H > 16 has no dense path; all paths give the same optimum."""
    p, H, rec, con = synth.config_batch(2, count=64, first_index=9000)
    out = {}
    for path in ("ipm", "gi", "off"):
        s = BatchedConvexQPSolver(p, H, max_batch=64, dense_path=path)
        assert s.dense_path == path
        out[path] = s.solve(rec, con)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    for path, (g, st, it) in out.items():
        assert np.all(st == 0) and rel_err(g, ref) <= TOL_REGRESS, path
    assert np.array_equal(out["ipm"][2], out["off"][2])                 # same Newton systems
    assert not np.array_equal(out["gi"][2], out["ipm"][2])              # active-set steps instead
    monkeypatch.setenv("LMPC_DENSE", "0")  # the old override is gone: the explicit choice stands
    assert BatchedConvexQPSolver(p, H, max_batch=4, dense_path="gi").dense_path == "gi"
    assert BatchedConvexQPSolver(p, H, max_batch=4).dense_path == "ipm"
    monkeypatch.delenv("LMPC_DENSE")
    p30, H30, _, _ = synth.config_batch(5, count=1)
    assert BatchedConvexQPSolver(p30, H30, max_batch=1, dense_path="gi").dense_path == "off"
    # the single-QP mirror (ConvexMpc drop-in) runs the interior point (round 3: lower latency than the dual active set)
    from legged_mpc_control_amd import ConvexQPSolver
    assert ConvexQPSolver(p.q_weights, p.r_weights, horizon=10)._dev.dense_path == "ipm"


def test_gi_step_cap_hands_over_to_riccati():
    """A dual active-set QP that reaches the step cap is solved by the Riccati kernel in the same
    launch: same optimum, and its iteration word carries the interior-point counts (polish rounds
    >= 1 in the high bits) instead of the active-set steps."""
    p, H, rec, con = synth.config_batch(2, count=256, first_index=4242)
    g, st, it = BatchedConvexQPSolver(p, H, max_batch=256, dense_path="gi",
                                      options=solver_options(gi_max_steps=20)).solve(rec, con)
    g2, st2, it2 = BatchedConvexQPSolver(p, H, max_batch=256, dense_path="gi",
                                         options=solver_options(gi_max_steps=1000)).solve(rec, con)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    assert fails == 0 and np.all(st == 0) and np.all(st2 == 0)
    handed = (it2 & 0xFFFF) > 20
    assert 0 < handed.sum() < 256
    assert np.all((it[handed] >> 16) >= 1)        # Riccati: polish rounds in the high bits
    assert np.array_equal(it[~handed], it2[~handed])
    assert rel_err(g, ref) <= TOL_REGRESS and rel_err(g2, ref) <= TOL_REGRESS


@pytest.mark.parametrize("cid", [5, 2])
def test_warm_start(cid):
    """lmpc_solve_batch_warm: the polish from a verified set re-verifies in one round with no interior-point
    iteration and the same answer; from a neighbouring QP's set (perturbed state) it reaches the perturbed QP's
    optimum in fewer iterations than cold; from arbitrary bytes it falls back to the cold interior point."""
    p, H, rec, con = synth.config_batch(cid, count=64, first_index=777)
    s = BatchedConvexQPSolver(p, H, max_batch=64)
    op = O.params_from(p)
    g0, st0, it0, a0 = s.solve_warm(rec, con)  # cold, on the Riccati kernel
    ref, _, fails = O.solve_batch(op, H, rec, con, n_threads=8)
    assert fails == 0 and np.all(st0 == 0) and rel_err(g0, ref) <= TOL_REGRESS
    assert np.all(a0[con == 0] == 0)
    g1, st1, it1, a1 = s.solve_warm(rec, con, act_in=a0)
    assert np.all(st1 == 0) and np.all((it1 & 0xFFFF) == 0) and np.all((it1 >> 16) == 1)
    assert np.array_equal(a1, a0) and rel_err(g1, g0) <= 1e-12
    rec2 = rec.copy()
    rec2[:, 6:12] += np.random.default_rng(cid).normal(0.0, 0.02, (64, 6))  # angular / linear velocity
    ref2, _, fails = O.solve_batch(op, H, rec2, con, n_threads=8)
    gw, stw, itw, _ = s.solve_warm(rec2, con, act_in=a0)
    gc, stc, itc, _ = s.solve_warm(rec2, con)
    assert fails == 0 and np.all(stw == 0) and np.all(stc == 0)
    assert rel_err(gw, ref2) <= TOL_REGRESS and rel_err(gc, ref2) <= TOL_REGRESS
    work = lambda it: 2 * (it & 0xFFFF) + (it >> 16)  # solves per QP
    assert work(itw).mean() < 0.5 * work(itc).mean()
    junk = np.random.default_rng(1).integers(0, 256, a0.shape).astype(np.uint8)
    gj, stj, _, _ = s.solve_warm(rec, con, act_in=junk)
    assert np.all(stj == 0) and rel_err(gj, ref) <= TOL_REGRESS
    sh = BatchedConvexQPSolver.shift_active_set(a0)
    assert np.array_equal(sh[:, :-1], a0[:, 1:]) and np.array_equal(sh[:, -1], a0[:, -1])


@pytest.mark.parametrize("path", ["host", "device"])
def test_ipm_iteration_cap_hands_over_to_riccati(path, torch_dev):
    """A condensed interior-point QP left without a verified optimum is solved by the Riccati kernel in the same
    call, as the dual active set's are: with the dense kernel capped at 3 iterations
    (lmpc_options.dense_iter_cap) every config-2 QP is handed over, so the answer, status and iteration word are the
    Riccati kernel's own, bit for bit."""
    import torch

    p, H, rec, con = synth.config_batch(2, count=256, first_index=606)

    def run(mode, cap=0):
        s = BatchedConvexQPSolver(p, H, max_batch=256, dense_path=mode, options=solver_options(dense_iter_cap=cap))
        if path == "host":
            return s.solve(rec, con)
        out = torch.empty((256, H, 12), dtype=torch.float64, device=torch_dev)
        st = torch.empty(256, dtype=torch.int32, device=torch_dev)
        it = torch.empty(256, dtype=torch.int32, device=torch_dev)
        s.solve_device(torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev), out, st, it)
        torch.cuda.synchronize()
        return out.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()

    gc, sc, ic = run("ipm", 3)
    gd, sd, idn = run("ipm")
    gr, sr, ir = run("off")
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    assert fails == 0 and np.all(sc == 0) and np.all(sd == 0) and np.all(sr == 0)
    assert np.all((idn & 0xFFFF) > 3)                       # uncapped: every QP needs more than 3 iterations
    assert np.array_equal(gc, gr) and np.array_equal(ic, ir)  # capped: all solved by the Riccati kernel
    assert rel_err(gc, ref) <= TOL_REGRESS and rel_err(gd, ref) <= TOL_REGRESS


@pytest.mark.parametrize("cid", [2, 4])
def test_fused_launch_equals_two_launches(cid, torch_dev):
    """At most one QP per SIMD (batch <= 4 x CUs) the device path runs the dense interior point and the Riccati
    fallback as one launch (lmpc_dense_lq_kernel, round 5); one QP more and it launches the two kernels (the Riccati
    one in its two-wave instance).  The QPs both batches share get the same bits: config 2 (every QP on the dense
    path) and config 4's mixed gaits with terrain (a quarter dense-eligible, the rest solved by the Riccati body
    inside the fused kernel)."""
    import torch

    cus = torch.cuda.get_device_properties(torch_dev).multi_processor_count
    n = 4 * cus
    p, H, rec, con = synth.config_batch(cid, count=n + 1)
    nrm = synth.config_normals(cid, n + 1) if cid == 4 else None
    s = BatchedConvexQPSolver(p, H, max_batch=0, dense_path="ipm")

    def run(b):
        out = torch.empty((b, H, 12), dtype=torch.float64, device=torch_dev)
        st = torch.empty(b, dtype=torch.int32, device=torch_dev)
        it = torch.empty(b, dtype=torch.int32, device=torch_dev)
        d_nrm = None if nrm is None else torch.from_numpy(nrm[:b]).to(torch_dev).contiguous()
        s.solve_device(torch.from_numpy(rec[:b]).to(torch_dev), torch.from_numpy(con[:b]).to(torch_dev), out, st, it,
                       normals=d_nrm)
        torch.cuda.synchronize()
        return out.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()

    g1, s1, i1 = run(n)      # fused
    g2, s2, i2 = run(n + 1)  # two launches
    assert np.all(s1 == 0) and np.all(s2 == 0)
    assert np.array_equal(g1, g2[:n]) and np.array_equal(i1, i2[:n])
    idx = np.random.default_rng(cid).choice(n, 16, replace=False)
    ref, _, fails = O.solve_batch(O.params_from(p), H, rec[idx], con[idx], n_threads=8,
                                  normals=None if nrm is None else nrm[idx])
    assert fails == 0 and rel_err(g1[idx], ref) <= TOL


def test_mixed_streams_and_host_path_share_one_context(torch_dev):
    """One context, three calls in flight: an asynchronous device solve on stream A (Riccati kernel: per-QP
    factor scratch), a host-pointer solve (the context's own stream, same scratch slots) issued before A has
    finished, then a device solve on stream B.  The context orders them, so each result equals the
    same solve run alone.  The caller's current device is left as it was."""
    import torch

    p, H, rec, con = synth.config_batch(3, count=4096, first_index=1)    # H = 20: ~7 ms of Riccati kernel
    _, _, rec2, con2 = synth.config_batch(3, count=512, first_index=90001)
    _, _, rec3, con3 = synth.config_batch(3, count=2048, first_index=50001)
    s = BatchedConvexQPSolver(p, H, max_batch=512)

    def alone_device(r, c):
        out = torch.empty((r.shape[0], H, 12), dtype=torch.float64, device=torch_dev)
        s.solve_device(torch.from_numpy(r).to(torch_dev), torch.from_numpy(c).to(torch_dev), out)
        torch.cuda.synchronize()
        return out.cpu().numpy()

    ref1, ref3 = alone_device(rec, con), alone_device(rec3, con3)
    ref2, st2, _ = s.solve(rec2, con2)
    assert np.all(st2 == 0)
    dev_before = torch.cuda.current_device()
    a, b = torch.cuda.Stream(torch_dev), torch.cuda.Stream(torch_dev)
    d1 = (torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev))
    d3 = (torch.from_numpy(rec3).to(torch_dev), torch.from_numpy(con3).to(torch_dev))
    torch.cuda.synchronize()
    o1 = torch.empty((rec.shape[0], H, 12), dtype=torch.float64, device=torch_dev)
    o3 = torch.empty((rec3.shape[0], H, 12), dtype=torch.float64, device=torch_dev)
    s.solve_device(d1[0], d1[1], o1, stream=a)      # returns at once; the kernel runs for milliseconds
    g2, st2b, _ = s.solve(rec2, con2)              # host path on the context's stream, same scratch slots
    s.solve_device(d3[0], d3[1], o3, stream=b)
    torch.cuda.synchronize()
    assert torch.cuda.current_device() == dev_before
    assert np.array_equal(o1.cpu().numpy(), ref1)
    assert np.array_equal(g2, ref2) and np.all(st2b == 0)
    assert np.array_equal(o3.cpu().numpy(), ref3)


def test_stream_gone_before_the_next_call(torch_dev):
    """Round 6: a context records its cross-stream ordering event only when the stream changes, so a device-path call
    on a caller's stream A leaves nothing recorded on A.  If A is destroyed right after that call (its solve still
    running), the context's next host-pointer call, lmpc_sync and lmpc_destroy must wait for the device instead of
    touching A: no crash, and every result equals the same solve run alone."""
    import ctypes

    import torch

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    p, H, rec, con = synth.config_batch(3, count=4096, first_index=7)     # H = 20: milliseconds of Riccati kernel
    _, _, rec2, con2 = synth.config_batch(3, count=512, first_index=70001)
    s = BatchedConvexQPSolver(p, H, max_batch=512)
    d_rec, d_con = torch.from_numpy(rec).to(torch_dev), torch.from_numpy(con).to(torch_dev)
    ref1 = torch.empty((rec.shape[0], H, 12), dtype=torch.float64, device=torch_dev)
    s.solve_device(d_rec, d_con, ref1)
    torch.cuda.synchronize()
    ref2, _, _ = s.solve(rec2, con2)
    for after in ("host", "sync", "destroy"):
        t = BatchedConvexQPSolver(p, H, max_batch=512)
        a = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(a), 1) == 0  # hipStreamNonBlocking
        out = torch.empty_like(ref1)
        torch.cuda.synchronize()
        t.solve_device(d_rec, d_con, out, stream=a.value)   # returns at once
        assert hip.hipStreamDestroy(a) == 0                 # the caller's stream is gone; its solve may still run
        if after == "host":
            g2, st2, _ = t.solve(rec2, con2)               # host path: waits for the device, never for A
            assert np.array_equal(g2, ref2) and np.all(st2 == 0)
        elif after == "sync":
            t.sync()
        t.close()
        torch.cuda.synchronize()
        assert torch.equal(out, ref1), after


def test_python_dropin_warm_ticks_match_oracle():
    """The Python drop-in warm-starts by default, like the C++ one: over consecutive ticks of a trot (FSM phase
    advancing, state drifting) every tick's u_0 equals the oracle's, and the later ticks re-verify the shifted
    active set with few interior-point iterations."""
    from legged_mpc_control_amd import ConvexQPSolver, LeggedContactFSM, LeggedState

    p = synth.params("go1")
    H = 10
    solver = ConvexQPSolver(p.q_weights, p.r_weights, horizon=H)
    assert solver.warm_start
    st = LeggedState()
    st.param.gait_counter_speed = 4.0
    fsm = [LeggedContactFSM() for _ in range(4)]
    for i in range(4):
        fsm[i].reset_params(st, i)
        fsm[i].gait_phase = 0.1
    feet = np.array([[0.17, 0.12, -0.3], [0.17, -0.17, -0.3], [-0.17, 0.17, -0.3], [-0.17, -0.12, -0.3]]).T
    st.ctrl.root_pos_d = np.array([0, 0, 0.28])
    st.ctrl.root_lin_vel_d_rel = np.array([0.4, 0.0, 0.0])
    op = O.params_from(p)
    ipm = []
    for tick in range(6):
        st.fbk.root_pos = np.array([0.004 * tick, 0.0, 0.27])
        st.fbk.root_lin_vel = np.array([0.4, 0.0, 0.0])
        st.fbk.foot_pos_abs = feet
        for i in range(4):
            st.ctrl.plan_contacts[i] = bool(fsm[i].get_contact_state())
        solver.calc_mpc_reference(st, fsm)
        u0 = solver.compute_grfs(st)
        ref, _, _ = O.solve(op, H, solver._rec[0], solver._con[0])
        assert solver.last_status == 0 and rel_err(u0, ref[0]) <= TOL_REGRESS, tick
        ipm.append(solver.last_iterations & 0xFFFF)
        for i in range(4):
            fsm[i].gait_phase = (fsm[i].gait_phase + 4.0 * 0.01) % 1.0
    assert ipm[0] > 0 and min(ipm[1:]) == 0  # tick 0 cold; later ticks start from the shifted verified set


def test_eigen_signature_dropin_vs_oracle():
    """include/lmpc/ConvexQPSolverEigen.hpp under the reference's own ConvexMpc lines (ConvexMpc.cpp:13-14,70-75,
    tests/cpp/eigen_dropin_test.cpp; Eigen and the reference headers are test stand-ins here): u_0 of every tick equals
    the oracle's on the record and schedule the program reports, the horizon is the reference's PLAN_HORIZON (30),
    v_d_world is written back (ConvexQPSolver.cpp:260), and warm-started later ticks need fewer iterations."""
    from legged_mpc_control_amd import build as B

    exe = B.build_cpp_eigen_test()
    out = subprocess.run([exe, "3"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    p = synth.params("go1")
    op = O.params_from(p)
    H = 30
    assert len(lines) == 15
    for i in range(0, len(lines), 5):
        assert lines[i].endswith("status 0")
        rec = np.array(lines[i + 1].split()[1:], dtype=np.float64)
        con = np.array(lines[i + 2].split()[1:], dtype=np.uint8).reshape(H, 4)
        vdw = np.array(lines[i + 3].split()[1:], dtype=np.float64)
        u0 = np.array(lines[i + 4].split()[1:], dtype=np.float64)
        assert rec.size == 33 + 12 * H
        R = rec[12:21].reshape(3, 3)
        np.testing.assert_allclose(vdw, R @ np.array([0.4, 0.0, 0.0]), rtol=0, atol=1e-15)
        ref, _, _ = O.solve(op, H, rec, con)
        assert rel_err(u0, ref[0]) <= TOL_REGRESS

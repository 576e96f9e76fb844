"""The LDS-resident Riccati kernel (csrc/lmpc_lq.hip, round 4) against the exact oracle and against the global-
workspace Riccati kernel it replaces for cold solves (lmpc_set_riccati_path).

Every QP is checked against oracle/ (the CPU restatement of ConvexQPSolver.cpp:16-346, solved exactly): the
committed golden fixtures (every config and edge set, terrain included), live samples of configs 2-5 with the dense
path off (so every QP runs on this kernel), horizons 1..32 (both leg-step layouts), and the status / NaN contract.
Tolerance: the bench's parity bar |f_gpu - f_ref| / max(1, |f_ref|) <= 1e-7 (the north star asks 1e-4).
"""
import os

import numpy as np
import pytest

from conftest import golden_files, lmpc_params_from, load_golden

TOL = 1e-7


@pytest.fixture
def torch_dev():
    import torch

    return torch.device("cuda:0")


def _solver(p, H, batch, dense="off", riccati="lds", **kw):
    from legged_mpc_control_amd import BatchedConvexQPSolver

    return BatchedConvexQPSolver(p, H, max_batch=batch, dense_path=dense, riccati_path=riccati, **kw)


def _oracle(p, H, rec, con, nrm=None):
    from oracle import oracle as O

    ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8, normals=nrm)
    return ref


def _err(g, ref):
    return float(np.max(np.abs(g - ref) / np.maximum(1.0, np.abs(ref))))


@pytest.mark.gpu
@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p))
def test_lq_golden_fixtures(path):
    d = load_golden(path)
    p, H, rec, con, ref = lmpc_params_from(d["params"]), d["H"], d["rec"], d["contact"], d["grf"]
    nrm = d["normals"]
    g, st, _ = _solver(p, H, rec.shape[0]).solve(rec, con, normals=nrm)
    assert (st == 0).all(), st
    assert _err(g, ref) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("cid,count,first", [(2, 256, 5000), (3, 64, 777), (4, 512, 12345), (5, 32, 99)])
def test_lq_live_samples_vs_oracle(cid, count, first):
    from legged_mpc_control_amd import synth

    p, H, rec, con = synth.config_batch(cid, count=count, first_index=first)
    nrm = synth.config_normals(cid, count, first) if cid == 4 else None
    g, st, it = _solver(p, H, count).solve(rec, con, normals=nrm)
    assert (st == 0).all(), np.unique(st, return_counts=True)
    assert _err(g, _oracle(p, H, rec, con, nrm)) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("cid", [2, 4])
def test_lq_two_wave_instance_vs_oracle(cid):
    """Batches of more than one QP per SIMD run the two-waves-per-SIMD instance (at H <= 10 with the closed-loop
    rows in LDS, a different forward-sweep formula): every QP of a 2048-QP batch against the oracle."""
    from legged_mpc_control_amd import synth

    count = 2048
    p, H, rec, con = synth.config_batch(cid, count=count, first_index=3 * cid)
    nrm = synth.config_normals(cid, count, 3 * cid) if cid == 4 else None
    g, st, _ = _solver(p, H, count).solve(rec, con, normals=nrm)
    assert (st == 0).all(), np.unique(st, return_counts=True)
    assert _err(g, _oracle(p, H, rec, con, nrm)) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("H,terrain", [(4, False), (7, True), (11, False), (11, True), (16, False), (16, True),
                                       (17, False), (20, False), (20, True), (21, False), (26, False)])
def test_lq_two_wave_instance_other_horizons(H, terrain):
    """the two-waves-per-SIMD instance (batches above one QP per SIMD) at H != 10 -- H < 10 and H = 11..16,
    where the closed-loop rows are not kept (H > 10), and since round 6 H = 17..21 (two leg-steps per lane, six or
    more QPs per CU; H = 26 keeps the lone wave) -- with and without terrain: every QP of a 2048-QP batch against the oracle, and the batch's bits
    equal to the lone-wave instance's on 512 of the same records (a QP's answer must not depend on the batch it is
    solved in)."""
    from legged_mpc_control_amd import synth

    count = 2048
    p, _, rec, con = synth.config_batch(4, count=count, first_index=100 * H, H=H)
    nrm = synth.config_normals(4, count, 100 * H) if terrain else None
    g, st, _ = _solver(p, H, count).solve(rec, con, normals=nrm)
    assert (st == 0).all(), np.unique(st, return_counts=True)
    assert _err(g, _oracle(p, H, rec, con, nrm)) <= TOL
    sl = slice(256, 768)
    g1, st1, _ = _solver(p, H, 512).solve(rec[sl], con[sl], normals=None if nrm is None else nrm[sl])
    assert np.array_equal(st1, st[sl]) and np.array_equal(g1, g[sl])


@pytest.mark.gpu
@pytest.mark.parametrize("H", [1, 2, 10, 16, 17, 32])
def test_lq_horizon_range(H):
    """LS = 1 (H <= 16, two waves per SIMD) and LS = 2 (H > 16) instances, the whole horizon range."""
    from legged_mpc_control_amd import synth

    p, _, rec, con = synth.config_batch(2, count=64, first_index=31 * H, H=H)
    g, st, _ = _solver(p, H, 64).solve(rec, con)
    assert (st == 0).all()
    assert _err(g, _oracle(p, H, rec, con)) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("cid", [2, 4, 5])
def test_lq_agrees_with_scratch_kernel(cid):
    """Both Riccati kernels return the same verified optimum (to rounding) and the same status."""
    from legged_mpc_control_amd import synth

    count = 256
    p, H, rec, con = synth.config_batch(cid, count=count, first_index=4242)
    nrm = synth.config_normals(cid, count, 4242) if cid == 4 else None
    g1, s1, _ = _solver(p, H, count, riccati="lds").solve(rec, con, normals=nrm)
    g2, s2, _ = _solver(p, H, count, riccati="scratch").solve(rec, con, normals=nrm)
    assert (s1 == s2).all()
    assert _err(g1, g2) <= TOL


@pytest.mark.gpu
def test_lq_edge_cases_and_status():
    """All-swing QPs (zeros, converged), a NaN record (zeros, LMPC_QP_NAN), and QPs beside them unaffected."""
    from legged_mpc_control_amd import synth

    p, H, rec, con = synth.config_batch(4, count=16, first_index=7)
    con = con.copy()
    rec = rec.copy()
    con[3] = 0                      # every leg swinging over the whole horizon
    con[5, :4] = 0                  # step 0 all swing
    rec[9, 40] = np.nan             # a NaN in x_ref
    g, st, _ = _solver(p, H, 16).solve(rec, con)
    assert st[3] == 0 and np.all(g[3] == 0.0)
    assert st[9] == 2 and np.all(g[9] == 0.0)
    keep = [b for b in range(16) if b not in (3, 9)]
    assert (st[keep] == 0).all()
    assert _err(g[keep], _oracle(p, H, rec[keep], con[keep])) <= TOL


@pytest.mark.gpu
def test_lq_is_the_default_and_device_path_matches_host_path(torch_dev):
    """A context runs the LDS kernel unless told otherwise; the device-pointer entry point gives the host path's bits."""
    import torch

    from legged_mpc_control_amd import BatchedConvexQPSolver, synth

    p, H, rec, con = synth.config_batch(3, count=96, first_index=11)
    s = BatchedConvexQPSolver(p, H, max_batch=96)
    assert s.riccati_path == "lds"
    g, st, _ = s.solve(rec, con)
    d_rec = torch.from_numpy(rec).to(torch_dev)
    d_con = torch.from_numpy(con).to(torch_dev)
    d_g = torch.empty((96, H, 12), dtype=torch.float64, device=torch_dev)
    d_s = torch.empty(96, dtype=torch.int32, device=torch_dev)
    s.solve_device(d_rec, d_con, d_g, d_s)
    torch.cuda.synchronize()
    assert np.array_equal(d_g.cpu().numpy(), g) and np.array_equal(d_s.cpu().numpy(), st)

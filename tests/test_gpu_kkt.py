"""Status 0 is a KKT certificate.

Every kernel's polish verification now checks, besides primal feasibility and the multiplier signs, that the gradient
vanishes on each stance leg-step's free directions (lmpc_kernel_common.h leg_kkt: |g + C_S'z| with the least-squares
multipliers z, legs with no active face included), and the Riccati kernels check that the trajectory the forward sweep
produced is the dynamics of the returned forces (x_{k+1} = A_k x_k + B u_k - g dt e11, ConvexQPSolver.cpp:198-228,294-297).

The proof, with test-only builds of the library (legged_mpc_control_amd/build.py TEST_VARIANTS) that re-inject bugs
into the LDS Riccati kernel's forward sweep (csrc/lmpc_lq.hip):
  - round 4's lost "+ za" (w = Z x without za, LMPC_BUG_ZA) is never certified (golden_config1: status != 0);
  - the next stage's yaw read for A_k (LMPC_BUG_YAW) leaves forces that are feasible and consistent with the wrong
    trajectory: round 4's verification (LMPC_KKT_OFF) returns status 0 on most QPs with relative errors of order 1,
    the product's verification on none.  Reference: ConvexQPSolver.cpp:318-326 (the reference ignores
OSQP's status; this build's status must mean what it says).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN, lmpc_params_from, load_golden, rel_err


def _variant(tag):
    """A test-only library variant (legged_mpc_control_amd/build.py TEST_VARIANTS), loaded beside the product."""
    from legged_mpc_control_amd import _native as N
    from legged_mpc_control_amd import build as B

    path = B.build_test_variants()[tag]
    L = ctypes.CDLL(path)
    vp, dp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
    i32p, u8p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint8)
    L.lmpc_create.argtypes = [ctypes.POINTER(N.LmpcParams), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L.lmpc_set_dense_path.argtypes = [vp, ctypes.c_int]
    L.lmpc_solve_batch_ex.argtypes = [vp, dp, u8p, dp, ctypes.c_int, dp, i32p, i32p]
    L.lmpc_destroy.argtypes = [vp]
    L.lmpc_destroy.restype = None
    return L


def _solve_with(L, p, H, rec, con, dense=0):
    B = rec.shape[0]
    ctx = ctypes.c_void_p()
    assert L.lmpc_create(ctypes.byref(p), H, B, 0, ctypes.byref(ctx)) == 0
    try:
        assert L.lmpc_set_dense_path(ctx, dense) == 0
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        con = np.ascontiguousarray(con, dtype=np.uint8)
        g = np.zeros((B, H, 12))
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros(B, dtype=np.int32)
        dp, i32 = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
        rc = L.lmpc_solve_batch_ex(ctx, rec.ctypes.data_as(dp), con.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), None,
                                   B, g.ctypes.data_as(dp), st.ctypes.data_as(i32), it.ctypes.data_as(i32))
        assert rc == 0
        return g, st, it
    finally:
        L.lmpc_destroy(ctx)


def _per_qp_err(g, ref):
    return np.max(np.abs(g - ref) / np.maximum(1.0, np.abs(ref)), axis=(1, 2))


def _workloads():
    """The LDS Riccati kernel's code paths: the A1-standing golden QP (one leg-step per lane, closed-loop rows, lone
    wave), a config-3 sample (two leg-steps per lane: the w = Z x + za sweep) and a config-2 batch of 2048 QPs with
    the dense path off (two waves per SIMD)."""
    from legged_mpc_control_amd import synth
    from oracle import oracle as O

    d = load_golden(os.path.join(GOLDEN, "golden_config1_a1_standing_h10.npz"))
    out = [("golden_config1", lmpc_params_from(d["params"]), d["H"], d["rec"], d["contact"], d["grf"])]
    for cid, count, first in ((3, 64, 4321), (2, 2048, 8765)):
        p, H, rec, con = synth.config_batch(cid, count=count, first_index=first)
        ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
        out.append((f"config{cid}@{count}", p, H, rec, con, ref))
    return out


@pytest.fixture(scope="module")
def workloads():
    return _workloads()


def _run(tag, workloads, bar):
    """Solve every workload with a variant -> [(name, status, per-QP error, wrong answers carrying status 0)]."""
    L = _variant(tag)
    out = []
    for name, p, H, rec, con, ref in workloads:
        g, st, _ = _solve_with(L, p, H, rec, con)
        err = _per_qp_err(g, ref)
        bad = int(((st == 0) & (err > bar)).sum())
        print(f"{tag}, {name}: status {np.bincount(st, minlength=3)}, wrong answers with status 0: {bad}, "
              f"max err {err.max():.3g}")
        out.append((name, st, err, bad))
    return out


@pytest.mark.gpu
def test_reinjected_za_bug_is_never_certified(workloads):
    """round 4's lost "+ za" in the forward sweep, re-injected (LMPC_BUG_ZA), returns status != 0
    on golden_config1 (round 4's kernel returned status 0 there, relative error 1.03), and no wrong answer anywhere
    carries status 0."""
    for name, st, err, bad in _run("bugza", workloads, 1e-7):
        assert bad == 0, name
        if name == "golden_config1":
            assert (st != 0).all(), st


@pytest.mark.gpu
def test_round4_verification_certifies_wrong_forces(workloads):
    """The hole the certificate closes: the next stage's yaw read for A_k in the forward sweep (LMPC_BUG_YAW) leaves the
    forces consistent with the (wrong) trajectory the kernel swept -- feasible, multipliers of the right sign -- so round
    4's verification (LMPC_KKT_OFF) returns status 0 on most QPs with errors of order 1."""
    slipped = sum(bad for _, _, _, bad in _run("bugyaw_nokkt", workloads, 1e-5))
    assert slipped > 0, "the re-injected bug no longer slips through round 4's verification: this test proves nothing"


@pytest.mark.gpu
def test_certificate_rejects_the_wrong_forces(workloads):
    """The same bug under the product's verification: the dynamics and stationarity checks reject every wrong answer
    (they go to the retry ladder and end unverified); a QP the bug does not touch (the standing golden QP: zero yaw
    rate) still verifies."""
    for name, st, err, bad in _run("bugyaw", workloads, 1e-7):
        assert bad == 0, name
        if name == "golden_config1":
            assert (st == 0).all() and err.max() <= 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize("dense", ["off", "ipm", "gi"])
def test_certificate_passes_every_golden_qp(dense):
    """The product build: every committed golden QP still verifies (status 0) on every path, at the parity bar."""
    import glob

    from legged_mpc_control_amd import BatchedConvexQPSolver

    for path in sorted(glob.glob(os.path.join(GOLDEN, "golden_*.npz"))):
        d = load_golden(path)
        p, H = lmpc_params_from(d["params"]), d["H"]
        s = BatchedConvexQPSolver(p, H, max_batch=d["rec"].shape[0], dense_path=dense)
        g, st, _ = s.solve(d["rec"], d["contact"], normals=d["normals"])
        assert (st == 0).all(), (os.path.basename(path), st)
        assert rel_err(g, d["grf"]) <= 1e-7, os.path.basename(path)


@pytest.mark.gpu
def test_range_space_rounds_match_refactorised_rounds():
    """the dense polish's range-space rounds (rows-only and bordered updates of the last factorisation,
    lmpc_dense_kernel.h) against a build that refactorises every round (LMPC_POLISH_SCHUR=0): the same iteration words
    and status on a config-2 batch, forces within rounding of each other and of the oracle -- and not bit-identical
    (so the updates really ran).  The batch is the bench's first 1024 QPs, which holds the QP whose update ended
    1.8e-9 from the optimum in round 5; the refinement of such rounds (LMPC_POLISH_REFINE) brings it back to <= 2e-10."""
    from legged_mpc_control_amd import _native as N
    from legged_mpc_control_amd import synth
    from oracle import oracle as O

    p, H, rec, con = synth.config_batch(2, count=1024, first_index=0)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8)
    g0, st0, it0 = _solve_with(N.lib(), p, H, rec, con, dense=1)
    g1, st1, it1 = _solve_with(_variant("noschur"), p, H, rec, con, dense=1)
    assert (st0 == 0).all() and (st1 == 0).all()
    assert (it0 == it1).all(), f"iteration words differ on {(it0 != it1).sum()} QPs"
    e0, e1 = _per_qp_err(g0, ref), _per_qp_err(g1, ref)
    print(f"range-space updates: max err {e0.max():.3g}; refactorised: {e1.max():.3g}; "
          f"QPs whose bits differ: {(g0 != g1).any(axis=(1, 2)).sum()}")
    assert e0.max() <= 2e-10 and e1.max() <= 2e-10
    assert np.max(np.abs(g0 - g1)) <= 1e-9
    assert (g0 != g1).any(axis=(1, 2)).sum() > 0, "no range-space round ran: the test proves nothing"

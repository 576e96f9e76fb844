"""The reference's solver, OSQP (absent here; oracle/osqp_restate.py restates its published ADMM with the
reference's settings, ConvexQPSolver.cpp:182-194), against the exact optimum the oracle and the kernels
return.  CPU only."""
import numpy as np
import pytest

from conftest import golden_files, load_golden, lmpc_params_from
from oracle import oracle as O
from oracle import osqp_restate as Q


def _golden(name):
    path = [p for p in golden_files() if name in p][0]
    g = load_golden(path)
    return lmpc_params_from(g["params"]), g


def _exact_point(P, q, A, l, grf, H):
    """Full sparse-QP point of the exact optimum: u from the oracle, states from the dynamics rows."""
    n, dyn = 24 * H, 12 * H
    x = np.zeros(n)
    ucols = [c for i in range(H) for c in range(24 * i, 24 * i + 12)]
    xcols = [c for i in range(H) for c in range(24 * i + 12, 24 * i + 24)]
    x[ucols] = grf.reshape(-1)
    x[xcols] = np.linalg.solve(A[:dyn][:, xcols], l[:dyn] - A[:dyn][:, ucols] @ x[ucols])
    return x


@pytest.mark.parametrize("name,b", [("config1", 0), ("config2", 3)])
def test_restated_osqp_converges_to_the_exact_optimum(name, b):
    """Pins the restatement: with tight tolerances it converges to the oracle's optimum."""
    p, g = _golden(name)
    op = O.params_from(p)
    grf, info = Q.grf(op, g["H"], g["rec"][b], g["contact"][b], eps_abs=1e-9, eps_rel=1e-10, max_iter=100000)
    assert info["converged"]
    assert np.max(np.abs(grf - g["grf"][b])) <= 1e-2


def test_reference_settings_give_an_approximate_optimum():
    """At the reference's settings (eps_abs 1e-3, eps_rel 1e-4, cold start) OSQP stops at an
    approximate optimum: its objective is above the exact one, and the exact optimum is feasible.
    The force difference is large along the cost's flat directions."""
    p, g = _golden("config2")
    op = O.params_from(p)
    H = g["H"]
    gaps, du0 = [], []
    for b in range(4):
        P, q, A, l, u = O.build_sparse_qp(op, H, g["rec"][b], g["contact"][b])
        x, info = Q.solve(P, q, A, l, u)
        assert info["converged"] and info["iters"] < 4000
        xe = _exact_point(P, q, A, l, g["grf"][b], H)
        Axe = A @ xe
        assert np.all(Axe >= l - 1e-7) and np.all(Axe <= u + 1e-7)
        f = lambda v: 0.5 * v @ (P * v) + q @ v  # noqa: E731
        gaps.append((f(x) - f(xe)) / max(1.0, abs(f(xe))))
        du0.append(np.max(np.abs(x[:12] - xe[:12])))
    assert min(gaps) > -1e-9          # the exact optimum is never beaten
    assert max(gaps) < 0.1            # OSQP is close in objective ...
    assert max(du0) > 1.0             # ... but not in force space


@pytest.mark.parametrize("name", ["config2", "config4t", "config5"])
def test_c_admm_restatement_matches_numpy(name):
    """oracle/osqp_admm.c (the CPU baseline bench.py times as the reference's algorithm) takes the numpy
    restatement's iterates: same termination iteration, same point to rounding (it solves the reduced KKT system
    by an envelope Cholesky instead of numpy's dense one), on flat and terrain instances."""
    p, g = _golden(name)
    op = O.params_from(p)
    H = g["H"]
    for b in range(min(3, g["rec"].shape[0])):
        nrm = None if g["normals"] is None else g["normals"][b]
        P, q, A, l, u = O.build_sparse_qp(op, H, g["rec"][b], g["contact"][b], nrm)
        xr, info = Q.solve(P, q, A, l, u)
        xc, it, cv, _ = O.osqp_solve(P, q, A, l, u)
        assert it == info["iters"] and cv == info["converged"]
        assert np.max(np.abs(xc - xr)) <= 1e-6 * max(1.0, np.max(np.abs(xr)))
    # the batch entry point returns each instance's u_0..u_{H-1}, as Q.grf does
    B = min(4, g["rec"].shape[0])
    grf, iters, conv = O.osqp_grf_batch(op, H, g["rec"][:B], g["contact"][:B], n_threads=2,
                                        normals=None if g["normals"] is None else g["normals"][:B])
    for b in range(B):
        gr, info = Q.grf(op, H, g["rec"][b], g["contact"][b], None if g["normals"] is None else g["normals"][b])
        assert iters[b] == info["iters"] and conv[b]
        assert np.max(np.abs(grf[b] - gr)) <= 1e-6 * max(1.0, np.max(np.abs(gr)))

"""Restatement of the reference's QP solver, OSQP, for parity checks (TEST INFRASTRUCTURE ONLY).

The reference solves its convex-MPC QP with OSQP through OsqpEigen
(src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:182-194 settings, :314-327 solve).
OSQP is a third-party dependency that is not vendored in the reference: the Dockerfile clones
github.com/oxfordcontrol/osqp at an unpinned HEAD (.devcontainer/Dockerfile:55; image dated
2022-10-03, so the v0.6.x line).  This module restates its published algorithm -- B. Stellato et al.,
"OSQP: an operator splitting solver for quadratic programs", Math. Prog. Comp. 12 (2020), Alg. 1,
with the v0.6 implementation choices -- on the exact sparse problem the reference builds
(oracle.build_sparse_qp), so the tests can show what the reference's solver returns: an
approximation of the unique optimum, within its own termination tolerances.

Settings: the reference's (eps_abs 1e-3, eps_rel 1e-4, warm start; ConvexQPSolver.cpp:183-185) and
OSQP 0.6 defaults for the rest: rho 0.1, sigma 1e-6, alpha 1.6, Ruiz scaling 10 passes (bounds
[1e-4, 1e4]), rho 1e3x on equality rows and 1e-6 on free rows, termination checked every 25
iterations on unscaled residuals, max_iter 4000, polish off.  Adaptive rho uses the fixed
interval of 4 termination checks (100 iterations): OSQP's default derives the interval from the
measured setup time when built with profiling, which no restatement can reproduce.  Instances
here are independent, so every solve starts cold (x = z = y = 0), as the reference's first tick does.

Linear algebra: OSQP factors the quasi-definite KKT matrix [P + sigma I, A'; A, -diag(1/rho)] with
QDLDL; this restatement solves the equivalent reduced system (P + sigma I + A' diag(rho) A) x = r
with a dense Cholesky.  Both give the same iterates up to rounding.
"""
from __future__ import annotations

import numpy as np

OSQP_INFTY = 1e30
RHO_MIN, RHO_MAX = 1e-6, 1e6
RHO_EQ_OVER_RHO_INEQ = 1e3
RHO_TOL = 1e-4
MIN_SCALING, MAX_SCALING = 1e-4, 1e4
ADAPTIVE_RHO_TOLERANCE = 5.0


def _limit(v):
    v = np.where(v < MIN_SCALING, 1.0, v)
    return np.minimum(v, MAX_SCALING)


def _ruiz(P, q, A, iters):
    """OSQP scale_data: modified Ruiz equilibration of [P A'; A 0] plus cost scaling c."""
    n, m = P.shape[0], A.shape[0]
    D, E, c = np.ones(n), np.ones(m), 1.0
    P, q, A = P.copy(), q.copy(), A.copy()
    for _ in range(iters):
        col = np.maximum(np.max(np.abs(P), axis=0), np.max(np.abs(A), axis=0) if m else 0.0)
        row = np.max(np.abs(A), axis=1) if m else np.zeros(0)
        Dt = 1.0 / np.sqrt(_limit(col))
        Et = 1.0 / np.sqrt(_limit(row))
        P = Dt[:, None] * P * Dt[None, :]
        A = Et[:, None] * A * Dt[None, :]
        q = Dt * q
        D *= Dt
        E *= Et
        cost = max(np.mean(np.max(np.abs(P), axis=0)), np.max(np.abs(q)))
        ct = 1.0 / _limit(np.array([cost]))[0]
        P *= ct
        q *= ct
        c *= ct
    return P, q, A, D, E, c


def _rho_vec(l, u, rho):
    loose = (l < -OSQP_INFTY * MIN_SCALING) & (u > OSQP_INFTY * MIN_SCALING)
    eq = (~loose) & (u - l < RHO_TOL)
    return np.where(loose, RHO_MIN, np.where(eq, RHO_EQ_OVER_RHO_INEQ * rho, rho))


def solve(Pd, q, A, l, u, eps_abs=1e-3, eps_rel=1e-4, rho=0.1, sigma=1e-6, alpha=1.6, scaling=10,
          max_iter=4000, check_termination=25, adaptive_rho_interval=100):
    """OSQP ADMM on min 1/2 x'Px + q'x s.t. l <= Ax <= u (P diagonal here: Pd = its diagonal).
    Returns (x, info) with info = {iters, converged, prim_res, dual_res, rho}."""
    P0 = np.diag(np.asarray(Pd, dtype=np.float64))
    l = np.clip(np.asarray(l, dtype=np.float64), -OSQP_INFTY, OSQP_INFTY)
    u = np.clip(np.asarray(u, dtype=np.float64), -OSQP_INFTY, OSQP_INFTY)
    P, qs, As, D, E, c = _ruiz(P0, np.asarray(q, dtype=np.float64), np.asarray(A, dtype=np.float64), scaling)
    inf_l, inf_u = l <= -OSQP_INFTY, u >= OSQP_INFTY
    ls = np.where(inf_l, -OSQP_INFTY, E * l)
    us = np.where(inf_u, OSQP_INFTY, E * u)
    n, m = P.shape[0], As.shape[0]
    rv = _rho_vec(ls, us, rho)

    def factor(rv):
        return np.linalg.cholesky(P + sigma * np.eye(n) + As.T @ (rv[:, None] * As))

    Lk = factor(rv)
    x, z, y = np.zeros(n), np.zeros(m), np.zeros(m)
    info = dict(iters=max_iter, converged=False, prim_res=np.inf, dual_res=np.inf, rho=rho)
    Dinv, Einv = 1.0 / D, 1.0 / E
    for it in range(1, max_iter + 1):
        xp, zp = x, z
        r = sigma * xp - qs + As.T @ (rv * zp - y)
        xt = np.linalg.solve(Lk.T, np.linalg.solve(Lk, r))
        zt = As @ xt
        x = alpha * xt + (1.0 - alpha) * xp
        zr = alpha * zt + (1.0 - alpha) * zp
        z = np.clip(zr + y / rv, ls, us)
        y = y + rv * (zr - z)
        check = (it % check_termination == 0) or it == max_iter
        if check:
            Ax, Px, Aty = As @ x, P @ x, As.T @ y
            prim = np.max(np.abs(Einv * (Ax - z))) if m else 0.0
            ptol = eps_abs + eps_rel * max(np.max(np.abs(Einv * Ax)), np.max(np.abs(Einv * z)))
            dual = np.max(np.abs(Dinv * (Px + qs + Aty))) / c
            dtol = eps_abs + eps_rel / c * max(np.max(np.abs(Dinv * Px)), np.max(np.abs(Dinv * Aty)),
                                               np.max(np.abs(Dinv * qs)))
            info.update(prim_res=prim, dual_res=dual)
            if prim <= ptol and dual <= dtol:
                info.update(iters=it, converged=True)
                break
        if adaptive_rho_interval and it % adaptive_rho_interval == 0:
            Ax, Px, Aty = As @ x, P @ x, As.T @ y
            pn = np.max(np.abs(Ax - z)) / (max(np.max(np.abs(Ax)), np.max(np.abs(z))) + 1e-10)
            dn = np.max(np.abs(Px + qs + Aty)) / (max(np.max(np.abs(Px)), np.max(np.abs(Aty)),
                                                      np.max(np.abs(qs))) + 1e-10)
            est = min(max(rho * np.sqrt(pn / (dn + 1e-10)), RHO_MIN), RHO_MAX)
            if est > rho * ADAPTIVE_RHO_TOLERANCE or est < rho / ADAPTIVE_RHO_TOLERANCE:
                rho = est
                rv = _rho_vec(ls, us, rho)
                Lk = factor(rv)
                info["rho"] = rho
    return D * x, info


def grf(p, H, rec, contact, normals=None, **kw):
    """The reference's compute_grfs restated: OSQP on the reference's sparse QP -> (grf[H,12], info).
    (The reference returns u_0 = grf[0] only, ConvexQPSolver.cpp:319-320.)"""
    from . import oracle as O

    P, q, A, l, u = O.build_sparse_qp(p, H, rec, contact, normals)
    x, info = solve(P, q, A, l, u, **kw)
    if not np.all(np.isfinite(x)):
        return np.zeros((H, 12)), info  # NaN -> zeros (ConvexQPSolver.cpp:321-326)
    return np.stack([x[24 * i:24 * i + 12] for i in range(H)]), info

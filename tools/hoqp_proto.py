#!/usr/bin/env python3
"""Dev tool (CPU): numpy replica of the planned HoQp device algorithm, to size iterations and accuracy before
writing the kernel.  Per level (HoQp.cpp:65-174): G = A Z, Hy = G'G + 1e-12 I, c = G'(A x - b), frozen rows
P = D_prev Z with the reference's slack pairing, current rows Dz = D Z; the level QP over (y, v) solved by a
Mehrotra interior point with the slacks v eliminated (K = Hy + R' diag(w) R, R = [P; Dz]); x += Z y;
Z <- Z ker(G) (Eigen FullPivLU basis).  Compared against oracle/hoqp.py (exact active set, x87)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import hoqp as Q  # noqa: E402


PIV_FLOOR = 1e-13   # relative to the largest diagonal entry of K
PIV_BIG = 1e64      # a pivot below the floor is replaced by this: that Cholesky coordinate does not move


def chol_floor(K):
    """Cholesky with a pivot floor: K = A'A + 1e-12 I is singular in double along ker(A) wherever no
    inequality weight acts (1e-12 is below the rounding of A'A), so pivots at rounding level freeze their
    coordinate instead of failing; along those directions the level's objective is flat at double precision."""
    n = K.shape[0]
    L = np.zeros_like(K)
    A = K.copy()
    thr = PIV_FLOOR * max(1.0, float(np.max(np.diag(K)))) if n else 0.0
    for k in range(n):
        p = A[k, k]
        if not p > thr:
            p = PIV_BIG
        d = np.sqrt(p)
        L[k, k] = d
        L[k + 1:, k] = A[k + 1:, k] / d
        A[k + 1:, k + 1:] -= np.outer(L[k + 1:, k], L[k + 1:, k])
    return L


def chol_solve(L, r):
    n = L.shape[0]
    u = np.zeros(n)
    for i in range(n):
        u[i] = (r[i] - L[i, :i] @ u[:i]) / L[i, i]
    x = np.zeros(n)
    for i in range(n - 1, -1, -1):
        x[i] = (u[i] - L[i + 1:, i] @ x[i + 1:]) / L[i, i]
    return x


def polish(Hy, c, P, h, Dz, g, y_ipm, s2, z2, s3, z3, scale, rounds=3):
    """Active-set refinement after the interior point (kernel plan): frozen rows with z > s held by an augmented
    Lagrangian (weight rho, multipliers from the IPM's z), own rows with z > s kept as 1/2 (d y - g)^2; the
    result is kept only if it verifies (feasible, consistent classification, nonnegative multipliers)."""
    p, s = P.shape[0], Dz.shape[0]
    actP = z2 > s2 if p else np.zeros(0, bool)
    slk = z3 > s3 if s else np.zeros(0, bool)
    dmax = max(1.0, float(np.max(np.diag(Hy))))
    rho = float(os.environ.get("RHO", 1e6)) * dmax
    K = Hy.copy()
    if s:
        K += Dz[slk].T @ Dz[slk]
    if p:
        K += rho * P[actP].T @ P[actP]
    L = chol_floor(K)
    lam = z2.copy() if p else np.zeros(0)
    y = y_ipm
    for _ in range(rounds):
        rhs = -c.copy()
        if s:
            rhs += Dz[slk].T @ g[slk]
        if p:
            rhs += P[actP].T @ (rho * h[actP] - lam[actP])
        y = chol_solve(L, rhs)
        if p:
            lam[actP] += rho * (P[actP] @ y - h[actP])
    tp = 1e-9 * scale
    ok = True
    if p:
        ok &= bool(np.all(P @ y <= h + tp)) and bool(np.all(lam[actP] >= -tp))
    if s:
        r = Dz @ y - g
        ok &= bool(np.all(r[slk] >= -tp)) and bool(np.all(r[~slk] <= tp))
    POLISH_STATS.append(ok)
    return y if ok else y_ipm


POLISH_STATS = []
XO_STATS = []


def crossover(Hy, c, P, h, Dz, g, y_ipm, s1, z1, s2, z2, scale, rounds=int(os.environ.get("XO_ROUNDS", 6))):
    """lmpc_hoqp.hip crossover(): frozen rows with z > s held exactly (Schur complement on the active rows), own
    rows with v > 0 (s1 > z1) as 1/2 (d y - g)^2; the classification repaired for a few rounds (violated frozen rows
    in, negative multipliers out, own rows moved to the side they land on); kept only if it verifies."""
    p, s = P.shape[0], Dz.shape[0]
    fa = (z2 > s2) if p else np.zeros(0, bool)
    ob = (z1 > s1) if s else np.zeros(0, bool)  # called with the row constraint's (s3, z3): violated where z3 > s3
    tol = 1e-9 * scale
    for rd in range(rounds):
        RA = P[fa] if p else np.zeros((0, len(c)))
        na = RA.shape[0]
        K = Hy + (Dz[ob].T @ Dz[ob] if s else 0)
        # augmented-Lagrangian term rho R_A'R_A: the same constrained optimum (R_A y = h_A there), and K stays
        # invertible where only the active rows bind (Hy is singular along ker G)
        rho = float(os.environ.get("XO_RHO", 0.0)) * max(1.0, float(np.max(np.diag(K))))
        K = K + rho * RA.T @ RA
        L = chol_floor(K)
        # a correction from the interior-point iterate: along directions where K is singular to rounding (flat
        # objective) the floored pivots keep the iterate's components, which satisfy the inactive rows
        rhs = -c + (Dz[ob].T @ g[ob] if s else 0) + rho * RA.T @ (h[fa] if p else np.zeros(0))
        y0 = y_ipm + chol_solve(L, rhs - K @ y_ipm)
        y = y0
        lam = np.zeros(0)
        if na:
            T = np.stack([chol_solve(L, RA[a]) for a in range(na)])  # rows K^-1 R_a'
            Sm = RA @ T.T
            e = RA @ y0 - h[fa]
            Ls = chol_floor(Sm)
            lam = chol_solve(Ls, e)
            y = y0 - T.T @ lam
        changed = False
        vmax = 0.0
        if os.environ.get("XO_VERBOSE"):
            tp_ = (P @ y - h) if p else np.zeros(0)
            t_ = (Dz @ y - g) if s else np.zeros(0)
            print(f"    xo rd {rd}: na {na} ob {int(ob.sum()) if s else 0} min lam {lam.min() if na else 0:.2e} "
                  f"frozen-inactive max {np.max(tp_[~fa]) if p and (~fa).any() else 0:.2e} "
                  f"own ob min {np.min(t_[ob]) if s and ob.any() else 0:.2e} own !ob max {np.max(t_[~ob]) if s and (~ob).any() else 0:.2e}"
                  f" |y-yipm| {np.max(np.abs(y - y_ipm)):.2e}")
        if na and np.any(lam < -tol):
            idx = np.nonzero(fa)[0]
            fa[idx[np.argmin(lam)]] = False
            vmax = max(vmax, -lam.min())
            changed = True
        if p:
            tp = P @ y - h
            bad = (~fa) & (tp > tol)
            if np.any(bad):
                k = np.argmax(np.where(bad, tp, -np.inf))
                fa[k] = True
                vmax = max(vmax, tp[k])
                changed = True
        if s:
            t = Dz @ y - g
            flip = (ob & (t < -tol)) | ((~ob) & (t > tol))
            if np.any(flip):
                ob = ob ^ flip
                vmax = max(vmax, np.max(np.abs(t[flip])))
                changed = True
        if not changed:
            # stationarity residual of the level's KKT system at the crossover point (diagnostic)
            lf = np.zeros(p)
            if na:
                lf[fa] = lam
            z3 = np.maximum(0.0, Dz @ y - g) if s else np.zeros(0)
            st = Hy @ y + c + (P.T @ lf if p else 0) + (Dz.T @ z3 if s else 0)
            sres = float(np.max(np.abs(st))) / scale
            if sres > 1e-9:
                XO_STATS.append((False, rd, sres))
                return y_ipm
            XO_STATS.append((True, rd, int(fa.sum()) if p else 0, int(ob.sum()) if s else 0, sres))
            return y
    XO_STATS.append((False, rounds, vmax / scale))
    return y_ipm


def level_ipm(Hy, c, P, h, Dz, g, max_iter=60, tol=float(os.environ.get('TOL', 1e-13)), frac=0.99, stats=None):
    """min 1/2 y'Hy y + c'y + 1/2 v'v  s.t. -v <= 0, P y <= h, Dz y - v <= g.  Returns (y, v, iters)."""
    nd, p, s = Hy.shape[0], P.shape[0], Dz.shape[0]
    m = 2 * s + p
    init = os.environ.get("INIT", "zero")
    y = np.zeros(nd)
    if init == "ls" or (init == "ls0" and p == 0):  # unconstrained minimiser of the level objective (ls0: level 0)
        y = chol_solve(chol_floor(Hy), -c)
    floor = float(os.environ.get("SFLOOR", 1.0))
    v = np.maximum(0.0, (Dz @ y - g) if s else 0.0) + floor if s else np.zeros(0)
    # slacks of the three blocks; start them (and the duals) at least at the floor
    s1 = np.maximum(v, floor)
    s2 = np.maximum(h - P @ y, floor) if p else np.zeros(0)
    s3 = np.maximum(g - Dz @ y + v, floor) if s else np.zeros(0)
    z0 = float(os.environ.get("Z0", 1.0))
    z1, z2, z3 = z0 * np.ones(s), z0 * np.ones(p), z0 * np.ones(s)
    scale = 1.0 + max(np.max(np.abs(c)) if nd else 0.0, np.max(np.abs(h)) if p else 0.0,
                      np.max(np.abs(g)) if s else 0.0)
    # frozen rows the levels above left exactly tight (h ~ 0 after their crossover): the interior point gets a
    # margin of HFLOOR of the scale so its feasible set keeps an interior; the crossover uses the true bound
    h_true = h
    hf = float(os.environ.get("HFLOOR", 0.0))
    if p and hf:
        h = np.maximum(h, hf * scale)
        s2 = np.maximum(h - P @ y, floor)
    it = 0
    for it in range(max_iter):
        # residuals: r_d = H x + c + C'z, r_p = C x + sigma - d
        rdy = Hy @ y + c + (P.T @ z2 if p else 0) + (Dz.T @ z3 if s else 0)
        rdv = v - z1 - z3
        rp1 = -v + s1
        rp2 = P @ y + s2 - h
        rp3 = Dz @ y - v + s3 - g
        sig = np.concatenate([s1, s2, s3])
        zz = np.concatenate([z1, z2, z3])
        mu = sig @ zz / m if m else 0.0
        res = max(np.max(np.abs(rdy)) if nd else 0.0, np.max(np.abs(rdv)) if s else 0.0,
                  np.max(np.abs(np.concatenate([rp1, rp2, rp3]))) if m else 0.0)
        rtol = float(os.environ.get('RTOL', 1e-10))
        if (mu <= tol * scale and res <= rtol * scale) or (mu <= float(os.environ.get('STALL_MU', 1e-16)) * scale and res <= 1e3 * rtol * scale):
            break
        w1, w2, w3 = z1 / s1, z2 / s2, z3 / s3
        wcap = float(os.environ.get("WCAP", 0))
        if wcap:  # bounded weights: rows whose z/s passes the cap are held by a fixed penalty
            cap = wcap * max(1.0, float(np.max(np.diag(Hy))))
            w1, w2, w3 = np.minimum(w1, cap), np.minimum(w2, cap), np.minimum(w3, cap)
        dlt = 1.0 + w1 + w3
        w3h = w3 * (1.0 + w1) / dlt
        K = Hy + (P.T @ (w2[:, None] * P) if p else 0) + (Dz.T @ (w3h[:, None] * Dz) if s else 0)
        L = chol_floor(K)

        def newton(rc1, rc2, rc3):
            # dz = W (C dx) + (z r_p - r_c)/sigma ; (H + C'WC) dx = -r_d - C'(z r_p - r_c)/sigma
            e1 = (z1 * rp1 - rc1) / s1
            e2 = (z2 * rp2 - rc2) / s2
            e3 = (z3 * rp3 - rc3) / s3
            ry = -rdy - (P.T @ e2 if p else 0) - (Dz.T @ e3 if s else 0)
            rv = -rdv + e1 + e3
            rhs = ry + (Dz.T @ (w3 * rv / dlt) if s else 0)
            dy = chol_solve(L, rhs)
            dv = (rv + w3 * (Dz @ dy if s else 0)) / dlt if s else np.zeros(0)
            # C dx per block
            c1, c2, c3 = -dv, (P @ dy if p else np.zeros(0)), (Dz @ dy - dv if s else np.zeros(0))
            ds1, ds2, ds3 = -rp1 - c1, -rp2 - c2, -rp3 - c3
            dz1 = (-rc1 - z1 * ds1) / s1
            dz2 = (-rc2 - z2 * ds2) / s2
            dz3 = (-rc3 - z3 * ds3) / s3
            return dy, dv, (ds1, ds2, ds3), (dz1, dz2, dz3)

        def max_step(vals, dirs):
            a = 1.0
            for x, d in zip(vals, dirs):
                neg = d < 0
                if np.any(neg):
                    a = min(a, float(np.min(-x[neg] / d[neg])))
            return a

        dy, dv, ds, dz = newton(s1 * z1, s2 * z2, s3 * z3)
        a_aff = max_step((s1, s2, s3, z1, z2, z3), ds + dz)
        mu_aff = sum(((sx + a_aff * d1) @ (zx + a_aff * d2)) for sx, d1, zx, d2 in
                     zip((s1, s2, s3), ds, (z1, z2, z3), dz)) / m
        sc = (mu_aff / mu) ** 3 * mu
        dy, dv, ds2_, dz2_ = newton(s1 * z1 + ds[0] * dz[0] - sc, s2 * z2 + ds[1] * dz[1] - sc,
                                    s3 * z3 + ds[2] * dz[2] - sc)
        a = min(1.0, frac * max_step((s1, s2, s3, z1, z2, z3), ds2_ + dz2_))
        y = y + a * dy
        v = v + a * dv
        s1, s2, s3 = s1 + a * ds2_[0], s2 + a * ds2_[1], s3 + a * ds2_[2]
        z1, z2, z3 = z1 + a * dz2_[0], z2 + a * dz2_[1], z3 + a * dz2_[2]
    if stats is not None:
        stats.append(it)
    if os.environ.get("POLISH"):
        y = polish(Hy, c, P, h, Dz, g, y, s2, z2, s3, z3, scale)
    if os.environ.get("EXACT"):
        y = crossover(Hy, c, P, h_true, Dz, g, y, s3, z3, s2, z2, scale)
    if s and os.environ.get("VEXACT"):
        v = np.maximum(0.0, Dz @ y - g)
    if os.environ.get("VERBOSE"):
        print(f"    ipm it {it} mu {mu:.1e} res {res:.1e} scale {scale:.1e}")
        if os.environ.get("VERBOSE") == "2":
            print(f"      |rdy| {np.max(np.abs(rdy)) if nd else 0:.1e} |rdv| {np.max(np.abs(rdv)) if s else 0:.1e} "
                  f"|rp1| {np.max(np.abs(rp1)) if s else 0:.1e} |rp2| {np.max(np.abs(rp2)) if p else 0:.1e} "
                  f"|rp3| {np.max(np.abs(rp3)) if s else 0:.1e} max z2 {np.max(z2) if p else 0:.1e} "
                  f"min s2 {np.min(s2) if p else 0:.1e}")
    return y, v, it


def hoqp_device(tasks, stats=None):
    """tasks: list of oracle Task.  Returns per-level x and w, as the chain of HoQp objects would."""
    n = max(tasks[0].a.shape[1], tasks[0].d.shape[1])
    Z = np.eye(n)
    x = np.zeros(n)
    stk_d = np.zeros((0, n))  # stacked rows, current level first (HoQp.cpp:60)
    stk_f = np.zeros(0)
    stk_w = np.zeros(0)       # stacked slacks, current level last (HoQp.cpp:176-182)
    xs, ws = [], []
    for t in tasks:
        nd = Z.shape[1]
        has_eq = t.a.shape[0] > 0
        d = t.d if t.d.shape[1] else np.zeros((0, n))
        if has_eq:
            G = t.a @ Z
            Hy = G.T @ G + 1e-12 * np.eye(nd)
            c = G.T @ (t.a @ x - t.b)
        else:
            Hy = 1e-12 * np.eye(nd)
            c = np.zeros(nd)
        P = stk_d @ Z
        h = stk_f - stk_d @ x + stk_w
        if P.shape[0]:  # dead frozen rows (lmpc_hoqp.hip): projection zero up to rounding
            zmax = np.max(np.abs(Z))
            dead = np.max(np.abs(P), axis=1) <= 1e-12 * np.max(np.abs(stk_d), axis=1) * zmax
            P = P.copy(); h = h.copy()
            P[dead] = 0.0
            h[dead] = 1.0
        Dz = d @ Z
        g = t.f - d @ x if d.shape[0] else np.zeros(0)
        y, v, _ = level_ipm(Hy, c, P, h, Dz, g, stats=stats)
        x = x + Z @ y
        xs.append(x.copy())
        ws.append(v.copy())
        stk_d = np.vstack([d, stk_d])
        stk_f = np.concatenate([t.f if d.shape[0] else np.zeros(0), stk_f])
        stk_w = np.concatenate([stk_w, v])
        if has_eq:
            Z = Z @ Q.fullpivlu_kernel(t.a @ Z)
    return xs, ws


def random_task(rng, n, ne, ni, tight):
    a = rng.standard_normal((ne, n))
    d = rng.standard_normal((ni, n))
    f = rng.uniform(-0.5, 0.2, ni) if tight else rng.uniform(0.5, 2.0, ni)
    return Q.Task(a, rng.standard_normal(ne), d, f)


def compare(tasks, label, stats):
    t0 = time.time()
    lv = []
    for t in tasks:
        lv.append(Q.HoQp(t, lv[-1] if lv else None))
    t1 = time.time()
    xs, ws = hoqp_device(tasks, stats)
    ex = max(float(np.max(np.abs(xd - h.solution()))) / (1 + float(np.max(np.abs(h.solution()))))
             for xd, h in zip(xs, lv))
    ew = max(float(np.max(np.abs(wd - h.w_sol))) if wd.size else 0.0 for wd, h in zip(ws, lv))
    eax = max(float(np.max(np.abs(t.a @ (xd - h.solution())))) if t.a.shape[0] else 0.0
              for t, xd, h in zip(tasks, xs, lv))
    xf = float(np.max(np.abs(xs[-1] - lv[-1].solution()))) / (1 + float(np.max(np.abs(lv[-1].solution()))))
    if os.environ.get("VERBOSE"):
        for k, (t, xd, wd, h) in enumerate(zip(tasks, xs, ws, lv)):
            print(f"  level {k}: |A dx| {np.max(np.abs(t.a @ (xd - h.solution()))) if t.a.shape[0] else 0:.1e} "
                  f"|dw| {np.max(np.abs(wd - h.w_sol)) if wd.size else 0:.1e} |dx| {np.max(np.abs(xd - h.solution())):.1e}"
                  f" w>0: {int(np.sum(h.w_sol > 1e-9))}")
    return ex, ew, eax, xf, t1 - t0


def main():
    stats = []
    t0, t1 = Q.reference_test_tasks()
    print("reference test:", compare([t0, t1], "ref", stats))
    worst = np.zeros(4)
    for seed in range(12):
        rng = np.random.default_rng(100 + seed)
        n = 8
        tasks = [random_task(rng, n, 2, 3, tight=seed % 2 == 0), random_task(rng, n, 2, 2, tight=False),
                 random_task(rng, n, 3, 2, tight=seed % 3 == 0)]
        try:
            r = compare(tasks, "rand", stats)
        except ValueError:
            continue
        worst = np.maximum(worst, r[:4])
    print("random 3-level: max rel x err (per level, final) / w / A dx:", worst)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from legged_mpc_control_amd import wbc as W  # noqa: E402
    worst = np.zeros(4)
    tt = 0.0
    for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
        tasks = W.synth_wbc_tasks(seed)
        r = compare(tasks, "wbc", stats)
        worst = np.maximum(worst, r[:4])
        tt += r[4]
    print("wbc-shaped: max rel x err (levels, final) / w / A dx:", worst, f"oracle {tt:.1f}s")
    print("IPM iterations per level: mean %.1f max %d" % (np.mean(stats), np.max(stats)))


if __name__ == "__main__":
    main()

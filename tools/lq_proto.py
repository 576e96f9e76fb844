#!/usr/bin/env python3
"""Dev tool (CPU): numpy replica of the LDS-resident Riccati kernel (csrc/lmpc_lq.hip, round 4), step for step,
checked against the exact oracle before any of it runs on the GPU.

What it pins down (the formulas the kernel implements):
  factorisation (backward, stage k = H-1 .. 0), with the affine column 12 of the value function carried along
  (augmented state [x; 1]):
      C = P B^ (B^ rows 6-11: Bt | dv)      -> v = P d
      Guu = Bt' P22 Bt (+ Rr added at each 3x3 leg pivot: Rr is block diagonal)
      X = L^-1 [0 | Bt' | rr]               -> V = L^-1 Bt',  rho' = L^-1 rr
      KH = X'X                              -> K = V'V,  rho = V' rho' = Bt Guu^-1 rr
      S = V' L^-1 = Bt Guu^-1               (the corrector's rho = S rr')
      PA = P A^ (A^ = [A d; 0 1]) -> Z = rows 6-11 of PA (6 x 13: Z x + za, za = v2 + p2)
      P_k = Q^ + A^'PA - M'KH M' (M' = PA with row 12 = e12): its column 12 is p_k (the fused backward pass)
  forward  w = Z x + za ;  x' = A x + d - [0; K w + rho]
  inputs   from the costate, per leg: lambda2 = Z A^-1 x' + za - v2 (= P2 x' + p2),  u = -Rr^-1 (rr + Bt' lambda2)
  corrector backward (same matrix, new rr'):  rho = S rr' ;  y = p + v ; za = y[6:12] ;
           p_k = q_k + A'y - Z'(K za + rho)
The interior point and the polish are the kernels' (Mehrotra, split step lengths, hand-over at tol_mu with faces
active where z > 1e-3 s, per-leg null-space polish verified by an adjoint gradient).

  tools/lq_proto.py [config] [count]      -> max |u - oracle| / max(1, |oracle|), iterations
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

ACT_RATIO = 1e-3
STEP_FRAC = 0.99
# RED6=1: the reduced-input form of every Newton system -- the stage's inputs enter the dynamics only through
# f = Bt u (6 rows), so min_u {1/2 u'Rr u + rr'u : Bt u = f} = 1/2 |v|^2 + const with f = U v - g, W = Bt Rr^-1 Bt' =
# U U', g = Bt Rr^-1 rr: a Riccati step with 6 inputs of unit cost (two 3x3 pivots whatever the leg count), d' = d - E g
# and no linear input term; the corrector's new rr enters as rho = dg - K P22 dg (dg = g'' - g').
RED6 = os.environ.get("RED6", "0") == "1"
PSD_FLOOR = 1e-10
RED6_POLISH = os.environ.get("RED6_POLISH", "0") == "1"  # the polish too (loses digits on ill-conditioned W)


def skew(r):
    return np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])


def terrain_frame(n):
    n = np.asarray(n, float) / np.linalg.norm(n)
    nx, ny, c = n
    h = 1.0 / (1.0 + c)
    return np.array([[1 - nx * nx * h, -nx * ny * h, nx], [-nx * ny * h, 1 - ny * ny * h, ny], [-nx, -ny, c]])


def model(p, H, rec, con, normals=None):
    dt, m = p.dt, p.robot_mass
    x0 = rec[:12].copy()
    R = rec[12:21].reshape(3, 3)
    feet = rec[21:33].reshape(4, 3)
    xr = rec[33:].reshape(H, 12)
    Ib = np.array(p.trunk_inertia).reshape(3, 3)
    iw = np.linalg.inv(R @ Ib @ R.T)
    G0 = np.zeros((6, 12))
    Rf = [np.eye(3) if normals is None else terrain_frame(normals[j]) for j in range(4)]
    rw = np.array(p.r_weights)
    Rb = []
    for j in range(4):
        blk = np.vstack([dt * iw @ skew(feet[j]), dt / m * np.eye(3)])
        G0[:, 3 * j:3 * j + 3] = blk @ Rf[j]
        Rb.append(Rf[j].T @ np.diag(rw[3 * j:3 * j + 3]) @ Rf[j])
    A = []
    for k in range(H):
        c, s = np.cos(xr[k, 2]), np.sin(xr[k, 2])
        a = np.eye(12)
        a[0:3, 6:9] += dt * np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])
        a[3:6, 9:12] += dt * np.eye(3)
        A.append(a)
    return dict(H=H, dt=dt, g=p.gravity, mu=p.mu, fmax=p.f_max, mass=m, Q=np.array(p.q_weights), x0=x0, xr=xr,
                G0=G0, A=A, Rb=Rb, Rf=Rf, con=con.reshape(H, 4).astype(bool))


# ---------------------------------------------------------------------------------------------------------
def chol_psd(W):
    """Lower Cholesky factor of a PSD 6x6 with rounding-level pivots (rank-deficient W) floored to zero columns."""
    n = W.shape[0]
    L = np.zeros_like(W)
    for i in range(n):
        d = W[i, i] - L[i, :i] @ L[i, :i]
        if not (d > PSD_FLOOR * W[i, i]) or W[i, i] <= 0.0:
            continue
        L[i, i] = np.sqrt(d)
        for r in range(i + 1, n):
            L[r, i] = (W[r, i] - L[r, :i] @ L[i, :i]) / L[i, i]
    return L


def reduce6(Rr, Bt, rr):
    """Per stage: U (6x6, W = U U'), g = Bt Rr^-1 rr."""
    U, g = [], []
    for k in range(len(Bt)):
        W = np.zeros((6, 6))
        gk = np.zeros(6)
        for j in range(4):
            Bj = Bt[k][:, 3 * j:3 * j + 3]
            Ri = np.linalg.inv(Rr[k][j])
            W += Bj @ Ri @ Bj.T
            gk += Bj @ (Ri @ rr[k][3 * j:3 * j + 3])
        U.append(chol_psd(W))
        g.append(gk)
    return U, g


def p22_of(M, st, k):
    """P_{k+1}[6:12, 6:12] from Z_k = rows 6-11 of P_{k+1} A_k (A_k's columns 0-5 are unit columns)."""
    Z = st[k]["Z"][:, :12]
    dN = M["A"][k][0:6, 6:12]
    return Z[:, 6:12] - Z[:, 0:6] @ dN


def factor6(M, Rr, Bt, rr, dv):
    """The reduced-input factorisation: factor() on (I, [U | 0], 0, dv - g); returns (stages, g, dv')."""
    U, g = reduce6(Rr, Bt, rr)
    H = M["H"]
    I4 = [[np.eye(3)] * 4 for _ in range(H)]
    Bp = [np.hstack([U[k], np.zeros((6, 6))]) for k in range(H)]
    dvp = [dv[k] - g[k] for k in range(H)]
    st = factor(M, I4, Bp, [np.zeros(12)] * H, dvp, want_S=False)
    return st, g, dvp


def factor(M, Rr, Bt, rr, dv, want_S=True):
    """Rr[k][j] 3x3, Bt[k] 6x12, rr[k] 12, dv[k] 6 -> per-stage (Z 6x13, K, rho, S, v)."""
    H, Q = M["H"], M["Q"]
    Ph = np.zeros((13, 13))
    Ph[:12, :12] = np.diag(Q)
    Ph[:12, 12] = -Q * M["xr"][H - 1]
    out = [None] * H
    for k in range(H - 1, -1, -1):
        P, p = Ph[:12, :12], Ph[:12, 12]
        d = np.concatenate([np.zeros(6), dv[k]])
        v = P @ d
        Guu = Bt[k].T @ P[6:, 6:] @ Bt[k]
        for j in range(4):
            Guu[3 * j:3 * j + 3, 3 * j:3 * j + 3] += Rr[k][j]
        L = np.linalg.cholesky(Guu)
        Li = np.linalg.inv(L)
        V = Li @ Bt[k].T
        rho1 = Li @ rr[k]
        K = V.T @ V
        rho = V.T @ rho1
        S = V.T @ Li if want_S else None
        A = M["A"][k]
        Ahat = np.eye(13)
        Ahat[:12, :12] = A
        Ahat[:12, 12] = d
        PA = Ph @ Ahat
        Z = PA[6:12, :].copy()  # 6 x 13, column 12 = v2 + p2
        out[k] = dict(Z=Z, K=K, rho=rho, S=S, v=v)
        if k > 0:
            Mp = PA.copy()
            Mp[12, :] = 0.0
            Mp[12, 12] = 1.0
            KH = np.zeros((13, 13))
            KH[6:12, 6:12] = K
            KH[6:12, 12] = rho
            KH[12, 6:12] = rho
            KH[12, 12] = rho1 @ rho1
            Qh = np.zeros((13, 13))
            Qh[:12, :12] = np.diag(Q)
            Qh[:12, 12] = -Q * M["xr"][k - 1]
            Pn = Qh + Ahat.T @ PA - Mp.T @ KH @ Mp
            Pn[12, :12] = Pn[:12, 12]  # symmetric (the kernel never reads row 12)
            Ph = Pn
    return out


def backward_corr(M, st, rho_new):
    """Corrector: same factorisation, new rho (= S rr') -> new za in st[k]['Z'][:, 12]."""
    H, Q = M["H"], M["Q"]
    p = -Q * M["xr"][H - 1]
    for k in range(H - 1, -1, -1):
        s = st[k]
        y = p + s["v"]
        za = y[6:]
        s["Z"][:, 12] = za
        s["rho"] = rho_new[k]
        if k > 0:
            t = s["K"] @ za + s["rho"]
            p = -Q * M["xr"][k - 1] + M["A"][k].T @ y - s["Z"][:, :12].T @ t


def forward(M, st, dv):
    x = M["x0"].copy()
    xs = []
    for k in range(M["H"]):
        s = st[k]
        w = s["Z"][:, :12] @ x + s["Z"][:, 12]
        xn = M["A"][k] @ x
        xn[6:] += dv[k] - (s["K"] @ w + s["rho"])
        xs.append(xn)
        x = xn
    return xs


def costate_u(M, st, xs, Rr, rr, Bt):
    """u per (k, j): -Rr^-1 (rr + Bt_j' lambda2), lambda2 = Z A^-1 x' + za - v2."""
    H = M["H"]
    u = np.zeros((H, 4, 3))
    for k in range(H):
        s = st[k]
        Ainv = np.linalg.inv(M["A"][k])
        lam2 = s["Z"][:, :12] @ (Ainv @ xs[k]) + s["Z"][:, 12] - s["v"][6:]
        for j in range(4):
            b = rr[k][3 * j:3 * j + 3] + Bt[k][:, 3 * j:3 * j + 3].T @ lam2
            u[k, j] = -np.linalg.solve(Rr[k][j], b)
    return u


def adjoint_lam2(M, xs):
    """lambda_{k+1}[6:12] for every k from the trajectory (the polish verification's independent gradient)."""
    H, Q = M["H"], M["Q"]
    lam = Q * (xs[H - 1] - M["xr"][H - 1])
    out = [None] * H
    out[H - 1] = lam[6:].copy()
    for k in range(H - 1, 0, -1):
        lam = Q * (xs[k - 1] - M["xr"][k - 1]) + M["A"][k].T @ lam
        out[k - 1] = lam[6:].copy()
    return out


# ---- leg-step helpers (lmpc_kernel_common.h) ----
def cons_rows(mu):
    return np.array([[-1, 0, -mu], [1, 0, -mu], [0, -1, -mu], [0, 1, -mu], [0, 0, 1.0]])


def leg_basis(act, mu, fmax):
    """f = up + T y (T columns orthonormal); apex (f = 0) when a pair of opposite faces is active."""
    if (act & 3) == 3 or (act & 12) == 12:
        return np.zeros((3, 3)), np.zeros(3), True
    C = cons_rows(mu)
    b = np.array([0, 0, 0, 0, fmax])
    rows = [i for i in range(5) if (act >> i) & 1][:3]
    if not rows:
        return np.eye(3), np.zeros(3), False
    Cs = C[rows]
    up = np.linalg.lstsq(Cs, b[rows], rcond=None)[0]
    U, sv, Vt = np.linalg.svd(Cs)
    T = np.zeros((3, 3))
    ns = Vt[len(rows):].T  # null space
    T[:, :ns.shape[1]] = ns
    return T, up, False


def solve(M, tol_mu=1e-4, max_iter=40, max_rounds=8, max_attempts=3):
    H, mu, fmax, G0 = M["H"], M["mu"], M["fmax"], M["G0"]
    con = M["con"]
    C = cons_rows(mu)
    bvec = np.array([0, 0, 0, 0, fmax])
    nst = con.sum()
    f = np.zeros((H, 4, 3))
    s = np.ones((H, 4, 5))
    z = np.ones((H, 4, 5))
    for k in range(H):
        cnt = max(con[k].sum(), 1)
        for j in range(4):
            if con[k, j]:
                f[k, j, 2] = min(0.5 * fmax, M["mass"] * M["g"] / cnt)
                s[k, j] = bvec - C @ f[k, j]
                z[k, j] = 1.0 / s[k, j]
    mc = 5.0 * nst
    tol, it_end, ipm_it, rounds, att = tol_mu, max_iter, 0, 0, 0
    gdt = np.zeros(6)
    gdt[5] = -M["g"] * M["dt"]
    mode = "pred"
    act = np.zeros((H, 4), int)
    Bt_ipm = [G0 * np.repeat(con[k], 3)[None, :] for k in range(H)]
    dv_ipm = [gdt.copy() for _ in range(H)]
    u = np.zeros((H, 4, 3))
    while True:
        if mode == "pred":
            muc = np.sum(s[con] * z[con]) / mc
            if muc < tol or ipm_it >= it_end:
                for k in range(H):
                    for j in range(4):
                        a = 0
                        if con[k, j]:
                            for i in range(5):
                                if z[k, j, i] > ACT_RATIO * s[k, j, i]:
                                    a |= 1 << i
                            if np.max(np.abs(f[k, j])) < 1e-6 * fmax:
                                a = 15
                        act[k, j] = a
                mode = "polish"
                rd = 0
                continue
            W = z / s
            Rr = [[(M["Rb"][j] + C.T @ np.diag(W[k, j]) @ C) if con[k, j] else np.eye(3) for j in range(4)]
                  for k in range(H)]
            rr = [np.concatenate([C.T @ (W[k, j] * (s[k, j] - bvec)) if con[k, j] else np.zeros(3)
                                  for j in range(4)]) for k in range(H)]
            if RED6:
                st, g1, dvp = factor6(M, Rr, Bt_ipm, rr, dv_ipm)
                xs = forward(M, st, dvp)
            else:
                st = factor(M, Rr, Bt_ipm, rr, dv_ipm)
                xs = forward(M, st, dv_ipm)
            ua = costate_u(M, st, xs, Rr, rr, Bt_ipm)
            # predictor step
            dsa = np.zeros_like(s)
            dza = np.zeros_like(z)
            amax = 1.0
            for k in range(H):
                for j in range(4):
                    if not con[k, j]:
                        continue
                    o = C @ ua[k, j] - bvec
                    dsa[k, j] = -o - s[k, j]
                    dza[k, j] = -z[k, j] - z[k, j] / s[k, j] * dsa[k, j]
                    for i in range(5):
                        if dsa[k, j, i] < 0:
                            amax = min(amax, -s[k, j, i] / dsa[k, j, i])
                        if dza[k, j, i] < 0:
                            amax = min(amax, -z[k, j, i] / dza[k, j, i])
            ratio = np.sum(((s + amax * dsa) * (z + amax * dza))[con]) / np.sum((s * z)[con])
            smu = ratio ** 3 * muc
            rr2 = [np.concatenate([C.T @ ((z[k, j] * (s[k, j] - bvec) + smu - dsa[k, j] * dza[k, j]) / s[k, j])
                                   if con[k, j] else np.zeros(3) for j in range(4)]) for k in range(H)]
            if RED6:
                _, g2 = reduce6(Rr, Bt_ipm, rr2)
                rho_new = []
                for k in range(H):
                    dg = g2[k] - g1[k]
                    rho_new.append(dg - st[k]["K"] @ (p22_of(M, st, k) @ dg))
                backward_corr(M, st, rho_new)
                xs = forward(M, st, dvp)
            else:
                rho_new = [st[k]["S"] @ rr2[k] for k in range(H)]
                backward_corr(M, st, rho_new)
                xs = forward(M, st, dv_ipm)
            uc = costate_u(M, st, xs, Rr, rr2, Bt_ipm)
            ds = np.zeros_like(s)
            dz = np.zeros_like(z)
            amax = dmax = 1.0
            for k in range(H):
                for j in range(4):
                    if not con[k, j]:
                        continue
                    o = C @ uc[k, j] - bvec
                    ds[k, j] = -o - s[k, j]
                    dz[k, j] = (smu - z[k, j] * s[k, j] - dsa[k, j] * dza[k, j] - z[k, j] * ds[k, j]) / s[k, j]
                    for i in range(5):
                        if ds[k, j, i] < 0:
                            amax = min(amax, -s[k, j, i] / ds[k, j, i])
                        if dz[k, j, i] < 0:
                            dmax = min(dmax, -z[k, j, i] / dz[k, j, i])
            al = min(1.0, STEP_FRAC * amax)
            ad = min(1.0, STEP_FRAC * dmax)
            f[con] += al * (uc[con] - f[con])
            s[con] += al * ds[con]
            z[con] += ad * dz[con]
            ipm_it += 1
            continue
        # ---- polish ----
        rounds += 1
        Tm = np.zeros((H, 4, 3, 3))
        upm = np.zeros((H, 4, 3))
        apex = np.zeros((H, 4), bool)
        for k in range(H):
            for j in range(4):
                if con[k, j]:
                    Tm[k, j], upm[k, j], apex[k, j] = leg_basis(act[k, j], mu, fmax)
        Rr, rr, Bt, dv = [], [], [], []
        for k in range(H):
            Rk, rk = [], []
            B = np.zeros((6, 12))
            d = gdt.copy()
            for j in range(4):
                T, up = Tm[k, j], upm[k, j]
                R3 = T.T @ M["Rb"][j] @ T
                fixed = np.all(T == 0, axis=0)
                for a in range(3):
                    if fixed[a]:
                        R3[a, :] = 0
                        R3[:, a] = 0
                        R3[a, a] = 1
                Rk.append(R3)
                rk.append(T.T @ (M["Rb"][j] @ up))
                B[:, 3 * j:3 * j + 3] = G0[:, 3 * j:3 * j + 3] @ T
                d += G0[:, 3 * j:3 * j + 3] @ up
            Rr.append(Rk)
            rr.append(np.concatenate(rk))
            Bt.append(B)
            dv.append(d)
        if RED6 and RED6_POLISH:
            st, _, dvp = factor6(M, Rr, Bt, rr, dv)
            xs = forward(M, st, dvp)
        else:
            st = factor(M, Rr, Bt, rr, dv, want_S=False)
            xs = forward(M, st, dv)
        y = costate_u(M, st, xs, Rr, rr, Bt)
        for k in range(H):
            for j in range(4):
                u[k, j] = upm[k, j] + Tm[k, j] @ y[k, j] if con[k, j] else 0.0
        lam2 = adjoint_lam2(M, xs)
        gscale = 1.0
        g = np.zeros((H, 4, 3))
        for k in range(H):
            for j in range(4):
                g[k, j] = M["Rb"][j] @ u[k, j] + G0[:, 3 * j:3 * j + 3].T @ lam2[k]
                gscale = max(gscale, np.max(np.abs(g[k, j])))
        changed = False
        for k in range(H):
            for j in range(4):
                if not con[k, j]:
                    continue
                o = C @ u[k, j] - bvec
                viol = [(o[i], i) for i in range(5) if not (act[k, j] >> i) & 1 and o[i] > 1e-9 * fmax]
                if viol:
                    act[k, j] |= 1 << max(viol)[1]
                    changed = True
                    continue
                if apex[k, j]:
                    gg = g[k, j]
                    if gg[2] / mu < abs(gg[0]) + abs(gg[1]) - 1e-9 * gscale:
                        act[k, j] = (2 if gg[0] < 0 else 1) | (8 if gg[1] < 0 else 4)
                        changed = True
                    continue
                rows = [i for i in range(5) if (act[k, j] >> i) & 1]
                if rows:
                    zz = np.linalg.lstsq(C[rows].T, -g[k, j], rcond=None)[0]
                    i = int(np.argmin(zz))
                    if zz[i] < -1e-9 * gscale:
                        act[k, j] &= ~(1 << rows[i])
                        changed = True
        if not changed:
            return u, ipm_it, rounds, True
        rd += 1
        if rd >= max_rounds:
            att += 1
            if att >= max_attempts:
                return f, ipm_it, rounds, False
            tol = min(tol * 1e-3, 1e-8 * 1e-4 ** (att - 1))
            it_end += max_iter
            mode = "pred"


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    p, H, rec, con = synth.config_batch(cid, count=cnt)
    nrm = None
    if cid == 4:
        nrm = np.zeros((cnt, 4, 3))
        lib_n = synth.normals(cnt, synth.BASE_SEED + 4) if hasattr(synth, "normals") else None
        nrm = None if lib_n is None else lib_n.reshape(cnt, 4, 3)
    op = O.params_from(p)
    worst, its, rds, bad = 0.0, [], [], 0
    for b in range(cnt):
        M = model(p, H, rec[b], con[b], None if nrm is None else nrm[b])
        u, it, rd, ok = solve(M)
        ref, _, _ = O.solve(op, H, rec[b], con[b], normals=None if nrm is None else nrm[b])
        ref = np.asarray(ref).reshape(H, 4, 3)
        if nrm is not None:  # the prototype works in contact-frame forces
            u = np.einsum("jab,kjb->kja", np.array(M["Rf"]), u)
        err = float(np.max(np.abs(u - ref) / np.maximum(1.0, np.abs(ref))))
        worst = max(worst, err)
        its.append(it)
        rds.append(rd)
        bad += not ok
    print(f"config {cid} H={H}: {cnt} QPs, max rel err {worst:.2e}, ipm {np.mean(its):.2f} (max {max(its)}), "
          f"rounds {np.mean(rds):.2f} (max {max(rds)}), unverified {bad}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Dev tool (CPU): numpy replica of the dense path's active-set polish (lmpc_dense.hip: per stance leg-step an
active-face bitmask, the leg's null-space basis T / particular solution up, T'HT y = -T'(H up + g), then one face
added (most violated) or dropped (most negative multiplier) per leg-step per round), driven from different
starting guesses, to price strategies for the B = 1024 tail before touching the kernel:
  ipm:K   -- K Mehrotra iterations (or to tol_mu) then the polish from z > s (the kernel's rule);
  gi:K    -- K dual active-set steps then the polish from the GI working set;
  a third field picks the polish update: single (the kernel's, default) or pdas (primal-dual active set).
Cost model in cycles per QP from the v15 stamps: IPM iteration 55 k, polish round 45 k,
GI step 10.5 k, GI start (Cholesky + J) 45 k, prologue + condensation 55 k."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_proto import leg_cons, reduced_qp  # noqa: E402
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

# polish face rows as the kernel numbers them (cons_resid: o = C f - b <= 0)
CR = lambda mu: np.array([[-1, 0, -mu], [1, 0, -mu], [0, -1, -mu], [0, 1, -mu], [0, 0, 1.0]])


def leg_basis(act, mu, fmax):
    """T (3x3, orthonormal null-space columns, zero-padded), up, apex (lmpc_kernel_common.h leg_basis)."""
    T = np.zeros((3, 3))
    up = np.zeros(3)
    if (act & 3) == 3 or (act & 12) == 12:
        return T, up, True
    rows = [i for i in range(5) if (act >> i) & 1][:3]
    C = CR(mu)
    b = np.array([0, 0, 0, 0, fmax])
    if not rows:
        return np.eye(3), up, False
    A = C[rows]
    up = np.linalg.lstsq(A, b[rows], rcond=None)[0]
    _, _, Vt = np.linalg.svd(A)
    r = np.linalg.matrix_rank(A)
    N = Vt[r:].T
    T[:, :N.shape[1]] = N
    return T, up, False


def drop_face(act, g, mu, zmin):
    rows = [i for i in range(5) if (act >> i) & 1][:3]
    C = CR(mu)[rows]
    z = np.linalg.lstsq(C.T, -g, rcond=None)[0]
    k = int(np.argmin(z))
    return rows[k] if z[k] < zmin else -1


def polish(Hm, g, act, mu, fmax, max_rounds=12, tol_p=1e-9, tol_d=1e-9, rule="single"):
    nls = len(act)
    act = list(act)
    for rd in range(1, max_rounds + 1):
        Ts, ups, apex = [], [], []
        for b in range(nls):
            T, up, ap = leg_basis(act[b], mu, fmax)
            Ts.append(T); ups.append(up); apex.append(ap)
        Tb = np.zeros((3 * nls, 3 * nls))
        upv = np.zeros(3 * nls)
        for b in range(nls):
            Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3] = Ts[b]
            upv[3 * b:3 * b + 3] = ups[b]
        M = Tb.T @ Hm @ Tb
        fixed = np.where(np.abs(Tb).sum(0) == 0)[0]
        M[fixed, fixed] += 1.0
        y = np.linalg.solve(M, -Tb.T @ (Hm @ upv + g))
        u = upv + Tb @ y
        grad = Hm @ u + g
        gscale = max(1.0, np.max(np.abs(grad)))
        C = CR(mu)
        bb = np.array([0, 0, 0, 0, fmax])
        changed = False
        for b in range(nls):
            o = C @ u[3 * b:3 * b + 3] - bb
            gl = grad[3 * b:3 * b + 3]
            if rule == "pdas" and not apex[b]:
                # primal-dual active set: every violated face in, every face with a negative multiplier out
                rows = [i for i in range(5) if (act[b] >> i) & 1][:3]
                lam = np.zeros(5)
                if rows:
                    lam[rows] = np.linalg.lstsq(C[rows].T, -gl, rcond=None)[0]
                score = np.where([(act[b] >> i) & 1 for i in range(5)], lam, -(-o))  # active: lambda; inactive: violation
                new = 0
                order = np.argsort(-score)
                for i in order:
                    isact = (act[b] >> i) & 1
                    keep = (isact and lam[i] >= -tol_d * gscale) or (not isact and o[i] > tol_p * fmax)
                    if keep and bin(new).count("1") < 3:
                        cand = new | (1 << int(i))
                        if np.linalg.matrix_rank(C[[k for k in range(5) if (cand >> k) & 1]]) == bin(cand).count("1") \
                                or (cand & 3) == 3 or (cand & 12) == 12:
                            new = cand
                if new != act[b]:
                    act[b] = new
                    changed = True
                continue
            cand = [(o[i], i) for i in range(5) if not (act[b] >> i) & 1 and o[i] > tol_p * fmax]
            if cand and rule == "multi":
                # every violated face in, most violated first, while the active rows stay independent (an
                # opposite pair is the lift-off apex)
                new = act[b]
                for _, i in sorted(cand, reverse=True):
                    c2 = new | (1 << i)
                    rows = [k for k in range(5) if (c2 >> k) & 1]
                    if (c2 & 3) == 3 or (c2 & 12) == 12 or (len(rows) <= 3 and np.linalg.matrix_rank(C[rows]) == len(rows)):
                        new = c2
                act[b] = new
                changed = True
            elif cand:
                act[b] |= 1 << max(cand)[1]
                changed = True
            elif apex[b]:
                if gl[2] / mu < abs(gl[0]) + abs(gl[1]) - tol_d * gscale:
                    act[b] = (2 if gl[0] < 0 else 1) | (8 if gl[1] < 0 else 4)
                    changed = True
            elif act[b]:
                df = drop_face(act[b], gl, mu, -tol_d * gscale)
                if df >= 0:
                    act[b] &= ~(1 << df)
                    changed = True
        if not changed:
            return u, rd, True
    return u, max_rounds, False


def ipm_sz(Hm, g, st, p, tol, max_iter, frac=0.99):
    """tools/ipm_proto.py's Mehrotra loop, returning the final (f, s, z, iterations)."""
    nls = len(st)
    mu_f, fmax = p.mu, p.f_max
    Cl = CR(mu_f)
    bl = np.array([0, 0, 0, 0, fmax])
    n = 3 * nls
    C = np.zeros((5 * nls, n))
    for b in range(nls):
        C[5 * b:5 * b + 5, 3 * b:3 * b + 3] = Cl
    bvec = np.tile(bl, nls)
    cnt = {}
    for (k, j) in st:
        cnt[k] = cnt.get(k, 0) + 1
    f = np.zeros(n)
    for b, (k, j) in enumerate(st):
        f[3 * b + 2] = min(0.5 * fmax, p.robot_mass * 9.8 / cnt[k])
    s = -(C @ f - bvec)
    z = 1.0 / s
    m = 5 * nls
    it = 0
    while True:
        mu = s @ z / m
        if mu < tol or it >= max_iter:
            return f, s, z, it
        W = z / s
        Kinv = np.linalg.inv(Hm + C.T @ (W[:, None] * C))
        u = Kinv @ -(g + C.T @ (W * (s - bvec)))
        dsa = -(C @ u - bvec) - s
        dza = -z - W * dsa
        amax = 1.0
        for v, d in ((s, dsa), (z, dza)):
            neg = d < 0
            if neg.any():
                amax = min(amax, np.min(-v[neg] / d[neg]))
        mu_aff = (s + amax * dsa) @ (z + amax * dza) / m
        smu = (mu_aff / mu) ** 3 * mu
        wv = (z * (s - bvec) + smu - dsa * dza) / s
        u = Kinv @ -(g + C.T @ wv)
        ds = -(C @ u - bvec) - s
        dz = (smu - z * s - dsa * dza - z * ds) / s
        a = 1.0
        for v, d in ((s, ds), (z, dz)):
            neg = d < 0
            if neg.any():
                a = min(a, np.min(-v[neg] / d[neg]))
        a = min(1.0, frac * a)
        f = f + a * (u - f)
        s = s + a * ds
        z = z + a * dz
        it += 1


def ipm_then_act(Hm, g, st, p, K, tol=1e-8):
    """Mehrotra for at most K iterations (or to tol_mu); the kernel's active-set guess: z > s, lift-off -> apex."""
    nls = len(st)
    f, s, z, it = ipm_sz(Hm, g, st, p, tol, K)
    act = []
    for b in range(nls):
        a = 0
        for i in range(5):
            if z[5 * b + i] > s[5 * b + i]:
                a |= 1 << i
        if np.max(np.abs(f[3 * b:3 * b + 3])) < 1e-6 * p.f_max:
            a = 15
        act.append(a)
    return act, it


def gi_then_act(Hm, g, nls, p, K):
    """At most K dual active-set steps (tools/gi_proto.py); its working set as the polish guess (constraint
    5b + f of the GI = face f of leg-step b in the kernel's numbering; a pair of opposite faces = the apex)."""
    from gi_proto import gi
    stats = dict(adds=0, drops=0)
    gi(Hm, g, nls, p.mu, p.f_max, stats, max_steps=K)
    act = [0] * nls
    for c in stats["active"]:
        b, f = divmod(c, 5)
        act[b] |= 1 << f
    return act, stats["iters"]


def main():
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    strategies = sys.argv[2:] or ["ipm:40", "ipm:6", "ipm:5", "ipm:4"]
    p, H, rec, con = synth.config_batch(2, count=cnt)
    op = O.params_from(p)
    data = []
    for b in range(cnt):
        Hm, g, st, idx = reduced_qp(op, H, rec[b], con[b])
        ref, _, _ = O.solve(op, H, rec[b], con[b])
        data.append((Hm, g, st, idx, ref))
    for spec in strategies:
        parts = spec.split(":")
        kind, K = parts[0], int(parts[1])
        rule = parts[2] if len(parts) > 2 else "single"
        costs, rounds, fails, err = [], [], 0, 0.0
        for Hm, g, st, idx, ref in data:
            if kind == "ipm":
                act, it = ipm_then_act(Hm, g, st, p, K)
                cost = 55e3 + it * 55e3
            else:
                act, it = gi_then_act(Hm, g, len(st), p, K)
                cost = 55e3 + 45e3 + it * 10.5e3
            u, rd, ok = polish(Hm, g, act, p.mu, p.f_max, rule=rule)
            fails += not ok
            cost += rd * 45e3
            costs.append(cost)
            rounds.append(rd)
            mine = np.zeros(12 * H)
            mine[idx] = u
            err = max(err, float(np.max(np.abs(mine - ref.reshape(-1)) / np.maximum(1, np.abs(ref.reshape(-1))))))
        costs = np.array(costs)
        print(f"{spec:8s} polish rounds mean {np.mean(rounds):.2f} max {np.max(rounds)} fails {fails} | model cycles "
              f"mean {costs.mean() / 1e3:.0f}k p99 {np.percentile(costs, 99) / 1e3:.0f}k max {costs.max() / 1e3:.0f}k "
              f"| max err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()

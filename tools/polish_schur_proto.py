#!/usr/bin/env python3
"""Dev tool (CPU): the dense path's polish rounds after the first priced as range-space (Schur complement) updates of
the last factorisation instead of refactorisations, in the numpy replica (tools/hybrid_proto.py polish, rule
"single"; tools/ipm_step_proto.py interior point, hand-over at complementarity 1e-4).

A round whose active faces contain every face of the factorised round's set (faces only added; a leg-step may also
turn apex, u = 0, when none of its base faces is the f_max face) is the factorised QP with k more equality rows on
the base coordinates y: c'(up + T y) = b -> (c'T) y = b - c'up.  Its solution is
    y = y0 - M^-1 A' (A M^-1 A')^-1 (A y0 - d),   M = T'HT (the factorised reduced Hessian),
k + 1 solves with the factorisation plus a k x k Cholesky.  Any other round refactorises.
Prints the per-round transition mix, a check that the update reproduces the direct solve, and the modelled
cycles per QP (IPM iteration 42 k, full polish round 45 k, update round `schur_k` k + per-constraint solves).
    python tools/polish_schur_proto.py [count] [schur_base_k] [schur_per_row_k]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gi_proto import reduced_qp  # noqa: E402
from hybrid_proto import CR, drop_face, leg_basis  # noqa: E402
from ipm_step_proto import ipm  # noqa: E402
from polish_guess_proto import guess  # noqa: E402
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def bases(act, mu, fmax):
    nls = len(act)
    Tb = np.zeros((3 * nls, 3 * nls))
    upv = np.zeros(3 * nls)
    apex = []
    for b in range(nls):
        T, up, ap = leg_basis(act[b], mu, fmax)
        Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3] = T
        upv[3 * b:3 * b + 3] = up
        apex.append(ap)
    return Tb, upv, apex


def direct(Hm, g, act, mu, fmax):
    Tb, upv, apex = bases(act, mu, fmax)
    M = Tb.T @ Hm @ Tb
    fixed = np.where(np.abs(Tb).sum(0) == 0)[0]
    M[fixed, fixed] += 1.0
    y = np.linalg.solve(M, -Tb.T @ (Hm @ upv + g))
    return upv + Tb @ y, apex


def schur_rows(base, new, mu, fmax):
    """Equality rows (a, d) on the base coordinates u = up_b + T_b y that turn the base set into `new`, or None."""
    C = CR(mu)
    bb = np.array([0, 0, 0, 0, fmax])
    rows = []
    for b, (a0, a1) in enumerate(zip(base, new)):
        T, up, ap0 = leg_basis(a0, mu, fmax)
        _, _, ap1 = leg_basis(a1, mu, fmax)
        if a0 == a1:
            continue
        if ap0:
            return None  # apex base: nothing to add, any change is a drop
        if ap1:
            if a0 & 16:
                return None
            # u_b = 0: T y = -up on the free directions
            for j in range(3):
                if np.abs(T[:, j]).sum() > 0:
                    rows.append((b, T[:, j].copy(), 0.0, up))
            continue
        if a1 & a0 != a0:
            return None  # a base face dropped
        for i in range(5):
            if (a1 >> i) & 1 and not (a0 >> i) & 1:
                rows.append((b, C[i], bb[i], up))
    return rows


def schur_solve(Hm, g, base, rows, mu, fmax):
    Tb, upv, _ = bases(base, mu, fmax)
    M = Tb.T @ Hm @ Tb
    fixed = np.where(np.abs(Tb).sum(0) == 0)[0]
    M[fixed, fixed] += 1.0
    rhs = -Tb.T @ (Hm @ upv + g)
    y0 = np.linalg.solve(M, rhs)
    n = M.shape[0]
    A = np.zeros((len(rows), n))
    d = np.zeros(len(rows))
    for r, (b, c, bv, up) in enumerate(rows):
        # c'(up + T y) = bv with T the leg's 3x3 block of Tb
        A[r, 3 * b:3 * b + 3] = c @ Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3]
        d[r] = bv - c @ up
    keep = np.linalg.matrix_rank(A) == len(rows)
    MiA = np.linalg.solve(M, A.T)
    S = A @ MiA
    lam = np.linalg.lstsq(S, A @ y0 - d, rcond=None)[0] if not keep else np.linalg.solve(S, A @ y0 - d)
    y = y0 - MiA @ lam
    return upv + Tb @ y


def polish_traced(Hm, g, act, mu, fmax, max_rounds=12, tol_p=1e-9, tol_d=1e-9):
    """hybrid_proto.polish(rule="single") keeping every round's active set."""
    nls = len(act)
    act = list(act)
    trace = [list(act)]
    for rd in range(1, max_rounds + 1):
        u, apex = direct(Hm, g, act, mu, fmax)
        grad = Hm @ u + g
        gscale = max(1.0, np.max(np.abs(grad)))
        C = CR(mu)
        bb = np.array([0, 0, 0, 0, fmax])
        changed = False
        for b in range(nls):
            o = C @ u[3 * b:3 * b + 3] - bb
            gl = grad[3 * b:3 * b + 3]
            cand = [(o[i], i) for i in range(5) if not (act[b] >> i) & 1 and o[i] > tol_p * fmax]
            if cand:
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
            return u, rd, True, trace
        trace.append(list(act))
    return u, max_rounds, False, trace


def main():
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    sbase = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
    srow = float(sys.argv[3]) if len(sys.argv) > 3 else 2.5
    p, H, rec, con = synth.config_batch(2, count=cnt)
    op = O.params_from(p)
    mu, fmax = p.mu, p.f_max
    base_c, new_c, errs = [], [], []
    kinds = {"first": 0, "schur": 0, "refactor": 0}
    ks = []
    slow = []
    for q in range(cnt):
        Hm, g, st, idx = reduced_qp(op, H, rec[q], con[q])
        f, s, z, it = ipm(Hm, g, st, p, "split", tol=1e-4)
        u, rd, ok, trace = polish_traced(Hm, g, guess(f, s, z, fmax, 1e-3), mu, fmax)
        cost0 = 55 + 42 * it + 45 * rd
        # the scheme: round 1 factorises; round r solves trace[r-1]; a Schur round when trace[r-1] only adds to the
        # factorised base set
        cost = 55 + 42 * it
        basei = 0
        kinds["first"] += 1
        cost += 45
        for r in range(1, rd):
            rows = schur_rows(trace[basei], trace[r], mu, fmax)
            if rows is not None and len(rows) <= 12:
                us = schur_solve(Hm, g, trace[basei], rows, mu, fmax)
                ud, _ = direct(Hm, g, trace[r], mu, fmax)
                errs.append(np.max(np.abs(us - ud)) / max(1.0, np.max(np.abs(ud))))
                kinds["schur"] += 1
                ks.append(len(rows))
                cost += sbase + srow * len(rows)
            else:
                kinds["refactor"] += 1
                basei = r
                cost += 45
        base_c.append(cost0)
        new_c.append(cost)
        slow.append((cost0, cost, it, rd, [len(schur_rows(trace[0], t, mu, fmax) or []) if schur_rows(trace[0], t, mu, fmax) is not None else -1 for t in trace[1:]]))
    base_c, new_c = np.array(base_c), np.array(new_c)
    print(f"{cnt} QPs: rounds {kinds}; update rows per Schur round mean {np.mean(ks) if ks else 0:.2f} max {max(ks) if ks else 0}")
    print(f"  update vs direct solve: max rel err {max(errs) if errs else 0:.2e}")
    print(f"  modelled kcycles/QP: base mean {base_c.mean():.1f} max {base_c.max():.0f}; Schur rounds mean {new_c.mean():.1f} max {new_c.max():.0f}")
    for c0, c1, it, rd, kk in sorted(slow, reverse=True)[:10]:
        print(f"    base {c0:.0f} -> {c1:.0f}  ipm {it} rounds {rd} rows-vs-first {kk}")


if __name__ == "__main__":
    main()

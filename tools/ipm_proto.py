#!/usr/bin/env python3
"""Dev tool (CPU): numpy replica of the dense-path interior point (lmpc_dense.hip: weight-share start,
Mehrotra predictor-corrector, step fraction 0.99, stop at mean complementarity < tol_mu) on the reduced
condensed QP, to measure iteration counts of variants before touching the kernel -- here Gondzio
centrality correctors (each one more solve with the same factorisation).  The polish is not modelled."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_proto import reduced_qp  # noqa: E402
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def ipm(Hm, g, st, p, H, tol=1e-8, ncorr=0, frac=0.99, max_iter=40):
    nls = len(st)
    mu_f, fmax = p.mu, p.f_max
    # rows: o = C f - b <= 0 ; faces -fx-mu fz, fx-mu fz, -fy-mu fz, fy-mu fz, fz-fmax
    Cl = np.array([[-1, 0, -mu_f], [1, 0, -mu_f], [0, -1, -mu_f], [0, 1, -mu_f], [0, 0, 1.0]])
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
    solves = 0
    while True:
        mu = s @ z / m
        if mu < tol or it >= max_iter:
            return f, it, solves
        W = z / s
        K = Hm + C.T @ (W[:, None] * C)
        Kinv = np.linalg.inv(K)  # one factorisation per iteration
        # predictor: full point u_aff
        u = Kinv @ -(g + C.T @ (W * (s - bvec)))
        solves += 1
        dsa = -(C @ u - bvec) - s
        dza = -z - W * dsa
        amax = 1.0
        for v, d in ((s, dsa), (z, dza)):
            neg = d < 0
            if neg.any():
                amax = min(amax, np.min(-v[neg] / d[neg]))
        mu_aff = (s + amax * dsa) @ (z + amax * dza) / m
        sig = (mu_aff / mu) ** 3
        smu = sig * mu
        # corrector (combined direction), written for the full point
        wv = (z * (s - bvec) + smu - dsa * dza) / s
        u = Kinv @ -(g + C.T @ wv)
        solves += 1
        ds = -(C @ u - bvec) - s
        dz = (smu - z * s - dsa * dza - z * ds) / s
        df = u - f

        def step(df, ds, dz):
            a = 1.0
            for v, d in ((s, ds), (z, dz)):
                neg = d < 0
                if neg.any():
                    a = min(a, np.min(-v[neg] / d[neg]))
            return a

        a = step(df, ds, dz)
        for _ in range(ncorr):  # Gondzio centrality correctors
            at = min(1.0, 1.5 * a + 0.1)
            v = (s + at * ds) * (z + at * dz)
            lo, hi = 0.1 * smu, 10.0 * smu
            t = np.clip(v, lo, hi) - v
            t = np.maximum(t, -hi)
            dfc = Kinv @ -(C.T @ (t / s))
            solves += 1
            dsc = -(C @ dfc)
            dzc = t / s - W * dsc
            a2 = step(df + dfc, ds + dsc, dz + dzc)
            if a2 >= 1.01 * a:
                df, ds, dz, a = df + dfc, ds + dsc, dz + dzc, a2
            else:
                break
        a = min(1.0, frac * a)
        f = f + a * df
        s = s + a * ds
        z = z + a * dz
        it += 1


def main():
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    p, H, rec, con = synth.config_batch(2, count=cnt)
    op = O.params_from(p)
    res = {}
    for ncorr in (0, 1, 2):
        its, sol, err = [], [], 0.0
        for b in range(cnt):
            Hm, g, st, idx = reduced_qp(op, H, rec[b], con[b])
            f, it, ns = ipm(Hm, g, st, p, H, ncorr=ncorr)
            its.append(it)
            sol.append(ns)
            ref, _, _ = O.solve(op, H, rec[b], con[b])
            mine = np.zeros(12 * H)
            mine[idx] = f
            err = max(err, np.max(np.abs(mine - ref.reshape(-1)) / np.maximum(1, np.abs(ref.reshape(-1)))))
        its = np.array(its)
        print(f"gondzio correctors {ncorr}: IPM iterations mean {its.mean():.2f} p99 {np.percentile(its, 99):.0f} "
              f"max {its.max()}; solves mean {np.mean(sol):.1f}; IPM-only max rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()

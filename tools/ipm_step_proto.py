#!/usr/bin/env python3
"""Dev tool (CPU): step-length rules of the dense-path interior point (lmpc_dense.hip), priced on the B = 1024 tail
before touching the kernel.  numpy replica of the kernel's Mehrotra loop (weight-share start, one combined
predictor-corrector per iteration, stop at mean complementarity < tol_mu) followed by the kernel's active-set polish
(tools/hybrid_proto.py polish: z > s, lift-off apex, one face in or out per leg-step per round).  Variants:
  same    -- one step length for f, s, z (the kernel's rule), fraction 0.99;
  split   -- separate primal (f, s) and dual (z) step lengths, each fraction 0.99;
  adapt   -- one step length, fraction 1 - min(0.01, mu) (Mehrotra's adaptive fraction to the boundary).
Cost model (cycles per QP, DESIGN.md 4b stamps): IPM iteration 42 k, polish round 45 k, prologue 55 k."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_proto import reduced_qp  # noqa: E402
from hybrid_proto import CR, polish  # noqa: E402
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


CORR = [0, 0]  # gondzio: correctors accepted / rejected


def ipm(Hm, g, st, p, rule="same", tol=1e-8, max_iter=40):
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

    def step(v, d):
        neg = d < 0
        return min(1.0, np.min(-v[neg] / d[neg])) if neg.any() else 1.0

    while True:
        mu = s @ z / m
        if mu < tol or it >= max_iter:
            return f, s, z, it
        W = z / s
        K = Hm + C.T @ (W[:, None] * C)
        Kinv = np.linalg.inv(K)
        u = Kinv @ -(g + C.T @ (W * (s - bvec)))
        dsa = -(C @ u - bvec) - s
        dza = -z - W * dsa
        amax = min(step(s, dsa), step(z, dza))
        mu_aff = (s + amax * dsa) @ (z + amax * dza) / m
        smu = (mu_aff / mu) ** float(os.environ.get("SIGMA_EXP", 3)) * mu
        wv = (z * (s - bvec) + smu - dsa * dza) / s
        u = Kinv @ -(g + C.T @ wv)
        ds = -(C @ u - bvec) - s
        dz = (smu - z * s - dsa * dza - z * ds) / s
        df = u - f
        if rule.startswith("gondzio"):  # multiple centrality correctors (Colombo & Gondzio), same factorisation
            kmax = int(rule[7:].rstrip("s") or 2)
            a0 = min(step(s, ds), step(z, dz))
            for _ in range(kmax):
                at = min(1.0, 1.5 * a0 + 0.1)
                v = (s + at * ds) * (z + at * dz)
                mt = smu if smu > 0 else mu * 0.1
                t = np.where(v < 0.1 * mt, 0.1 * mt - v, np.where(v > 10 * mt, np.maximum(10 * mt - v, -10 * mt), 0.0))
                dfc = Kinv @ -(C.T @ (t / s))
                dsc = -C @ dfc
                dzc = (t - z * dsc) / s
                ds2, dz2, df2 = ds + dsc, dz + dzc, df + dfc
                a1 = min(step(s, ds2), step(z, dz2))
                if a1 >= a0 + 0.1 * (at - a0) * 0.1 + 1e-12 and a1 > a0:
                    ds, dz, df, a0 = ds2, dz2, df2, a1
                    CORR[0] += 1
                else:
                    CORR[1] += 1
                    break
            if rule.endswith("s"):  # gondzioNs: correctors, then separate primal / dual step lengths
                ap, ad = min(1.0, 0.99 * step(s, ds)), min(1.0, 0.99 * step(z, dz))
            else:
                ap = ad = min(1.0, 0.99 * a0)
        elif rule.startswith("split"):  # split[frac]: separate primal / dual step lengths (the kernels, round 3)
            fr = float(rule[5:] or 0.99)
            ap = min(1.0, fr * step(s, ds))
            ad = min(1.0, fr * step(z, dz))
        elif rule.startswith("frac"):  # fixed fraction to the boundary, e.g. frac0.995
            ap = ad = min(1.0, float(rule[4:]) * min(step(s, ds), step(z, dz)))
        else:
            frac = 0.99 if rule == "same" else 1.0 - min(0.01, mu)
            ap = ad = min(1.0, frac * min(step(s, ds), step(z, dz)))
        f = f + ap * df
        s = s + ap * ds
        z = z + ad * dz
        it += 1


def ipm_history(Hm, g, st, p, tol=1e-8, max_iter=40):
    """Run the kernel's rule ('same') and keep every iterate (f, s, z, mu) for hand-over studies."""
    hist = []
    nls = len(st)
    for k in range(1, max_iter + 1):
        f, s, z, it = ipm(Hm, g, st, p, "same", tol=tol, max_iter=k)
        hist.append((f, s, z, float(s @ z / len(s))))
        if it < k:
            break
    return hist


def active_guess(f, s, z, fmax):
    nls = len(f) // 3
    act = []
    for b in range(nls):
        a = 0
        for i in range(5):
            if z[5 * b + i] > s[5 * b + i]:
                a |= 1 << i
        if np.max(np.abs(f[3 * b:3 * b + 3])) < 1e-6 * fmax:
            a = 15
        act.append(a)
    return act


def handover(cnt=256, mthr=1e-3, stable=1):
    """Hand the IPM iterate to the polish once the active-set guess has been stable for `stable` iterations and the
    mean complementarity is below mthr; a failed polish falls back to the full IPM + polish (its rounds paid)."""
    p, H, rec, con = synth.config_batch(2, count=cnt)
    op = O.params_from(p)
    base, new = [], []
    for b in range(cnt):
        Hm, g, st, idx = reduced_qp(op, H, rec[b], con[b])
        hist = ipm_history(Hm, g, st, p)
        f, s, z, mu = hist[-1]
        _, rd, ok = polish(Hm, g, active_guess(f, s, z, p.f_max), p.mu, p.f_max)
        full = 55e3 + 42e3 * len(hist) + 45e3 * rd
        base.append(full)
        cyc = None
        for k in range(stable, len(hist)):
            gk = active_guess(*hist[k][:3], p.f_max)
            if hist[k][3] < mthr and all(active_guess(*hist[k - j][:3], p.f_max) == gk for j in range(1, stable + 1)):
                _, rdk, okk = polish(Hm, g, gk, p.mu, p.f_max)
                cyc = 55e3 + 42e3 * (k + 1) + 45e3 * rdk if okk else full + 45e3 * rdk
                break
        new.append(cyc if cyc is not None else full)
    base, new = np.array(base), np.array(new)
    print(f"handover mthr {mthr:g} stable {stable}: mean {base.mean() / 1e3:.0f}k -> {new.mean() / 1e3:.0f}k, "
          f"max {base.max() / 1e3:.0f}k -> {new.max() / 1e3:.0f}k, p99 {np.percentile(new, 99) / 1e3:.0f}k", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "handover":
        for mthr in (1e-2, 1e-3, 1e-4):
            for stable in (1, 2):
                handover(int(sys.argv[2]) if len(sys.argv) > 2 else 256, mthr, stable)
        return
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rules = sys.argv[2].split(",") if len(sys.argv) > 2 else ["same", "split", "adapt"]
    p, H, rec, con = synth.config_batch(2, count=cnt)
    op = O.params_from(p)
    qps = [reduced_qp(op, H, rec[b], con[b]) for b in range(cnt)]
    for rule in rules:
        its, rds, cyc, bad = [], [], [], 0
        for b, (Hm, g, st, idx) in enumerate(qps):
            f, s, z, it = ipm(Hm, g, st, p, rule)
            u, rd, ok = polish(Hm, g, active_guess(f, s, z, p.f_max), p.mu, p.f_max)
            bad += not ok
            its.append(it)
            rds.append(rd)
            cyc.append(55e3 + 42e3 * it + 45e3 * rd)
        if rule.startswith("gondzio"):
            print(f"  correctors accepted {CORR[0]} rejected {CORR[1]} (each ~3 k cycles: one more solve)")
            CORR[0] = CORR[1] = 0
        its, rds, cyc = np.array(its), np.array(rds), np.array(cyc)
        print(f"{rule:6s}: ipm mean {its.mean():.2f} max {its.max()} | rounds mean {rds.mean():.2f} max {rds.max()} | "
              f"model cycles mean {cyc.mean() / 1e3:.0f} k max {cyc.max() / 1e3:.0f} k p99 {np.percentile(cyc, 99) / 1e3:.0f} k"
              f" | polish failed {bad}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Dev tool (CPU): the interior point's hand-over to the polish, priced in the numpy replica of the dense path
(tools/ipm_step_proto.py loop + tools/hybrid_proto.py polish) on config 2 QPs.

For a grid of hand-over tolerances (mean complementarity) and active-set classification thresholds
(face active where z > theta * s), report the interior-point iterations, the polish rounds and the modelled
cycles per QP (DESIGN.md 4b stamps: IPM iteration 42 k, polish round 45 k, prologue 55 k); the launch at
B = 1024 waits for the slowest QP, so the max matters as much as the mean.
  tools/polish_guess_proto.py [count] [first_index]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gi_proto import reduced_qp  # noqa: E402
from hybrid_proto import polish  # noqa: E402
from ipm_step_proto import ipm  # noqa: E402
from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def guess(f, s, z, fmax, theta):
    nls = len(f) // 3
    act = []
    for b in range(nls):
        a = 0
        for i in range(5):
            if z[5 * b + i] > theta * s[5 * b + i]:
                a |= 1 << i
        if np.max(np.abs(f[3 * b:3 * b + 3])) < 1e-6 * fmax:
            a = 15
        act.append(a)
    return act


def main():
    cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    p, H, rec, con = synth.config_batch(int(os.environ.get("PG_CFG", "2")), count=cnt, first_index=first)
    op = O.params_from(p)
    qps = [reduced_qp(op, H, rec[b], con[b]) for b in range(cnt)]
    for tol in [float(x) for x in os.environ.get("PG_TOLS", "1e-8,1e-6,1e-5").split(",")]:
        for rule in os.environ.get("PG_RULES", "same").split(","):
            runs = [ipm(Hm, g, st, p, rule, tol=tol) for (Hm, g, st, idx) in qps]
            for theta in [float(x) for x in os.environ.get("PG_THETAS", "1,0.1,10").split(",")]:
                its, rds, bad = [], [], 0
                for (Hm, g, st, idx), (f, s, z, it) in zip(qps, runs):
                    _, rd, ok = polish(Hm, g, guess(f, s, z, p.f_max, theta), p.mu, p.f_max, max_rounds=12,
                                       rule=os.environ.get("PG_POLISH", "single"))
                    bad += not ok
                    its.append(it)
                    rds.append(rd)
                its, rds = np.array(its), np.array(rds)
                cyc = 55e3 + 42e3 * its + 45e3 * rds
                print(f"{rule:9s} tol {tol:.0e} theta {theta:g}: ipm {its.mean():.2f} (max {its.max()}) rounds"
                      f" {rds.mean():.2f} (max {rds.max()}) cycles mean {cyc.mean() / 1e3:.0f}k max {cyc.max() / 1e3:.0f}k"
                      f" p99 {np.percentile(cyc, 99) / 1e3:.0f}k failed {bad}", flush=True)


if __name__ == "__main__":
    main()

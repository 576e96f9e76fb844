#!/usr/bin/env python3
"""Dev tool (CPU): speculative polish from every interior-point iterate, priced in the numpy
replica of the dense path: the earliest verified polish over the iterates (oracle choice), per QP, against the kernel's
hand-over at complementarity 1e-4.  python tools/tail_spec_polish_proto.py [count] [theta]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tools'))
from gi_proto import reduced_qp
from hybrid_proto import polish
from ipm_step_proto import ipm
from polish_guess_proto import guess
from legged_mpc_control_amd import synth
from oracle import oracle as O

cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
theta = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
p, H, rec, con = synth.config_batch(2, count=cnt)
op = O.params_from(p)
cyc = lambda its, rds: 55 + 42 * its + 45 * rds
base, spec = [], []
hist = []
for b in range(cnt):
    Hm, g, st, idx = reduced_qp(op, H, rec[b], con[b])
    f, s, z, it = ipm(Hm, g, st, p, "split", tol=1e-4)
    _, rd0, ok0 = polish(Hm, g, guess(f, s, z, p.f_max, 1e-3), p.mu, p.f_max, max_rounds=12)
    t0 = cyc(it, rd0)
    best = t0
    rk = []
    for k in range(1, it):
        f2, s2, z2, _ = ipm(Hm, g, st, p, "split", tol=0.0, max_iter=k)
        _, rd, ok = polish(Hm, g, guess(f2, s2, z2, p.f_max, theta), p.mu, p.f_max, max_rounds=8)
        rk.append(rd if ok else 99)
        if ok:
            best = min(best, cyc(k, rd))
    hist.append((it, rd0, rk))
    base.append(t0); spec.append(best)
base, spec = np.array(base), np.array(spec)
print(f"theta {theta}: base mean {base.mean():.0f} max {base.max()}; speculative polish from every iterate (oracle-earliest): mean {spec.mean():.0f} max {spec.max()}")
for q in np.argsort(-base)[:8]:
    print(q, hist[q], base[q], spec[q])

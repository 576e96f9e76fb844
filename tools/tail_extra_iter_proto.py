#!/usr/bin/env python3
"""Dev tool (CPU): the config-2 launch tail in the numpy replica of the dense path (tools/ipm_step_proto.py +
tools/hybrid_proto.py, which reproduce the kernel's 5.30 / 1.51 mean and 7 / 4 max interior-point iterations /
polish rounds): polish rounds when the hand-over waits 0..3 more interior-point iterations, per QP; cycle model
55k + 42k x iterations + 45k x rounds.  python tools/tail_extra_iter_proto.py [count]"""
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
p, H, rec, con = synth.config_batch(2, count=cnt)
op = O.params_from(p)
rows = []
for b in range(cnt):
    Hm, g, st, idx = reduced_qp(op, H, rec[b], con[b])
    f, s, z, it = ipm(Hm, g, st, p, "split", tol=1e-4)
    res = [it]
    for extra in range(4):
        f2, s2, z2, it2 = ipm(Hm, g, st, p, "split", tol=0.0, max_iter=it + extra)
        _, rd, ok = polish(Hm, g, guess(f2, s2, z2, p.f_max, 1e-3), p.mu, p.f_max, max_rounds=12)
        res.append(rd if ok else 99)
    rows.append(res)
rows = np.array(rows)
cyc = lambda its, rds: 55 + 42 * its + 45 * rds
base = cyc(rows[:, 0], rows[:, 1])
print("base mean", base.mean(), "max", base.max())
order = np.argsort(-base)
for q in order[:15]:
    print(q, "it", rows[q, 0], "rounds at +0..+3:", rows[q, 1:], "cyc", [cyc(rows[q,0]+e, rows[q,1+e]) for e in range(4)])
best = np.min([cyc(rows[:, 0] + e, rows[:, 1 + e]) for e in range(4)], axis=0)
print("oracle-best extra iterations: mean", best.mean(), "max", best.max())

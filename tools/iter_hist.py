"""Dev tool: joint distribution of IPM iterations / polish rounds over a config batch (run under gpurun)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

torch.cuda.init()
from legged_mpc_control_amd import BatchedConvexQPSolver, synth

for cid in (2, 4):
    p, H, rec, con = synth.config_batch(cid, count=4096 if cid == 4 else None)
    s = BatchedConvexQPSolver(p, H, len(rec))
    grf, st, it = s.solve(rec, con)
    ipm, rd = it & 0xFFFF, it >> 16
    c = collections.Counter(zip(ipm.tolist(), rd.tolist()))
    print(f"config {cid} B={len(rec)}: ipm mean {ipm.mean():.2f} max {ipm.max()} | rounds mean {rd.mean():.2f} max {rd.max()} | status {np.bincount(st, minlength=3)}")
    for (a, b), n in sorted(c.items()):
        print(f"  ipm {a:2d} rounds {b}: {n}")

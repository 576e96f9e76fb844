import sys, numpy as np
sys.path.insert(0, '.')
import torch; torch.cuda.init()
from legged_mpc_control_amd import BatchedConvexQPSolver, synth
for cid, cnt in ((2, 1024), (4, 4096)):
    p, H, rec, con = synth.config_batch(cid, count=cnt)
    s = BatchedConvexQPSolver(p, H, cnt)
    grf, st, it = s.solve(rec, con)
    ipm, rd = it & 0xFFFF, it >> 16
    f = grf.reshape(cnt, H, 4, 3)
    stance = con.astype(bool)
    apex = (np.abs(f).max(-1) == 0.0) & stance          # stance leg-step at the apex (f = 0)
    napex = apex.sum((1, 2))
    fz = f[..., 2]
    mu = 0.3
    # friction-face activity in the solution
    fric = (np.abs(np.abs(f[..., 0]) - mu * fz) < 1e-9) | (np.abs(np.abs(f[..., 1]) - mu * fz) < 1e-9)
    nfric = (fric & stance & ~apex).sum((1, 2))
    top = (np.abs(fz - 180.0) < 1e-9).sum((1, 2))
    print(f"config {cid}: ipm mean {ipm.mean():.2f}")
    for k in sorted(set(napex.tolist()))[:8]:
        m = napex == k
        print(f"  apex leg-steps {k:3d}: n={m.sum():5d} ipm mean {ipm[m].mean():.2f} max {ipm[m].max()} rounds mean {rd[m].mean():.2f} max {rd[m].max()}")
    for lo, hi in ((0, 1), (1, 5), (5, 20), (20, 100)):
        m = (nfric >= lo) & (nfric < hi)
        if m.any():
            print(f"  friction-active leg-steps [{lo},{hi}): n={m.sum():5d} ipm mean {ipm[m].mean():.2f} max {ipm[m].max()} rounds {rd[m].mean():.2f}")
    m = top > 0
    print(f"  fz=fmax active: n={m.sum()} ipm mean {ipm[m].mean() if m.any() else 0:.2f}")
    worst = np.argsort(-(ipm + rd))[:8]
    for b in worst:
        print(f"  worst b={b}: ipm {ipm[b]} rd {rd[b]} apex {napex[b]} fric {nfric[b]} stance {stance[b].sum()} gait-contacts {con[b].sum(0)}")

#!/usr/bin/env python3
"""Dev tool (CPU): per-QP cycles of the LDS Riccati kernel (tools/lq_stamps.py with LQ_STAMPS_DUMP, run on the box into
gpurun_out/cost/c{5,3}.npz) against features of the QP inputs -- is there a cost predictor for longest-first dispatch?"""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from legged_mpc_control_amd import synth
for cid in (5, 3):
    d = np.load(f"gpurun_out/cost/c{cid}.npz")
    cyc, it = d["cycles"], d["it"]
    n = len(cyc)
    p, H, rec, con = synth.config_batch(cid, count=n)
    ipm = it & 0xffff; rnd = it >> 16
    feats = {}
    con = con.reshape(n, -1)
    feats["stance leg-steps"] = con.sum(1)
    r = rec.reshape(n, -1)
    # per-record columns: x0 at the start (12), then R (9), feet (12), x_ref ...
    x0 = r[:, :12]
    feats["|x0 vel|"] = np.linalg.norm(x0[:, 6:12], axis=1)
    feats["|x0 ang|"] = np.linalg.norm(x0[:, 0:3], axis=1)
    xref = r[:, 40:40 + 12 * H].reshape(n, H, 12) if r.shape[1] >= 40 + 12 * H else None
    if xref is not None:
        feats["|xref0 - x0|"] = np.linalg.norm(xref[:, 0] - x0, axis=1)
        feats["|xref vel|"] = np.linalg.norm(xref[:, :, 6:12], axis=(1, 2))
    # contact switches
    c3 = con.reshape(n, H, 4)
    feats["contact switches"] = np.abs(np.diff(c3.astype(int), axis=1)).sum((1, 2))
    print(f"config {cid}: {n} QPs, cycles mean {cyc.mean():.0f} cv {cyc.std()/cyc.mean():.3f}; corr(cycles, ipm) {np.corrcoef(cyc, ipm)[0,1]:.2f}, corr(cycles, rounds) {np.corrcoef(cyc, rnd)[0,1]:.2f}")
    for k, v in feats.items():
        if np.std(v) > 0:
            print(f"   corr(cycles, {k:18s}) {np.corrcoef(cyc, v)[0,1]:+.3f}")
        else:
            print(f"   {k}: constant")

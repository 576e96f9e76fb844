#!/usr/bin/env python3
"""Dev tool (GPU box): bits of the fused dense + Riccati launch against the two launches, per QP and path.
    python tools/fused_check.py solve LIB OUT.npy [count]   (one process per library: LMPC_LIB is read at import)
    python tools/fused_check.py compare A.npy B.npy [count]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] == "solve":
    os.environ["LMPC_LIB"] = sys.argv[2]
    import torch
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    cnt = int(sys.argv[4]) if len(sys.argv) > 4 else 512
    p, H, rec, con = synth.config_batch(4, count=cnt)
    s = BatchedConvexQPSolver(p, H, max_batch=0, dense_path="ipm")
    dev = torch.device("cuda:0")
    out = torch.empty((cnt, H, 12), dtype=torch.float64, device=dev)
    st = torch.empty(cnt, dtype=torch.int32, device=dev)
    s.solve_device(torch.from_numpy(rec).to(dev), torch.from_numpy(con).to(dev), out, st)
    torch.cuda.synchronize()
    np.save(sys.argv[3], out.cpu().numpy())
else:
    from legged_mpc_control_amd import synth
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    cnt = a.shape[0]
    p, H, rec, con = synth.config_batch(4, count=cnt)
    nls = (con.reshape(cnt, -1) != 0).sum(1)
    diff = np.any(a.reshape(cnt, -1) != b.reshape(cnt, -1), axis=1)
    dense = (nls >= 1) & (nls <= 20)
    print(f"{cnt} QPs: {dense.sum()} dense-eligible; differing bits: {diff.sum()} ({(diff & dense).sum()} dense-eligible, "
          f"{(diff & ~dense).sum()} Riccati); max |diff| {np.max(np.abs(a - b)):.3e}")

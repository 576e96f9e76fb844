import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import torch; torch.cuda.init()
from test_gpu_hoqp import load, dims_from, unpack
from legged_mpc_control_amd import hoqp
for group in ("n64", "wbc"):
    g = load(group); dims = dims_from(g["dims"]); B = g["rec"].shape[0]
    x, w, st, it = hoqp.HoqpBatch(dims, B).solve(g["rec"])
    print(group, "status", st.tolist())
    print(" ipm", (it & 0xFFFF).tolist())
    print(" xo ", (it >> 16).tolist())
    for b in range(min(B, 3)):
        levels = unpack(g["rec"][b], dims)
        scale = 1.0 + max(float(np.max(np.abs(g["rec"][b]))), float(np.max(np.abs(g["x"][b]))))
        errs = [float(np.max(np.abs(a @ x[b][l] - a @ g["x"][b][l]))) / scale if a.shape[0] else 0.0 for l, (a, bb, d, f) in enumerate(levels)]
        print(" chain", b, "A dx / scale per level", ["%.1e" % e for e in errs], "slack err %.1e" % (np.max(np.abs(w[b] - g["w"][b])) / scale))

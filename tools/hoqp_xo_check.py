"""Dev tool (GPU): crossover outcome per level (iteration word bits 16-17: 1 tried, 3 verified) on the committed WBC
golden chains, with the default options and with crossover off, plus the largest deviation from the golden answers."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from legged_mpc_control_amd import hoqp as hq
import test_gpu_hoqp as T

g = T.load("wbc")
dims = T.dims_from(g["dims"])
B = g["rec"].shape[0]
on = hq.HoqpBatch(dims, B)
x1, w1, st1, it1 = on.solve(g["rec"])
print("status", np.bincount(st1, minlength=3), "ipm iters per level mean", (it1 & 0xFFFF).mean(0))
for l in range(it1.shape[1]):
    xo = it1[:, l] >> 16
    print(f"level {l}: crossover bits histogram {np.bincount(xo, minlength=4)}; chains not verified: {np.nonzero(xo != 3)[0][:10]}"
          f" (their ipm iterations {(it1[xo != 3, l] & 0xFFFF)[:10]})")
bad = 0
for b in range(B):
    try:
        T.check_against(g["rec"][b], dims, x1[b], w1[b], g["x"][b], g["w"][b], bool(g["pinned"]), 1e-9)
    except AssertionError as e:
        bad += 1
        if bad <= 5:
            print("chain", b, e)
print("chains beyond 1e-9:", bad, "of", B)

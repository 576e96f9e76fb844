#!/usr/bin/env python3
"""Dev tool (GPU box): per chain and level of a committed WBC golden group (tests/golden/hoqp_golden.npz): interior-point
iterations, the crossover's outcome and (on a -DLMPC_HQ_ITDIAG build) its failure reason and first-pass iterations,
and the level's A x deviation from the golden answer relative to the data's scale (the GPU tests' measure).

    LMPC_LIB=tools/build/liblmpc_TAG.so python tools/hoqp_golden_probe.py [group ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def main():
    import test_gpu_hoqp as T
    from legged_mpc_control_amd import hoqp as hq

    for group in sys.argv[1:] or ["n64"]:
        g = T.load(group)
        dims = T.dims_from(g["dims"])
        rec = g["rec"]
        x, w, st, word = hq.HoqpBatch(dims, rec.shape[0]).solve(rec)
        print(f"== {group}: status {np.bincount(st, minlength=3).tolist()}")
        for b in range(rec.shape[0]):
            levels = T.unpack(rec[b], dims)
            scale = 1.0 + max(float(np.max(np.abs(rec[b]))), float(np.max(np.abs(g["x"][b]))))
            cells = []
            for l, (a, bb, d, f) in enumerate(levels):
                err = float(np.max(np.abs(a @ x[b, l] - a @ g["x"][b, l]))) / scale if a.shape[0] else 0.0
                wd = int(word[b, l])
                cells.append(f"L{l} it {wd & 0xFFFF}/{(wd >> 20) & 0xFF} xo {(wd >> 16) & 3} why {(wd >> 28) & 7} "
                             f"err {err:.1e}")
            print(f"  chain {b}: " + " | ".join(cells))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Dev tool (CPU): compare tools/hoqp_dump.py's GPU answers with the restatement (oracle/hoqp.py) chain by chain:
every level's final x relative to the data's scale, as tools/bench_hoqp.py's parity sample does, over all chains.

    python tools/hoqp_parity_cpu.py gpurun_out/hqpar/gpu.npz [workers]
"""
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def one(args):
    i, seed0 = args
    from legged_mpc_control_amd import wbc as W
    from oracle import hoqp as Q

    tasks = W.synth_wbc_tasks(seed0 + i)
    lv = []
    for t in tasks:
        lv.append(Q.HoQp(Q.Task(t.a, t.b, t.d, t.f), lv[-1] if lv else None))
    return i, np.stack([h.solution() for h in lv]), [t.a for t in tasks]


def main():
    d = np.load(sys.argv[1], allow_pickle=False)
    x, seed0 = d["x"], int(d["seed0"])
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    n = x.shape[0]
    errs = np.zeros(n)
    axe = np.zeros(n)
    with Pool(workers) as p:
        for i, xr, As in p.imap_unordered(one, [(i, seed0) for i in range(n)], chunksize=8):
            errs[i] = np.max(np.abs(x[i, -1] - xr[-1])) / (1.0 + np.max(np.abs(xr[-1])))
            axe[i] = max(float(np.max(np.abs(a @ (x[i, l] - xr[l])))) if a.shape[0] else 0.0 for l, a in enumerate(As))
    order = np.argsort(-errs)
    print(f"{n} chains: final x relative error max {errs.max():.2e} p99 {np.percentile(errs, 99):.2e} "
          f"median {np.median(errs):.2e}; every level's A x: max abs {axe.max():.2e}; worst chains {order[:5].tolist()}")


if __name__ == "__main__":
    main()

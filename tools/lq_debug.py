#!/usr/bin/env python3
"""Dev tool (GPU): the LDS-resident Riccati kernel's iterates after 1..3 interior-point iterations (max_iter = n,
one polish round, one attempt: the kernel returns the interior-point iterate) and its final answer, on a few QPs of
configs 1 and 2 with the dense path off, saved to gpurun_out/lq_debug.npz for a CPU comparison against
tools/lq_proto.py (tools/lq_debug.py compare)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def cases():
    from legged_mpc_control_amd import synth

    out = []
    for cid, n in ((1, 1), (2, 2), (4, 2)):
        p, H, rec, con = synth.config_batch(cid, count=n)
        out.append((cid, p, H, rec, con))
    return out


def run_gpu():
    from legged_mpc_control_amd import BatchedConvexQPSolver
    from legged_mpc_control_amd.solver import solver_options

    res = {}
    for cid, p, H, rec, con in cases():
        for path in ("lds", "scratch"):
            for it in (1, 2, 3, 0):
                o = solver_options(max_iter=it, max_rounds=1, max_attempts=1) if it else solver_options()
                s = BatchedConvexQPSolver(p, H, max_batch=len(rec), dense_path="off", riccati_path=path, options=o)
                g, st, its = s.solve(rec, con)
                res[f"c{cid}_{path}_{it}"] = g
                res[f"c{cid}_{path}_{it}_st"] = st
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "lq_debug.npz"), **res)
    print("saved", len(res))


def compare():
    import lq_proto as Pr

    d = np.load(os.path.join(ROOT, "gpurun_out", "lq_debug.npz"))
    for cid, p, H, rec, con in cases():
        for it in (1, 2, 3, 0):
            for b in range(len(rec)):
                M = Pr.model(p, H, rec[b], con[b])
                kw = dict(max_iter=it, max_rounds=1, max_attempts=1) if it else {}
                u, _, _, ok = Pr.solve(M, **kw)
                u = u.reshape(H, 12)
                for path in ("lds", "scratch"):
                    g = d[f"c{cid}_{path}_{it}"][b]
                    err = np.max(np.abs(g - u) / np.maximum(1, np.abs(u)))
                    print(f"config {cid} QP {b} iters {it or 'all'} {path:8s}: max rel diff vs prototype {err:.2e}"
                          f"  step0 fz gpu {g[0, 2]:.4f} proto {u[0, 2]:.4f}")


if __name__ == "__main__":
    compare() if len(sys.argv) > 1 and sys.argv[1] == "compare" else run_gpu()

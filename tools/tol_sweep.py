"""Dev tool: IPM stopping tolerance vs polish work and parity (run under gpurun)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from legged_mpc_control_amd import BatchedConvexQPSolver, synth
from legged_mpc_control_amd import _native as N
from oracle import oracle as O


def main():
    cases = [(10, 0, 128), (10, -1, 128), (20, 0, 48), (30, -1, 32)]
    data = {}
    for (H, gait, B) in cases:
        p = synth.params("go1")
        rec, con = synth.fill(p, synth.synth_cfg("go1", gait), H, B, seed=4242 + H - gait)
        op = O.params_from(p)
        ref = np.stack([O.solve(op, H, rec[b], con[b])[0] for b in range(B)])
        data[(H, gait)] = (p, rec, con, ref)
    for tol in (1e-8, 1e-7, 1e-6, 1e-5, 1e-4):
        o = N.LmpcOptions()
        N.lib().lmpc_options_default(ctypes_byref(o))
        o.tol_mu = tol
        line = [f"tol_mu={tol:.0e}"]
        for (H, gait, B) in cases:
            p, rec, con, ref = data[(H, gait)]
            s = BatchedConvexQPSolver(p, H, B, options=o)
            grf, st, it = s.solve(rec, con)
            err = np.max(np.abs(grf - ref) / np.maximum(1.0, np.abs(ref)))
            line.append(f"H{H}g{gait}: err {err:.1e} st {np.bincount(st, minlength=3).tolist()} "
                        f"ipm {np.mean(it & 0xffff):.2f} rd {np.mean(it >> 16):.2f}")
        p, H, rec, con = synth.config_batch(2)
        s = BatchedConvexQPSolver(p, H, len(rec), options=o)
        s.solve(rec, con)
        t = time.perf_counter()
        for _ in range(5):
            s.solve(rec, con)
        line.append(f"cfg2 host-path {1e3 * (time.perf_counter() - t) / 5:.3f} ms")
        print(" | ".join(line), flush=True)


def ctypes_byref(o):
    import ctypes
    return ctypes.byref(o)


if __name__ == "__main__":
    main()

"""Dev tool: the Riccati kernel's interior-point stop (tol_mu) and polish budget (max_rounds) against
the factorisations per QP and the wall time, on the Riccati-path configurations (dense path off).
Every setting must return the same exact optimum (max rel diff against the default).  Run under gpurun.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from legged_mpc_control_amd import BatchedConvexQPSolver, synth
from legged_mpc_control_amd import solver as SV


def timed(fn, n=3):
    fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return out, float(np.median(ts))


def main():
    cases = [(4, True, 16384), (3, False, 8192), (5, False, 4096), (2, False, 1024)]
    tols = [float(x) for x in os.environ.get("HO_TOLS", "1e-8,1e-6,1e-5,1e-4,1e-3").split(",")]
    rds = [int(x) for x in os.environ.get("HO_ROUNDS", "4,8").split(",")]
    for cfg_id, terrain, B in cases:
        p, H, rec, con = synth.config_batch(cfg_id, count=B)
        nrm = synth.normals(B, synth.BASE_SEED + cfg_id) if terrain else None
        s = BatchedConvexQPSolver(p, H, B)
        s.set_dense_path("off")
        g0 = None
        for tol in tols:
            for mr in rds:
                s.set_options(SV.solver_options(tol_mu=tol, max_rounds=mr))
                (g, st, it), t = timed(lambda: s.solve(rec, con, nrm))
                if g0 is None:
                    g0 = g
                ipm, rd = it & 0xffff, it >> 16
                f = ipm + rd
                err = np.max(np.abs(g - g0) / np.maximum(1.0, np.abs(g0)))
                print(f"config {cfg_id}{'t' if terrain else ''} H={H} B={B} tol_mu {tol:.0e} max_rounds {mr}: {t*1e3:8.2f} ms"
                      f"  ipm {ipm.mean():.2f} (max {ipm.max()})  rounds {rd.mean():.2f} (max {rd.max()})"
                      f"  factorisations {f.mean():.2f} (p99 {np.percentile(f, 99):.0f}, max {f.max()})"
                      f"  status {np.bincount(st, minlength=3)}  max rel diff {err:.2e}", flush=True)
        s.close()


if __name__ == "__main__":
    main()

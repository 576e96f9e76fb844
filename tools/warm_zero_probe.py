"""Dev tool: cold interior point vs the active-set polish started from an empty active set.

For every Riccati-path configuration, solve the same batch (dense path off) cold and through
lmpc_solve_batch_warm with act_in = 0 (every stance leg-step unconstrained), and report the
Riccati factorisations per QP (interior-point iterations + polish rounds), the host-path wall
time and the largest GRF difference between the two answers.  Run under gpurun.
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
    cases = [(4, True, 16384), (4, False, 16384), (2, False, 1024), (3, False, 8192), (5, False, 4096)]
    rounds = [int(x) for x in os.environ.get("WZ_ROUNDS", "12").split(",")]
    for cfg_id, terrain, B in cases:
        p, H, rec, con = synth.config_batch(cfg_id, count=B)
        nrm = synth.normals(B, synth.BASE_SEED + cfg_id) if terrain else None
        s = BatchedConvexQPSolver(p, H, B)
        s.set_dense_path("off")
        (g0, st0, it0), t0 = timed(lambda: s.solve(rec, con, nrm))
        f0 = (it0 & 0xffff) + (it0 >> 16)
        print(f"config {cfg_id}{' terrain' if terrain else ''} H={H} B={B}: cold  {t0*1e3:8.2f} ms  ipm {np.mean(it0 & 0xffff):.2f}"
              f" rounds {np.mean(it0 >> 16):.2f}  factorisations mean {f0.mean():.2f} max {f0.max()}"
              f"  status {np.bincount(st0, minlength=3)}", flush=True)
        act = np.zeros((B, H, 4), dtype=np.uint8)
        for wr in rounds:
            s.set_options(SV.solver_options(warm_rounds=wr))
            (g1, st1, it1, a1), t1 = timed(lambda: s.solve_warm(rec, con, act, nrm))
            ipm, rd = it1 & 0xffff, it1 >> 16
            f1 = ipm + rd
            fell = np.mean(ipm > 0)
            err = np.max(np.abs(g1 - g0) / np.maximum(1.0, np.abs(g0)))
            print(f"   warm0 rounds<={wr:2d} {t1*1e3:8.2f} ms  fallback {fell*100:5.1f}%  rounds mean {np.mean(rd):.2f}"
                  f" p50 {np.median(rd):.0f} p99 {np.percentile(rd, 99):.0f}  factorisations mean {f1.mean():.2f} max {f1.max()}"
                  f"  status {np.bincount(st1, minlength=3)}  max rel diff {err:.2e}", flush=True)
            hist = np.bincount(np.minimum(rd[ipm == 0], 30), minlength=31)
            print("      rounds histogram (no fallback):", " ".join(f"{i}:{v}" for i, v in enumerate(hist) if v), flush=True)
        s.close()


if __name__ == "__main__":
    main()

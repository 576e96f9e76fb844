"""Dev tool (GPU): one QP per call through the host-pointer C-ABI (the per-tick shape of the drop-in) on each
dense path, over many different config-2 instances: wall time per call (H2D + kernels + D2H) mean / p50 / p99.
Run under gpurun."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from legged_mpc_control_amd import BatchedConvexQPSolver, synth


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    for H, paths in ((10, ("gi", "ipm")), (30, ("off",))):
        cid = 2 if H == 10 else 5
        p, _, rec, con = synth.config_batch(cid, count=n, first_index=50000)
        for path in paths:
            s = BatchedConvexQPSolver(p, H, max_batch=1, dense_path=path)
            for b in range(5):
                s.solve(rec[b:b + 1], con[b:b + 1])
            ts = []
            for b in range(n):
                t = time.perf_counter()
                s.solve(rec[b:b + 1], con[b:b + 1])
                ts.append(time.perf_counter() - t)
            ts = np.array(ts) * 1e3
            print(f"H={H} path {path}: one QP per call over {n} instances: mean {ts.mean():.3f} ms p50 "
                  f"{np.median(ts):.3f} p99 {np.percentile(ts, 99):.3f} max {ts.max():.3f}", flush=True)
            s.close()


if __name__ == "__main__":
    main()

"""Dev tool: quick GPU-vs-oracle parity + timing probe (run under gpurun)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from legged_mpc_control_amd import synth, BatchedConvexQPSolver
from oracle import oracle as O

def main():
    for (H, gait, B) in ((10, 0, 64), (10, -1, 64), (20, 0, 32), (30, 0, 32), (30, -1, 32)):
        p = synth.params("go1"); cfg = synth.synth_cfg("go1", gait)
        rec, con = synth.fill(p, cfg, H, B, seed=777 + H)
        s = BatchedConvexQPSolver(p, H, B)
        grf, st, it = s.solve(rec, con)
        op = O.params_from(p)
        errs = []
        for b in range(B):
            ref, kkt, na = O.solve(op, H, rec[b], con[b])
            errs.append(np.max(np.abs(grf[b] - ref) / np.maximum(1, np.abs(ref))))
        errs = np.array(errs)
        print(f"H={H} gait={gait} B={B} maxerr={errs.max():.3e} worst={errs.argmax()} status={np.bincount(st, minlength=3)} ipm_it={np.mean(it & 0xffff):.1f} rounds={np.mean(it >> 16):.2f}", flush=True)
    H = 10; B = 1024
    p, H, rec, con = synth.config_batch(2)
    s = BatchedConvexQPSolver(p, H, B)
    s.solve(rec, con)
    t = time.perf_counter(); n = 5
    for _ in range(n): s.solve(rec, con)
    dt = (time.perf_counter() - t) / n
    print(f"config2 B=1024 H=10 host-path time {dt*1e3:.3f} ms -> {B/dt:.3e} QP/s", flush=True)

if __name__ == "__main__":
    main()

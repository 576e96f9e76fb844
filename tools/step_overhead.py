#!/usr/bin/env python3
"""Dev tool (GPU box): where config 2's per-step time goes outside the kernel (round 6).

    python tools/step_overhead.py [steps] [reps]

The bench's ms_per_step (wall clock over K steps) sat ~6 us above the kernel time its HIP events measure.  This
times K back-to-back solves (a) with a HIP event pair around every step (bench.py's timed loop), (b) with one pair
around the whole loop, and prints each mode's wall ms per step and the event-measured kernel ms, alternating the
modes `reps` times on the same box.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch

    from legged_mpc_control_amd import BatchedConvexQPSolver, synth

    dev = torch.device("cuda", 0)
    cfg = synth.CONFIGS[2]
    H, B = cfg["H"], cfg["batch"]
    solver = BatchedConvexQPSolver(synth.params(cfg["robot"]), H, max_batch=0, device=0, dense_path="ipm")
    d_cmd = solver.synth_commands_device(synth.config_cfg(2), B, synth.BASE_SEED + 2, first_index=0, device=dev)
    d_rec, d_con = solver.build_records_device(d_cmd)
    d_grf = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
    d_st = torch.empty(B, dtype=torch.int32, device=dev)
    d_it = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    for _ in range(10):
        solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream)
    torch.cuda.synchronize(dev)
    for r in range(reps):
        for mode in ("per-step events", "one event pair"):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if mode == "per-step events":
                for i in range(steps):
                    evs[i][0].record(stream)
                    solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream)
                    evs[i][1].record(stream)
            else:
                e0.record(stream)
                for i in range(steps):
                    solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream)
                e1.record(stream)
            torch.cuda.synchronize(dev)
            wall = (time.perf_counter() - t0) / steps * 1e3
            if mode == "per-step events":
                k = float(np.mean([a.elapsed_time(b) for a, b in evs]))
            else:
                k = e0.elapsed_time(e1) / steps
            print(f"rep {r} {mode:16s}: wall {wall:.4f} ms/step, events {k:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Dev tool: the WBC bench's distinct chains solved on the GPU, saved for a CPU-side parity check against the
restatement (tools/hoqp_parity_cpu.py), which takes minutes for 1024 chains -- too long to run silently on the box.

    python tools/hoqp_dump.py [distinct] [out.npz]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def main():
    nd = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/hqpar/gpu.npz"
    from bench_hoqp import SEED0
    from legged_mpc_control_amd import hoqp as HQ
    from legged_mpc_control_amd import wbc as W

    chains = [W.synth_wbc_tasks(SEED0 + i) for i in range(nd)]
    dims = HQ.dims_of(chains[0])
    rec = np.ascontiguousarray(np.stack([HQ.pack(c, dims) for c in chains]))
    x, w, st, it = HQ.HoqpBatch(dims, nd).solve(rec)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez(out, x=x, w=w, st=st, it=it, seed0=SEED0)
    print("saved", out, x.shape, "status", np.bincount(st, minlength=3).tolist(), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Dev tool (GPU): the WBC chains of tools/bench_hoqp.py's batch that do not certify (status != 0), with their
per-level interior-point iterations and crossover outcome, with and without the crossover."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_mpc_control_amd import hoqp as HQ  # noqa: E402
from legged_mpc_control_amd import wbc as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
chains = [W.synth_wbc_tasks(1_000_000 + i) for i in range(n)]
dims = HQ.dims_of(chains[0])
rec = np.stack([HQ.pack(c, dims) for c in chains])
s = HQ.HoqpBatch(dims, n)
for xo in (1, 0):
    s.set_options(crossover=xo)
    x, w, st, it = s.solve(rec)
    bad = np.nonzero(st != 0)[0]
    print(f"crossover={xo}: {len(bad)} of {n} not certified; level-2 max iters {int((it[:, 2] & 0xFFFF).max())}")
    for b in bad[:20]:
        print("  chain", int(b), "status", int(st[b]), "ipm", (it[b] & 0xFFFF).tolist(), "xo", (it[b] >> 16).tolist())
    np.save(f"gpurun_out/hoqp_fail_x{xo}.npy", x)

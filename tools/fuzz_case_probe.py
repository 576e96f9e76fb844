#!/usr/bin/env python3
"""Dev tool (GPU box): re-solve one randomised-sweep case (tools/fuzz_parity.py) with a given library and show its
worst QPs against the oracle.
    python tools/fuzz_case_probe.py LIB ROBOT GAIT H TERRAIN(0/1) PATH SEED [BATCH]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["LMPC_LIB"] = sys.argv[1]
from legged_mpc_control_amd import BatchedConvexQPSolver, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

robot, gait, H, terrain, path, seed = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1", sys.argv[6], int(sys.argv[7])
B = int(sys.argv[8]) if len(sys.argv) > 8 else 1024
p = synth.params(robot)
rec, con = synth.fill(p, synth.synth_cfg(robot, gait), H, B, seed)
nrm = synth.normals(B, seed, theta_max=0.3) if terrain else None
for b in (B, 64):
    g, st, it = BatchedConvexQPSolver(p, H, max_batch=b, dense_path=path).solve(rec[:b], con[:b], normals=None if nrm is None else nrm[:b])
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec[:b], con[:b], n_threads=16, normals=None if nrm is None else nrm[:b])
    err = np.max(np.abs(g - ref).reshape(b, -1) / np.maximum(1.0, np.abs(ref).reshape(b, -1)), axis=1)
    o = np.argsort(-err)
    print(f"{os.path.basename(sys.argv[1])} batch {b}: max {err.max():.3e}; worst QPs:",
          ", ".join(f"{q} ({err[q]:.2e}, ipm {it[q] & 0xFFFF} rounds {it[q] >> 16}, st {st[q]})" for q in o[:4]))

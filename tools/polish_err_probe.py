#!/usr/bin/env python3
"""Dev tool (GPU box): per-QP GRF error of the dense path against the exact oracle, for one library build.

    python tools/polish_err_probe.py LIB OUT.npy [count] [first]   (one process per library)
    python tools/polish_err_probe.py cmp A.npy B.npy [...]

Round 6: the bordered range-space polish rounds raised config 2's full-batch error from 1.2e-10
to 1.8e-9; this finds which QPs carry it and whether a build (refinement, no bordered rounds) removes it.  Saves
[err, abs_err, iteration word, status] per QP.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] != "cmp":
    os.environ["LMPC_LIB"] = sys.argv[1]
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from oracle import oracle as O

    cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    first = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    p, H, rec, con = synth.config_batch(2, count=cnt, first_index=first)
    g, st, it = BatchedConvexQPSolver(p, H, max_batch=cnt, dense_path="ipm").solve(rec, con)
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=16)
    dif = np.abs(g - ref).reshape(cnt, -1)
    rel = np.max(dif / np.maximum(1.0, np.abs(ref).reshape(cnt, -1)), axis=1)
    ab = np.max(dif, axis=1)
    np.save(sys.argv[2], np.stack([rel, ab, it.astype(np.float64), st.astype(np.float64)]))
    o = np.argsort(-rel)
    print(f"{os.path.basename(sys.argv[1])}: max rel {rel.max():.3e} p99 {np.percentile(rel, 99):.3e} "
          f"median {np.median(rel):.3e}; > 2e-10: {(rel > 2e-10).sum()} QPs; status != 0: {(st != 0).sum()}")
    for q in o[:8]:
        print(f"  qp {q}: rel {rel[q]:.3e} abs {ab[q]:.3e} ipm {it[q] & 0xFFFF} rounds {it[q] >> 16}")
else:
    arrs = [np.load(f) for f in sys.argv[2:]]
    for f, a in zip(sys.argv[2:], arrs):
        rel, it = a[0], a[2].astype(np.int64)
        print(f"{os.path.basename(f)}: max {rel.max():.3e} p99 {np.percentile(rel, 99):.3e} >2e-10 {(rel > 2e-10).sum()} "
              f"ipm {np.mean(it & 0xFFFF):.3f} rounds {np.mean(it >> 16):.3f}")
    if len(arrs) >= 2:
        a, b = arrs[0], arrs[1]
        d = np.nonzero(a[2] != b[2])[0]
        print(f"iteration words differ on {len(d)} QPs")

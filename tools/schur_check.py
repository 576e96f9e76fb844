#!/usr/bin/env python3
"""Dev tool (GPU box): iteration words of the dense path with and without range-space polish rounds, per QP.
    python tools/schur_check.py LIB OUT.npy [count] [first]   (one process per library)
    python tools/schur_check.py cmp A.npy B.npy"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if sys.argv[1] != "cmp":
    os.environ["LMPC_LIB"] = sys.argv[1]
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    first = int(sys.argv[4]) if len(sys.argv) > 4 else 777
    p, H, rec, con = synth.config_batch(2, count=cnt, first_index=first)
    g, st, it = BatchedConvexQPSolver(p, H, max_batch=cnt, dense_path="ipm").solve(rec, con)
    np.save(sys.argv[2], np.stack([it.astype(np.int64), st.astype(np.int64)]))
else:
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    ia, ib = a[0], b[0]
    d = np.nonzero(ia != ib)[0]
    print(f"{len(d)} QPs differ; ipm mean {np.mean(ia & 0xFFFF):.2f} vs {np.mean(ib & 0xFFFF):.2f}, rounds mean "
          f"{np.mean(ia >> 16):.2f} vs {np.mean(ib >> 16):.2f}, max ipm {np.max(ia & 0xFFFF)} vs {np.max(ib & 0xFFFF)}")
    for q in d[:20]:
        print(q, (ia[q] & 0xFFFF, ia[q] >> 16), (ib[q] & 0xFFFF, ib[q] >> 16), a[1][q], b[1][q])

#!/usr/bin/env python3
"""Dev tool (GPU box): what the refinement of a verified range-space polish round changes, per QP (round 6).

    LMPC_LIB=tools/build/liblmpc_refinediag.so python tools/refine_diag.py [windows] [--out OUT.json]

The -DLMPC_REFINE_DIAG build records, for every QP whose last (verified) polish round was a range-space update,
the certificate's stationarity residual / gscale, K's smallest pivot ratio |d_c| / |K_cc|, the largest force
correction the refinement made and whether the refined forces were certified again.  Beside it, the QP's GRF error
against the exact oracle.  Used to choose which QPs need the refinement (it costs ~3 % of config 2 on every QP).
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    windows = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 4
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from legged_mpc_control_amd import _native as N
    from oracle import oracle as O

    L = N.lib()
    L.lmpc_debug_refine.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    L.lmpc_debug_refine.restype = ctypes.c_int
    L.lmpc_debug_refine_clear.restype = ctypes.c_int
    rows = []
    for w in range(windows):
        cnt, first = 1024, 1024 * w
        p, H, rec, con = synth.config_batch(2, count=cnt, first_index=first)
        assert L.lmpc_debug_refine_clear() == 0
        g, st, it = BatchedConvexQPSolver(p, H, max_batch=cnt, dense_path="ipm").solve(rec, con)
        dg = np.zeros((cnt, 4))
        assert L.lmpc_debug_refine(dg.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), cnt) == cnt
        ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=16)
        err = np.max(np.abs(g - ref).reshape(cnt, -1) / np.maximum(1.0, np.abs(ref).reshape(cnt, -1)), axis=1)
        for q in range(cnt):
            if dg[q, 3] != 0.0:
                rows.append([first + q, err[q], *dg[q].tolist(), int(it[q] & 0xFFFF), int(it[q] >> 16)])
    a = np.array(rows)
    print(f"{len(a)} QPs ended on a range-space round over {windows} x 1024; rejected refinements: {(a[:, 5] == 2).sum()}")
    print("  err after refinement: max %.3e" % a[:, 1].max())
    for name, col in (("sr/gscale", 2), ("kmin", 3), ("max |du|", 4)):
        v = a[:, col]
        print(f"  {name}: median {np.median(v):.3e} p90 {np.percentile(v, 90):.3e} p99 {np.percentile(v, 99):.3e} "
              f"max {v.max():.3e} min {v.min():.3e}")
    o = np.argsort(-a[:, 4])
    print("  largest corrections: qp, err, sr/gscale, kmin, |du|, ok, ipm, rounds")
    for r in a[o[:15]]:
        print("   ", int(r[0]), " ".join("%.3e" % x for x in r[1:5]), int(r[5]), int(r[6]), int(r[7]))
    for thr in (1e-13, 1e-12, 1e-11, 1e-10):
        sel = a[:, 4] > thr
        print(f"  |du| > {thr:.0e}: {sel.sum()} QPs; their sr/gscale min {a[sel, 2].min() if sel.any() else 0:.3e}, "
              f"kmin max {a[sel, 3].max() if sel.any() else 0:.3e}")
    if out:
        json.dump({"rows": a.tolist(), "cols": ["qp", "err", "sr_over_gscale", "kmin", "max_du", "ok", "ipm", "rounds"]},
                  open(out, "w"))


if __name__ == "__main__":
    main()

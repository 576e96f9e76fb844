#!/usr/bin/env python3
"""Dev tool (GPU box, LMPC_LIB=tools/build/liblmpc_kktdiag.so): QPs a workload leaves unverified, with the
certificate residuals each kernel recorded for them (tools/kkt_diag.py's arrays) and their error against the oracle."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import torch

    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from legged_mpc_control_amd import _native as N
    from oracle import oracle as O

    L = N.lib()
    for fn in ("lmpc_debug_kkt_lq", "lmpc_debug_kkt_dense"):
        getattr(L, fn).argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    cases = [(4, "ipm", False), (4, "off", False), (4, "gi", False), (4, "ipm", True), (3, "ipm", False), (5, "ipm", False)]
    for cid, dense, terrain in cases:
        L.lmpc_debug_kkt_lq_clear()
        L.lmpc_debug_kkt_dense_clear()
        p, H, rec, con = synth.config_batch(cid)
        B = rec.shape[0]
        nrm = synth.config_normals(cid, B) if terrain else None
        s = BatchedConvexQPSolver(p, H, max_batch=B, dense_path=dense)
        g, st, it = s.solve(rec, con, normals=nrm)
        bad = np.nonzero(st != 0)[0]
        print(f"config {cid} dense {dense} terrain {terrain}: status {np.bincount(st, minlength=3)}", flush=True)
        if len(bad) == 0:
            continue
        lq = np.zeros((B, 4)); dn = np.zeros((B, 4))
        L.lmpc_debug_kkt_lq(lq.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), B)
        L.lmpc_debug_kkt_dense(dn.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), B)
        ref, _, _ = O.solve_batch(O.params_from(p), H, rec[bad], con[bad], n_threads=8,
                                  normals=None if nrm is None else nrm[bad])
        for i, b in enumerate(bad[:20]):
            err = float(np.max(np.abs(g[b] - ref[i]) / np.maximum(1.0, np.abs(ref[i]))))
            print(f"  qp {b}: status {st[b]} iters {it[b] & 0xFFFF} rounds {it[b] >> 16} stance {int(con[b].sum())} "
                  f"err {err:.3g} lq[sr/g, dyn/x, gscale, rounds] {lq[b]} dense[sr/g, -, gscale] {dn[b, :3]}", flush=True)


if __name__ == "__main__":
    main()

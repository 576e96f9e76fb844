#!/usr/bin/env python3
"""Dev tool (GPU box): the flat config-4 QPs the round-5 certificate first rejected (26307, 64455), solved by the
round-4 library (tools/build/liblmpc_r4.so) and by the product, against the oracle; then the whole flat config-4
batch on the product (status counts, max error on a sample)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402


def main():
    import test_gpu_kkt as T
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from oracle import oracle as O

    p, H, rec, con = synth.config_batch(4)
    idx = np.array([26307, 64455])
    ref, _, _ = O.solve_batch(O.params_from(p), H, rec[idx], con[idx], n_threads=8)
    L4 = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "liblmpc_r4.so"))
    vp = ctypes.c_void_p
    from legged_mpc_control_amd import _native as N
    L4.lmpc_create.argtypes = [ctypes.POINTER(N.LmpcParams), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
    L4.lmpc_set_dense_path.argtypes = [vp, ctypes.c_int]
    dp, i32p, u8p = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint8)
    L4.lmpc_solve_batch_ex.argtypes = [vp, dp, u8p, dp, ctypes.c_int, dp, i32p, i32p]
    L4.lmpc_destroy.argtypes = [vp]
    L4.lmpc_destroy.restype = None
    g4, s4, i4 = T._solve_with(L4, p, H, rec[idx], con[idx])
    s = BatchedConvexQPSolver(p, H, max_batch=len(idx), dense_path="off")
    g5, s5, i5 = s.solve(rec[idx], con[idx])
    for k, b in enumerate(idx):
        e4 = float(np.max(np.abs(g4[k] - ref[k]) / np.maximum(1, np.abs(ref[k]))))
        e5 = float(np.max(np.abs(g5[k] - ref[k]) / np.maximum(1, np.abs(ref[k]))))
        print(f"qp {b}: round 4 status {s4[k]} rounds {i4[k] >> 16} err {e4:.3g} | round 5 status {s5[k]} "
              f"rounds {i5[k] >> 16} err {e5:.3g}", flush=True)
    for dense in ("off", "ipm"):
        s = BatchedConvexQPSolver(p, H, max_batch=rec.shape[0], dense_path=dense)
        g, st, it = s.solve(rec, con)
        smp = np.random.default_rng(3).choice(rec.shape[0], 2048, replace=False)
        smp = np.union1d(smp, idx)
        r, _, _ = O.solve_batch(O.params_from(p), H, rec[smp], con[smp], n_threads=8)
        e = float(np.max(np.abs(g[smp] - r) / np.maximum(1, np.abs(r))))
        print(f"flat config 4, dense {dense}: status {np.bincount(st, minlength=3)}, polish rounds max {np.max(it >> 16)},"
              f" max err over {len(smp)} sampled QPs {e:.3g}", flush=True)


if __name__ == "__main__":
    main()

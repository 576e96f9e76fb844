#!/usr/bin/env python3
"""Dev tool (GPU box): how far the polish's KKT certificate sits from its tolerances on real batches.

    LMPC_LIB=tools/build/liblmpc_kktdiag.so python tools/kkt_diag.py [--out gpurun_out/kkt_diag.json]

The -DLMPC_KKT_DIAG build records, per QP, at its last settled polish round: the stationarity residual on the stance
leg-steps' free directions / gscale (lmpc_kernel_common.h leg_kkt) and, for the LDS Riccati kernel, the dynamics
residual of the trajectory / the state scale.  The product accepts a settled active set when these are within tol_d
and tol_p (1e-9 each); this prints their distribution on the bench workloads (configs 2/2off/2gi/3/4/5 and the
committed goldens), so the margin between rounding level and the tolerance is measured, not assumed.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def stats(v):
    v = np.asarray(v, dtype=np.float64)
    if v.size == 0:
        return None
    return {"n": int(v.size), "median": float(np.median(v)), "p99": float(np.percentile(v, 99)),
            "max": float(np.max(v))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from legged_mpc_control_amd import _native as N

    L = N.lib()
    for fn in ("lmpc_debug_kkt_lq", "lmpc_debug_kkt_dense", "lmpc_debug_kkt_gi"):
        getattr(L, fn).argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        getattr(L, fn).restype = ctypes.c_int
    L.lmpc_debug_kkt_lq_clear.restype = ctypes.c_int
    L.lmpc_debug_kkt_dense_clear.restype = ctypes.c_int

    def dump(fn, n):
        a = np.zeros((n, 4))
        assert getattr(L, fn)(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n) == n
        return a

    dev = torch.device("cuda", 0)
    out = {}
    cases = [(2, "ipm"), (2, "off"), (2, "gi"), (3, None), (4, "off"), (5, None)]
    for cfg_id, dense in cases:
        cfg = synth.CONFIGS[cfg_id]
        H, B = cfg["H"], cfg["batch"]
        p = synth.params(cfg["robot"])
        solver = BatchedConvexQPSolver(p, H, max_batch=0, dense_path=dense or "ipm")
        seed = synth.BASE_SEED + cfg_id
        cmd = solver.synth_commands_device(synth.config_cfg(cfg_id), B, seed, device=dev)
        nrm = solver.synth_normals_device(B, seed, device=dev) if cfg_id == 4 else None
        rec, con = solver.build_records_device(cmd)
        grf = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
        st = torch.empty(B, dtype=torch.int32, device=dev)
        it = torch.empty(B, dtype=torch.int32, device=dev)
        L.lmpc_debug_kkt_lq_clear()
        L.lmpc_debug_kkt_dense_clear()
        solver.solve_device(rec, con, grf, st, it, normals=nrm)
        torch.cuda.synchronize()
        n = min(B, 65536)
        st = st.cpu().numpy()
        key = f"config{cfg_id}" + (f"/{dense}" if dense else "")
        row = {"status": {str(k): int((st == k).sum()) for k in (0, 1, 2)}}
        lq = dump("lmpc_debug_kkt_lq", n)
        used = lq[:, 2] > 0  # gscale >= 1 where the LQ kernel verified a settled set
        if used.any():
            row["lq_stationarity_over_gscale"] = stats(lq[used, 0])
            row["lq_dynamics_over_xscale"] = stats(lq[used, 1])
            row["lq_gscale"] = stats(lq[used, 2])
        if dense == "ipm":
            dn = dump("lmpc_debug_kkt_dense", n)
            used = dn[:, 2] > 0
            row["dense_stationarity_over_gscale"] = stats(dn[used, 0])
            row["dense_gscale"] = stats(dn[used, 2])
        if dense == "gi":
            gi = dump("lmpc_debug_kkt_gi", n)
            used = gi[:, 2] > 0
            row["gi_stationarity_over_gscale"] = stats(gi[used, 0])
            row["gi_failed"] = int((gi[used, 1] > 0).sum())
        out[key] = row
        print(key, json.dumps(row), flush=True)
        solver.close()
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()

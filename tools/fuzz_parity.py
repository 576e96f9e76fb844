#!/usr/bin/env python3
"""Randomised parity sweep (GPU box): many seeded batches over robots, gaits (trot / crawl / trot-with-stand / stand /
mixed), horizons 2..32, flat ground and tilted terrain, and all three dense-path settings (interior point, dual
active set, Riccati only), every QP compared with the exact oracle (oracle/, the checker, on the host threads).

    python tools/fuzz_parity.py [--seconds S] [--batch B] [--out FILE]

Prints one JSON summary: per case the batch, status counts, max relative GRF error (|f - f*| / max(1, |f*|)) and
the largest primal violation of the friction pyramid / bounds; overall maxima.  Parity bar: 1e-4 (north star)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90.0)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch

    torch.cuda.init()
    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from legged_mpc_control_amd import _native as N
    from oracle import oracle as O

    threads = min(16, os.cpu_count() or 1)
    try:
        threads = min(threads, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    rng = np.random.default_rng(20261017)
    gaits = [N.GAIT_TROT, 1, 2, 3, -1]  # trot, crawl, trot-with-stand, stand, mixed (synth.synth_cfg gait ids)
    paths = ["ipm", "gi", "off"]
    cases = []
    worst = {"err": 0.0, "viol": 0.0, "nonconverged": 0}
    t0 = time.perf_counter()
    solvers = {}
    while time.perf_counter() - t0 < args.seconds:
        robot = str(rng.choice(["go1", "a1"]))
        gait = int(rng.choice(gaits))
        H = int(rng.integers(2, 33))
        terrain = bool(rng.random() < 0.4)
        path = str(rng.choice(paths))
        seed = int(rng.integers(1, 2**31))
        B = args.batch
        p = synth.params(robot)
        rec, con = synth.fill(p, synth.synth_cfg(robot, gait), H, B, seed)
        nrm = synth.normals(B, seed, theta_max=0.3) if terrain else None
        key = (robot, H, path)
        if key not in solvers:
            solvers[key] = BatchedConvexQPSolver(p, H, max_batch=B, dense_path=path)
        s = solvers[key]
        grf, st, it = s.solve(rec, con, normals=nrm)
        ref, _, fails = O.solve_batch(O.params_from(p), H, rec, con, n_threads=threads, normals=nrm)
        err = float(np.max(np.abs(grf - ref) / np.maximum(1.0, np.abs(ref))))
        # primal feasibility of the GPU answer in the contact frame: |gx|, |gy| <= mu gz, 0 <= gz <= f_max c
        g = grf.reshape(B, H, 4, 3)
        if nrm is not None:
            R = np.stack([synth.terrain_frame(n) for n in nrm.reshape(-1, 3)]).reshape(B, 1, 4, 3, 3)
            g = np.einsum("bhlji,bhlj->bhli", np.broadcast_to(R, (B, H, 4, 3, 3)), g)
        c = con.astype(np.float64)
        viol = float(np.max(np.concatenate([
            (np.abs(g[..., 0]) - p.mu * g[..., 2]).ravel(), (np.abs(g[..., 1]) - p.mu * g[..., 2]).ravel(),
            (-g[..., 2]).ravel(), (g[..., 2] - p.f_max * c).ravel()])))
        nc = int(np.sum(st != 0))
        cases.append({"robot": robot, "gait": gait, "H": H, "terrain": terrain, "dense_path": s.dense_path, "seed": seed,
                      "batch": B, "status": np.bincount(st, minlength=3).tolist(), "oracle_fails": int(fails),
                      "max_rel_err": err, "max_violation_N": viol})
        worst["err"] = max(worst["err"], err)
        worst["viol"] = max(worst["viol"], viol)
        worst["nonconverged"] += nc
        print(f"{robot} gait {gait:2d} H {H:2d} terrain {int(terrain)} {s.dense_path:3s}: status {cases[-1]['status']} "
              f"err {err:.1e} viol {viol:.1e}", flush=True)
    summary = {"cases": len(cases), "qps": sum(c["batch"] for c in cases), "max_rel_err": worst["err"],
               "max_violation_N": worst["viol"], "non_converged": worst["nonconverged"], "oracle_threads": threads,
               "bar": 1e-4, "detail": cases}
    line = json.dumps(summary)
    if args.out:
        open(args.out, "w").write(line + "\n")
    print(json.dumps({k: v for k, v in summary.items() if k != "detail"}), flush=True)


if __name__ == "__main__":
    main()

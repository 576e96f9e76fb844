#!/usr/bin/env python3
"""Benchmark of the batched hierarchical QP (whole-body control) on MI355X.

    python tools/bench_hoqp.py [--gpus N] [--steps K] [--warmup W] [--batch B]

One step = one launch of lmpc_hoqp_kernel over B WBC-shaped hierarchies already resident in HBM (3 levels,
42 variables: legged_mpc_control_amd/wbc.py on synthetic Go1-scale dynamics; the reference solves one per
control tick with three qpOASES QProblems, wbc.cpp:93-99).  For N > 1 (torch.distributed.run, one rank per
GPU) every rank solves its own shard of global indices: independent instances, no collective (weak scaling).
Rank 0 prints ONE JSON line in bench.py's format: roofline of the kernel (HIP events on the launch stream),
parity of a seeded sample against the CPU restatement (oracle/hoqp.py), and at N = 1 that restatement timed
on a bounded sample as the CPU baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

SEED0 = 1_000_000  # synthetic WBC instances: global index i uses wbc.synth_wbc(SEED0 + i)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="hierarchies per GPU")
    ap.add_argument("--distinct", type=int, default=1024, help="distinct synthetic instances, tiled to the batch")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--parity-sample", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tol-mu", type=float, default=None, help="interior-point stop (lmpc_hoqp_options.tol_mu; A/B)")
    ap.add_argument("--crossover", type=int, default=1, choices=(0, 1),
                    help="lmpc_hoqp_options.crossover (exact active-set step after each level's interior point)")
    return ap.parse_args()


def null_dims(chain):
    """(nd, rank) per level: nd_{l+1} = nd_l - rank(A_l Z_l) (basis-independent), for the flop model."""
    n = chain[0].num_vars()
    Z = np.eye(n)
    out = []
    for t in chain:
        nd = Z.shape[1]
        if t.a.shape[0]:
            G = t.a @ Z
            r = int(np.linalg.matrix_rank(G))
            out.append((nd, r))
            _, _, vt = np.linalg.svd(G)
            Z = Z @ vt[r:].T if r < nd else np.zeros((n, 1))
        else:
            out.append((nd, 0))
    return out


def main():
    args = parse()
    import torch

    from legged_mpc_control_amd import dist as D
    from legged_mpc_control_amd import hoqp as HQ
    from legged_mpc_control_amd import roofline
    from legged_mpc_control_amd import wbc as W

    rank, world, local_rank = D.env_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    torch.cuda.init()
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("LMPC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    B = args.batch
    first = rank * B
    nd = min(args.distinct, B)
    chains = [W.synth_wbc_tasks(SEED0 + first + i) for i in range(nd)]
    dims = HQ.dims_of(chains[0])
    base = np.stack([HQ.pack(c, dims) for c in chains])
    rec = np.ascontiguousarray(np.resize(base, (B, base.shape[1])))
    solver = HQ.HoqpBatch(dims, B, local_rank)
    solver.set_options(crossover=args.crossover, tol_mu=args.tol_mu)
    d_rec = torch.from_numpy(rec).to(dev)
    d_x = torch.empty((B, dims.num_levels, dims.num_vars), dtype=torch.float64, device=dev)
    d_w = torch.empty((B, max(solver.slack_len, 1)), dtype=torch.float64, device=dev)
    d_st = torch.empty(B, dtype=torch.int32, device=dev)
    d_it = torch.empty((B, dims.num_levels), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # as bench.py (round 6): W warm-up steps and at least 30 ms of device time (the clock ramp), then one HIP event
    # pair around the K timed launches
    warm_run, tw = 0, time.perf_counter()
    while warm_run < args.warmup or time.perf_counter() - tw < 0.03:
        solver.solve_device(d_rec, d_x, d_w, d_st, d_it, stream)
        warm_run += 1
        torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        solver.solve_device(d_rec, d_x, d_w, d_st, d_it, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    t_max = D.max_over_ranks(time.perf_counter() - t0, dist, dev)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    x = d_x.cpu().numpy()
    w = d_w.cpu().numpy()[:, :solver.slack_len]
    st = d_st.cpu().numpy()
    it_word = d_it.cpu().numpy()
    it = it_word & 0xFFFF          # interior-point iterations; bits 16-17: crossover tried (1) / verified (3)
    xo = it_word >> 16
    # work model: measured iterations per level, null-space dimensions from the instances themselves
    nds = [null_dims(c) for c in chains[:128]]
    flop = 0.0
    for b in range(len(nds)):
        p = 0
        for l in range(dims.num_levels):
            ndl, rk = nds[b][l]
            flop += roofline.hoqp_level_flop(dims.num_vars, dims.eq_rows[l], dims.ineq_rows[l], p, ndl, rk,
                                             float(it[b, l]))
            p += dims.ineq_rows[l]
    flop_per = flop / len(nds)
    achieved_tf = flop_per * B / (kernel_ms * 1e-3) / 1e12
    bytes_per = roofline.hoqp_bytes(dims.num_vars, list(dims.eq_rows[:dims.num_levels]),
                                    list(dims.ineq_rows[:dims.num_levels]))

    # parity: a seeded sample of this rank's instances against the CPU restatement (the checker)
    from oracle import hoqp as Q

    rng = np.random.default_rng(7 + rank)
    idx = rng.choice(min(nd, B), min(args.parity_sample, nd), replace=False)
    err_x = err_w = err_ax = 0.0
    for b in idx:
        lv = []
        for t in chains[b]:
            lv.append(Q.HoQp(Q.Task(t.a, t.b, t.d, t.f), lv[-1] if lv else None))
        xr = lv[-1].solution()
        err_x = max(err_x, float(np.max(np.abs(x[b, -1] - xr)) / (1 + np.max(np.abs(xr)))))
        err_w = max(err_w, float(np.max(np.abs(w[b] - lv[-1].stacked_slack))))
        for l, t in enumerate(chains[b]):
            err_ax = max(err_ax, float(np.max(np.abs(t.a @ (x[b, l] - lv[l].solution())))))
    err_x = D.max_over_ranks(err_x, dist, dev)
    err_w = D.max_over_ranks(err_w, dist, dev)
    stats = D.sum_over_ranks([(st == 0).sum(), (st == 1).sum(), (st == 2).sum()], dist, dev)

    traffic = None  # HBM bytes per launch from the committed PMC passes (tools/profile_hoqp.sh)
    try:
        tr = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))["wbc_hoqp_3level_n42"]
        traffic = tr["bytes_per_qp"] * B
    except (OSError, ValueError, KeyError):
        traffic = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        t1 = time.perf_counter()
        done = 0
        while time.perf_counter() - t1 < args.cpu_seconds:
            c = chains[done % nd]
            lv = []
            for t in c:
                lv.append(Q.HoQp(Q.Task(t.a, t.b, t.d, t.f), lv[-1] if lv else None))
            done += 1
        ct = time.perf_counter() - t1
        cpu = {"value": done / ct, "unit": "hierarchies/s", "cores": 1, "kind": "port",
               "sample": f"{done} WBC hierarchies, oracle/hoqp.py (numpy, exact primal active set in x87 "
                         f"extended precision, one thread; qpOASES itself is absent), {ct:.1f} s wall"}

    if rank == 0:
        line = {
            "metric": "hierarchical QP solves/sec (WBC: 3 levels, 42 variables); max err vs CPU restatement",
            "value": B * world * args.steps / t_max,
            "unit": "hierarchies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_run,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (wbc.synth_wbc: Go1-scale SPD mass matrix, foot Jacobians, random gaits; "
                    f"{nd} distinct per rank, tiled)",
            "config": {"workload": "wbc_hoqp_3level_n42", "batch_per_gpu": B, "global_batch": B * world,
                       "levels": [[dims.eq_rows[l], dims.ineq_rows[l]] for l in range(dims.num_levels)],
                       "crossover": args.crossover,
                       "parallelism": f"dp{world} (independent hierarchies, no collective)"},
            "roofline": {
                "bound": "mfma",
                "achieved": achieved_tf,
                "peak": roofline.FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / roofline.FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "kernel": "lmpc_hoqp_kernel",
                "kernel_ms": kernel_ms,
                "flop_per_instance": flop_per,
                "flop_model": "roofline.hoqp_level_flop per level, measured iterations, nd/rank of the instances",
                "bytes_per_instance": bytes_per,
                "hbm_gbs": bytes_per * B / (kernel_ms * 1e-3) / 1e9,
            },
            "cpu_baseline": cpu,
            "parity": {"vs": "oracle/hoqp.py (exact active set, Eigen FullPivLU basis)", "sample": int(len(idx)),
                       "final_x_rel_err": err_x, "slack_abs_err": err_w, "level_Ax_abs_err": err_ax},
            "status": {"converged": int(stats[0]), "max_iter": int(stats[1]), "nan": int(stats[2])},
            "ipm_iters_per_level_mean": [float(v) for v in it.mean(axis=0)],
            "ipm_iters_per_level_max": [int(v) for v in it.max(axis=0)],
            "crossover_verified_per_level": [float(v) for v in (xo == 3).mean(axis=0)],
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: batched convex-MPC GRF QP solves/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2] [--batch B]

One step = one fused-kernel pass over one batch of synthetic QPs already
resident in HBM (config 2 by default: Go1 trot, horizon 10, 1024 QPs per GPU).
For N > 1 (launched by torch.distributed.run, one rank per GPU) each rank
builds and solves its own shard of global indices [rank*B, (rank+1)*B): no
data-path collective (independent QPs, weak scaling).  Rank 0 prints ONE JSON
line with the roofline of the dominant kernel (HIP events on the launch stream),
the max GRF error against the CPU oracle (N=1: every QP of the batch; N>1: a
seeded sample of every rank's shard, max over ranks) and, at N=1, the CPU
oracle timed on the host cores over the same instances.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--warmup-ms", type=float, default=30.0,
                    help="keep warming up (after --warmup steps) until the device has run this long (clock ramp)")
    ap.add_argument("--config", type=int, default=2, help="BASELINE.json config id (2,3,4,5)")
    ap.add_argument("--batch", type=int, default=None, help="QPs per GPU (default: config batch; config 4: 65536/N)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (wall seconds)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--flat", action="store_true", help="config 4 without its terrain normals (reference problem)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the second timed pass that also gathers all GRFs to rank 0")
    ap.add_argument("--dense", choices=["ipm", "gi", "off"], default=None,
                    help="dense-path kernel (lmpc_set_dense_path); default ipm, config 4: off")
    ap.add_argument("--riccati", choices=["lds", "scratch"], default="lds",
                    help="Riccati kernel of the QPs no dense kernel takes (lmpc_set_riccati_path); default lds")
    ap.add_argument("--index-offset", type=int, default=0,
                    help="shift the global instance indices (robustness checks on other samples; recorded in config)")
    ap.add_argument("--opt", action="append", default=[], metavar="FIELD=VALUE",
                    help="set an lmpc_options field for this run (A/B of solver settings; the line records it)")
    return ap.parse_args()


def host_cores():
    """Host CPUs this process may run on: the affinity set, bounded by the cgroup CPU quota when one is set
    (os.cpu_count() reports every CPU of the machine, also those a container's quota does not grant)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = total
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        quota = None
    usable = min(aff, quota) if quota else aff
    return usable, {"os_cpu_count": total, "affinity": aff, "cgroup_quota_cpus": quota}


def kernel_label(mode, riccati="lds", fused=False):
    """The kernels of one solve launch (lmpc_capi.cpp lmpc_solve_batch_device_ex); kernel_ms covers all."""
    ric = "lmpc_lq_kernel" if riccati == "lds" else "lmpc_qp_kernel"
    if mode == "off":
        return f"{ric} (Riccati, every QP)"
    if fused:
        return ("lmpc_dense_lq_kernel (one launch: the dense interior point for QPs with <= 20 stance leg-steps, "
                "the lone-wave Riccati solve in the same wave for the rest)")
    dense = "lmpc_gi_kernel" if mode == "gi" else "lmpc_dense_kernel"
    return f"{dense} (QPs with <= 20 stance leg-steps) + {ric} (the rest; exits at once when none)"


def global_batch_of(strong, cfg, B, world):
    return cfg["batch"] if strong else B * world


def main():
    args = parse()
    import torch

    from legged_mpc_control_amd import BatchedConvexQPSolver, roofline, synth
    from legged_mpc_control_amd import dist as D

    rank, world, local_rank = D.env_rank()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one GPU per rank on a node (LOCAL_RANK < device count); the modulo only matters when rehearsing
    # several ranks on fewer GPUs (a 1-GPU box), where it never changes what a rank computes
    local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        # RCCL (the product path); LMPC_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU, which RCCL
        # refuses ("duplicate GPU")
        backend = os.environ.get("LMPC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    cfg = synth.CONFIGS[args.config]
    H = cfg["H"]
    strong = args.batch is None and args.config == 4  # config 4: a fixed global batch split over the ranks
    if strong:
        first, last = D.split_range(rank, world, cfg["batch"])
        B = last - first
    else:
        B = args.batch if args.batch is not None else cfg["batch"]
        first, _ = D.shard_range(rank, world, B)
    first += args.index_offset
    p = synth.params(cfg["robot"])
    terrain = args.config == 4 and not args.flat  # config 4: terrain normals
    wl_name = cfg["name"] + ("+terrain" if terrain else "")

    # Inputs are generated ON THE DEVICE from (seed, global index): every rank builds its own shard in
    # HBM, no input bytes cross PCIe or xGMI.  Commands -> records + contact schedules
    # by the expansion kernel (8f-1); the timed step below is the QP solve over those records.
    # Dense-path kernel: the interior point where the batch is small enough that the Riccati kernel
    # runs one wave per SIMD (config 2: 0.18 ms against 0.31 ms on the Riccati kernel alone); config 4's 65536 QPs
    # go to the Riccati kernel alone, whose two-wave instance solves its trot QPs faster than the dense kernel's
    # one wave per SIMD does (round 4, DESIGN.md 4d: 9.8 ms against 10.5 ms split).  Fixed per context, so no
    # answer depends on the batch or the shard; --dense overrides it.
    default_dense = "off" if args.config == 4 else "ipm"
    dense = args.dense or default_dense
    solver = BatchedConvexQPSolver(p, H, max_batch=0, device=local_rank, dense_path=dense, riccati_path=args.riccati)
    opts = {}
    for kv in args.opt:
        k, v = kv.split("=", 1)
        opts[k] = float(v) if any(ch in v for ch in ".e") else int(v)
    if opts:
        from legged_mpc_control_amd.solver import solver_options
        solver.set_options(solver_options(**opts))
    seed = synth.BASE_SEED + args.config
    d_cmd = solver.synth_commands_device(synth.config_cfg(args.config), B, seed, first_index=first, device=dev)
    d_nrm = solver.synth_normals_device(B, seed, first_index=first, device=dev) if terrain else None
    d_rec, d_con = solver.build_records_device(d_cmd)
    torch.cuda.synchronize(dev)
    del d_cmd
    d_grf = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
    d_st = torch.empty(B, dtype=torch.int32, device=dev)
    d_it = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)  # dedicated launch stream: events below bracket exactly the kernels
    torch.cuda.set_stream(stream)

    # Warm-up: the W steps asked for, then more until the device has been busy for --warmup-ms: the GPU's clocks ramp
    # up over the first ~10-20 ms of sustained load, and a timed region that starts on a cold GPU measures the ramp
    # (config 2 at --warmup 5: 0.171 ms per step, the launches themselves 0.170; after 50 warm-up steps 0.165 / 0.164,
    # tools/r6_steps.sh, profiles/r06/steps/).  The line reports both counts.
    warm_run = 0
    tw = time.perf_counter()
    while warm_run < args.warmup or time.perf_counter() - tw < args.warmup_ms * 1e-3:
        for _ in range(args.warmup if warm_run == 0 and args.warmup > 0 else 4):
            solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream, normals=d_nrm)
            warm_run += 1
        torch.cuda.synchronize(dev)

    # One HIP event pair on the launch stream brackets the K launches of the timed region: kernel_ms = its elapsed
    # time / K, the average launch duration (back-to-back launches leave no measurable gap between them).  Until
    # round 5 every step had its own event pair, and those events cost ~5 us per step of their own: config 2 ran
    # 0.176 ms per step with them against 0.167 without (tools/step_overhead.py, profiles/r06/overhead/).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream, normals=d_nrm)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = D.max_over_ranks(elapsed, dist, dev)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    # N > 1: a second timed pass, solve + grouped point-to-point gather of every rank's GRFs to
    # rank 0 (SURVEY.md 8e "with and without the gather"); reported beside `value`, never as it.
    with_gather = None
    if dist is not None and not args.no_gather:
        if strong:
            counts = [b - a for a, b in (D.split_range(r, world, cfg["batch"]) for r in range(world))]
        else:
            counts = [B] * world
        full = D.gather_to_rank0(d_grf, dist, world, rank, counts)  # warm the p2p channels
        torch.cuda.synchronize(dev)
        if rank == 0:
            assert full.shape[0] == sum(counts) and torch.equal(full[:B], d_grf)
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        for i in range(args.steps):
            solver.solve_device(d_rec, d_con, d_grf, d_st, d_it, stream, normals=d_nrm)
            full = D.gather_to_rank0(d_grf, dist, world, rank, counts)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tg = D.max_over_ranks(time.perf_counter() - tg, dist, dev)
        with_gather = {
            "value": global_batch_of(strong, cfg, B, world) * args.steps / tg,
            "ms_per_step": tg / args.steps * 1e3,
            "gather_bytes": int(sum(counts[1:]) * H * 12 * 8),
            "how": "solve + grouped isend/irecv of all GRFs to rank 0 (batch_isend_irecv over RCCL)",
        }

    grf = d_grf.cpu().numpy()
    st = d_st.cpu().numpy()
    it = d_it.cpu().numpy()
    mode = solver.dense_path  # "ipm" (default), "gi" or "off" (H > 16, or --dense off)
    ipm_mean = float(np.mean(it & 0xFFFF))
    pol_mean = float(np.mean(it >> 16))
    con_host = d_con.cpu().numpy()
    stance_ls = con_host.reshape(B, -1).sum(axis=1)  # stance leg-steps per QP
    dense_qp = (stance_ls >= 1) & (stance_ls <= 20) & (mode != "off")  # the QPs a dense kernel takes (H <= 16)
    # The work model of the formulation each kernel runs:
    #   the condensed dense kernels: SURVEY.md 8(d)'s contract figure (F0 + K F_iter + rounds (N^3/3 + 2N^2), N = 12H),
    #     the headline definition of roofline.achieved, and beside it the same formulas on the condensed dimension the
    #     kernel really solves (N = 3 x stance leg-steps; roofline.dense_flop);
    #   the LDS Riccati kernel: its own useful flops (reduced inputs in the interior point, full / reduced inputs in the
    #     polish; roofline.lq_flop) -- SURVEY's F0 prices a dense N = 12H condensation it never performs (at H = 30 the
    #     contract figure exceeds the fp64 peak), so no contract fraction is printed for it.
    if mode == "gi":  # iteration word = active-set steps | drops << 16 on the dense QPs
        contract_per_qp = roofline.gi_flop(H, ipm_mean)
        flop_model = "SURVEY.md 8(d) F0 + steps * 6 * 64^2 (dual active set; steps = measured mean)"
    else:
        contract_per_qp = roofline.survey_flop(H, ipm_mean, pol_mean)
        flop_model = "SURVEY.md 8(d): F0 + K*F_iter + rounds*(N^3/3 + 2N^2), N = 12H, K/rounds = measured means"
    lq_sel = ~dense_qp
    useful_per_qp = 0.0
    if lq_sel.any():
        il, pl = it[lq_sel] & 0xFFFF, it[lq_sel] >> 16
        useful_per_qp += roofline.lq_flop(H, float(np.mean(il)), float(np.mean(pl)),
                                          float(np.mean(stance_ls[lq_sel])) / H) * lq_sel.sum() / B
    if dense_qp.any():
        idn, pdn = it[dense_qp] & 0xFFFF, it[dense_qp] >> 16
        useful_per_qp += roofline.dense_flop(H, float(np.mean(stance_ls[dense_qp])), float(np.mean(idn)),
                                             float(np.mean(pdn))) * dense_qp.sum() / B
    useful_tf = useful_per_qp * B / (kernel_ms * 1e-3) / 1e12
    headline_contract = mode != "off" and dense_qp.all()  # every QP on a condensed dense kernel (config 2)
    achieved_tf = (contract_per_qp if headline_contract else useful_per_qp) * B / (kernel_ms * 1e-3) / 1e12
    global_batch = global_batch_of(strong, cfg, B, world)
    total_qps = global_batch * args.steps / t_max

    stats = D.sum_over_ranks([(st == 0).sum(), (st == 1).sum(), (st == 2).sum()], dist, dev)

    cpu = None
    max_err = max_abs = None
    from oracle import oracle as O  # the checker: parity of the measured batch, and the CPU baseline

    op = O.params_from(p)
    nrm_all = None if d_nrm is None else d_nrm.cpu().numpy()
    rec_all, con_all = d_rec.cpu().numpy(), d_con.cpu().numpy()  # the very instances the GPU solved
    cores, cpu_info = host_cores()  # every host CPU this process may use (count stated in the line)
    if world == 1 and not args.no_cpu:
        idx = np.arange(B)  # N = 1: every QP of the batch
    else:
        # N > 1 (or no CPU baseline): each rank checks a seeded sample of its own shard; the max goes over ranks
        idx = np.sort(np.random.default_rng(1000 + rank).choice(B, min(B, 64), replace=False))
    ref, _, _ = O.solve_batch(op, H, rec_all[idx], con_all[idx], n_threads=cores,
                              normals=None if nrm_all is None else nrm_all[idx])
    dif = np.abs(grf[idx] - ref)
    max_err = D.max_over_ranks(float(np.max(dif / np.maximum(1.0, np.abs(ref)))), dist, dev)
    max_abs = D.max_over_ranks(float(np.max(dif)), dist, dev)
    parity_checked = D.sum_over_ranks([len(idx)], dist, dev)[0]
    cpu_exact = None
    if rank == 0 and world == 1 and not args.no_cpu:
        rec, con, nrm = rec_all, con_all, nrm_all
        # (1) the reference's own algorithm: OSQP's ADMM at the reference's settings (ConvexQPSolver.cpp:182-194),
        # restated in C on the reference's sparse QP (oracle/osqp_admm.c), over a bounded sample of the batch
        # (whole passes over a prefix of it, ~cpu_seconds of wall time)
        t1 = time.perf_counter()
        probe = min(B, 4 * cores)
        O.osqp_grf_batch(op, H, rec[:probe], con[:probe], n_threads=cores, normals=None if nrm is None else nrm[:probe])
        per_qp = max((time.perf_counter() - t1) / probe, 1e-6)
        ns = int(min(B, max(probe, args.cpu_seconds / per_qp)))
        t1 = time.perf_counter()
        g_admm, it_admm, cv_admm = O.osqp_grf_batch(op, H, rec[:ns], con[:ns], n_threads=cores,
                                                    normals=None if nrm is None else nrm[:ns])
        reps, done_qps = 1, ns
        while time.perf_counter() - t1 < args.cpu_seconds:
            O.osqp_grf_batch(op, H, rec[:ns], con[:ns], n_threads=cores, normals=None if nrm is None else nrm[:ns])
            reps += 1
            done_qps += ns
        ct = time.perf_counter() - t1
        du0 = np.max(np.abs(g_admm[:, 0, :] - ref[:ns, 0, :]), axis=1)
        cpu = {
            "value": done_qps / ct,
            "unit": "QP/s",
            "cores": cores,
            "kind": "port",
            "algorithm": "reference-algorithm restatement: OSQP ADMM (rho 0.1, sigma 1e-6, alpha 1.6, eps_abs 1e-3, "
                         "eps_rel 1e-4, Ruiz scaling, adaptive rho) on the reference's sparse QP, in C "
                         "(oracle/osqp_admm.c); OSQP itself is not in the image",
            "sample": f"{reps} x the first {ns} QPs of the rank-0 batch ({wl_name}) over {cores} host threads, "
                      f"{ct:.1f} s wall",
            "admm_iters_mean": float(np.mean(it_admm)),
            "admm_converged": int(np.sum(cv_admm)),
            "max_abs_dev_from_exact_optimum_N": float(np.max(np.abs(g_admm - ref[:ns]))) if world == 1 else None,
            # what the reference's tick consumes: u0 only (ConvexQPSolver.cpp:320-322) -- per QP max |du0| over its 12
            # forces, against the exact optimum this build returns
            "max_abs_dev_u0_N": float(np.max(du0)),
            "p50_abs_dev_u0_N": float(np.percentile(du0, 50)),
            "p99_abs_dev_u0_N": float(np.percentile(du0, 99)),
            "host": cpu_info,
        }
        # (2) the exact-optimum oracle (dense Goldfarb-Idnani), the parity checker, over the whole batch
        reps = 0
        t1 = time.perf_counter()
        while True:
            O.solve_batch(op, H, rec, con, n_threads=cores, normals=nrm)
            reps += 1
            if time.perf_counter() - t1 >= args.cpu_seconds:
                break
        ct = time.perf_counter() - t1
        cpu_exact = {
            "value": reps * B / ct,
            "unit": "QP/s",
            "cores": cores,
            "kind": "port",
            "algorithm": "exact optimum: fp64 dense Goldfarb-Idnani (oracle/lmpc_oracle.c), the parity checker",
            "sample": f"{reps} x the rank-0 batch ({B} QPs, {wl_name}) over {cores} host threads, {ct:.1f} s wall",
        }

    # HBM bytes per launch of this workload from the committed PMC pass (rocprofv3 FETCH_SIZE + WRITE_SIZE),
    # and the fp64 flops the kernels issued (SQ_INSTS_VALU_FLOPS_FP64 + 512 x SQ_INSTS_VALU_MFMA_MOPS_F64) -- a
    # diagnostic: the VALU counter counts exec-masked lanes and the MFMA one the padded 16x16 tiles
    traffic_bytes = None
    executed = None
    # the committed PMC figures are keyed by workload, plus "/<mode>" when --dense overrides the config's own path
    # (configs 3 and 5 run the Riccati kernel by default: H > 16 has no dense path); none for --riccati scratch (the
    # warm-start kernel)
    overridden = args.dense is not None and args.dense != default_dense
    wl = (f"{wl_name}/{mode}" if overridden else wl_name) if args.batch is None and args.riccati == "lds" else None
    try:
        tr = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
        if wl in tr:
            traffic_bytes = tr[wl]["bytes_per_qp"] * B  # this rank's launch (config 4 at N > 1: 65536/N QPs)
    except (OSError, ValueError, KeyError):
        traffic_bytes = None
    try:
        fl = json.load(open(os.path.join(ROOT, "profiles", "pmc_flops.json")))
        if wl in fl:
            e = fl[wl]["flop_per_qp"]
            executed = {
                "flop_per_qp": e,
                "what": "issued fp64 lane-flops: exec-masked lanes and padded MFMA tile entries included",
                "issued_over_useful": e / useful_per_qp,
                "achieved": e * B / (kernel_ms * 1e-3) / 1e12,
                "valu_share": fl[wl]["valu_flop_per_qp"] / e,
                # matrix-core issue: the executed MFMA flops per second against the fp64 MFMA peak
                "mfma_issue_frac": fl[wl]["mfma_flop_per_qp"] * B / (kernel_ms * 1e-3) / 1e12 / roofline.FP64_PEAK_TFLOPS,
                "source": fl[wl]["source"],
            }
    except (OSError, ValueError, KeyError, ZeroDivisionError):
        executed = None

    if rank == 0:
        line = {
            "metric": "QP solves/sec (Go1, horizon=10, 12 contacts); max GRF err vs exact-QP oracle",
            "value": total_qps,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm_run,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (Philox-seeded perturbed states, SURVEY.md 8d; generated on device)",
            "config": {
                "workload": wl_name if args.batch is None else f"{wl_name}@b{B}",
                "horizon": H,
                "batch_per_gpu": B,
                "global_batch": global_batch,
                "robot": cfg["robot"],
                "gait": "mixed" if cfg["gait"] < 0 else ["trot", "crawl", "trot_with_stand", "stand"][cfg["gait"]],
                "terrain": f"per-leg normals, tilt U(0, {synth.TERRAIN_THETA_MAX}) rad" if terrain else None,
                "parallelism": f"dp{world} (independent QP shards, no collective)",
                **({"options": opts} if opts else {}),
                **({"index_offset": args.index_offset} if args.index_offset else {}),
            },
            "roofline": {
                # fp64 compute, not HBM: a latency-bound wave per QP issuing fp64 VALU and MFMA work;
                # the fp64 peak is the same for both.  achieved / frac: SURVEY.md 8(d)'s contract flops where every QP
                # runs on a condensed dense kernel (config 2, the headline), else the useful flops of the formulation
                # the kernels run (roofline.lq_flop / dense_flop); never a fraction above 1
                "bound": "fp64-valu-latency",
                "achieved": achieved_tf,
                "peak": roofline.FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / roofline.FP64_PEAK_TFLOPS,
                "frac_source": "contract (SURVEY 8d)" if headline_contract else "useful flops of the formulation run",
                "flop_per_qp": contract_per_qp if headline_contract else useful_per_qp,
                "flop_model": flop_model if headline_contract else
                "roofline.lq_flop (LDS Riccati kernel) / roofline.dense_flop (condensed QP, N = 3 x stance leg-steps)",
                "useful_flop_per_qp": useful_per_qp,
                "useful_frac": useful_tf / roofline.FP64_PEAK_TFLOPS,
                **({"contract_flop_per_qp": contract_per_qp,
                    "contract_model": flop_model} if headline_contract else {}),
                "traffic": traffic_bytes,
                "kernel": kernel_label(mode, args.riccati, fused=mode == "ipm" and args.riccati == "lds" and 4 * H <= 64
                                       and B <= 4 * torch.cuda.get_device_properties(dev).multi_processor_count),
                "kernel_ms": kernel_ms,
                "executed": executed,
                "hbm_gbs": roofline.qp_bytes(H) * B / (kernel_ms * 1e-3) / 1e9,
            },
            "cpu_baseline": cpu,
            "cpu_baseline_exact": cpu_exact,
            "with_gather": with_gather,
            "max_grf_err": max_err,
            "max_grf_abs_err_N": max_abs,
            "parity": {
                "vs": "exact optimum of the reference's QP (oracle/: fp64 dense Goldfarb-Idnani, KKT-certified)",
                "err": "max over H x 12 forces of |f_gpu - f_ref| / max(1, |f_ref|)",
                "qps_checked": int(parity_checked),
                "reference_solver": "unpinned: the reference ships no fixtures for this path and its OSQP stops "
                                    "at eps_abs 1e-3 (ConvexQPSolver.cpp:183-184); DESIGN.md 6",
            },
            "qp_status": {"converged": int(stats[0]), "max_iter": int(stats[1]), "nan": int(stats[2])},
            "dense_path": mode,
            "riccati_path": args.riccati,
            "ipm_iters_mean": ipm_mean,
            "polish_rounds_mean": pol_mean,
            "ipm_iters_max": int(np.max(it & 0xFFFF)),
            "polish_rounds_max": int(np.max(it >> 16)),
            "ipm_iters_p99": float(np.percentile(it & 0xFFFF, 99)),
            "polish_rounds_p99": float(np.percentile(it >> 16, 99)),
            # per-QP iteration words of the measured batch (rank 0's shard): the launch waits for its slowest QP
            "iteration_histogram": {
                "ipm_iters": {str(k): int(v) for k, v in zip(*np.unique(it & 0xFFFF, return_counts=True))},
                "polish_rounds": {str(k): int(v) for k, v in zip(*np.unique(it >> 16, return_counts=True))},
            },
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

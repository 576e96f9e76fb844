#!/usr/bin/env python3
"""Dev tool: randomised parity of the WBC/HoQp kernel against the restatement (oracle/hoqp.py), beyond the committed
golden groups (round 6, after the crossover's non-negative multipliers).  Chains of the golden groups' families
(tests/golden/make_hoqp_golden.py: rand3 n = 8, n20, exhaust n = 6; infeasible chains -- the oracle raises -- are
skipped), many seeds each.  Three steps, because the oracle takes minutes and a GPU box must not sit silent:

    python tools/hoqp_fuzz.py gen  OUTDIR [count]   # CPU: chains + oracle answers -> OUTDIR/cases_<family>.npz
    python tools/hoqp_fuzz.py solve OUTDIR          # GPU box: the kernel's answers -> OUTDIR/gpu_<family>.npz
    python tools/hoqp_fuzz.py cmp  OUTDIR           # CPU: the GPU tests' measures (tests/test_gpu_hoqp.py)
(HQFUZZ_TAG=x: solve / cmp the answers of another library, LMPC_LIB, as gpux_<family>.npz)

The comparison is test_gpu_hoqp.check_against's: every level's A x and every slack within 1e-6 of the data's scale,
the final x where the hierarchy pins every variable.
"""
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402

FAMILIES = {  # name: (seed base, pinned, generator)
    "rand3": (700_000, False, lambda r, s: [_task(r, 8, 2, 3, s % 2 == 0), _task(r, 8, 2, 2, False),
                                            _task(r, 8, 3, 2, s % 3 == 0)]),
    "n20": (800_000, True, lambda r, s: [_task(r, 20, 6, 10, True), _task(r, 20, 5, 6, False),
                                         _task(r, 20, 9, 0, False)]),
    "exhaust": (900_000, True, lambda r, s: [_task(r, 6, 2, 3, True), _task(r, 6, 4, 2, False),
                                             _task(r, 6, 2, 2, False)]),
}


def _task(rng, n, ne, ni, tight):
    from legged_mpc_control_amd import hoqp as HQ

    a = rng.standard_normal((ne, n))
    d = rng.standard_normal((ni, n))
    f = rng.uniform(-0.5, 0.2, ni) if tight else rng.uniform(0.5, 2.0, ni)
    return HQ.Task(a, rng.standard_normal(ne), d, f)


def _one(args):
    fam, seed = args
    from oracle import hoqp as Q

    base, _, make = FAMILIES[fam]
    c = make(np.random.default_rng(base + seed), seed)
    lv = []
    try:
        for t in c:
            lv.append(Q.HoQp(Q.Task(t.a, t.b, t.d, t.f), lv[-1] if lv else None))
    except ValueError:
        return seed, None
    return seed, (np.stack([h.solution() for h in lv]), lv[-1].stacked_slack)


def gen(out, count):
    from legged_mpc_control_amd import hoqp as HQ

    os.makedirs(out, exist_ok=True)
    for fam, (base, pinned, make) in FAMILIES.items():
        with Pool(8) as p:
            res = sorted((s, r) for s, r in p.imap_unordered(_one, [(fam, s) for s in range(count)], chunksize=16)
                         if r is not None)
        seeds = [s for s, _ in res]
        chains = [make(np.random.default_rng(base + s), s) for s in seeds]
        dims = HQ.dims_of(chains[0])
        rec = np.stack([HQ.pack(c, dims) for c in chains])
        d = np.array([dims.num_vars, dims.num_levels] + list(dims.eq_rows) + list(dims.ineq_rows), dtype=np.int32)
        np.savez(os.path.join(out, f"cases_{fam}.npz"), rec=rec, dims=d, x=np.stack([r[0] for _, r in res]),
                 w=np.stack([r[1] for _, r in res]), pinned=np.array(pinned), seeds=np.array(seeds))
        print(f"{fam}: {len(seeds)} feasible chains of {count}", flush=True)


def solve(out):
    import test_gpu_hoqp as T
    from legged_mpc_control_amd import hoqp as HQ

    for fam in FAMILIES:
        d = np.load(os.path.join(out, f"cases_{fam}.npz"), allow_pickle=False)
        dims = T.dims_from(d["dims"])
        x, w, st, it = HQ.HoqpBatch(dims, d["rec"].shape[0]).solve(d["rec"])
        np.savez(os.path.join(out, f"gpu{os.environ.get('HQFUZZ_TAG', '')}_{fam}.npz"), x=x, w=w, st=st, it=it)
        print(f"{fam}: {d['rec'].shape[0]} chains solved, status {np.bincount(st, minlength=3).tolist()}", flush=True)


def cmp(out):
    import test_gpu_hoqp as T

    for fam in FAMILIES:
        d = np.load(os.path.join(out, f"cases_{fam}.npz"), allow_pickle=False)
        g = np.load(os.path.join(out, f"gpu{os.environ.get('HQFUZZ_TAG', '')}_{fam}.npz"), allow_pickle=False)
        dims = T.dims_from(d["dims"])
        bad, worst = [], 0.0
        for b in range(d["rec"].shape[0]):
            rec = d["rec"][b]
            scale = 1.0 + max(float(np.max(np.abs(rec))), float(np.max(np.abs(d["x"][b]))))
            for l, (a, bb, dd, f) in enumerate(T.unpack(rec, dims)):
                if a.shape[0]:
                    worst = max(worst, float(np.max(np.abs(a @ (g["x"][b, l] - d["x"][b, l])))) / scale)
            try:
                T.check_against(rec, dims, g["x"][b], g["w"][b], d["x"][b], d["w"][b], bool(d["pinned"]), T.TOL)
            except AssertionError as e:
                bad.append((int(d["seeds"][b]), str(e)))
        xo = (g["it"] >> 16) & 3
        print(f"{fam}: {d['rec'].shape[0]} chains, status {np.bincount(g['st'], minlength=3).tolist()}, "
              f"levels verified {float((xo == 3).mean()):.4f}, worst level A x {worst:.1e} of the scale, "
              f"beyond the tests' 1e-6: {len(bad)} {bad[:3]}")


if __name__ == "__main__":
    cmd, out = sys.argv[1], sys.argv[2]
    if cmd == "gen":
        gen(out, int(sys.argv[3]) if len(sys.argv) > 3 else 2000)
    elif cmd == "solve":
        solve(out)
    else:
        cmp(out)

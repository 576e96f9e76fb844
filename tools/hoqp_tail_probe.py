#!/usr/bin/env python3
"""Dev tool (GPU box): where the WBC bench batch's long chains come from (round 6).

    LMPC_LIB=tools/build/liblmpc_itd.so python tools/hoqp_tail_probe.py [distinct]

Needs a -DLMPC_HQ_ITDIAG build (the first interior-point pass's iteration count in bits 20-27 of each level's
iteration word).  Solves the bench's distinct synthetic WBC chains (tools/bench_hoqp.py, same seeds) and prints per
level how many chains resumed the interior point after a first-pass crossover that did not verify, the iteration
histograms, and the chains with the most iterations over their three levels.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def main():
    nd = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    from legged_mpc_control_amd import hoqp as HQ
    from legged_mpc_control_amd import wbc as W
    from bench_hoqp import SEED0

    chains = [W.synth_wbc_tasks(SEED0 + i) for i in range(nd)]
    dims = HQ.dims_of(chains[0])
    rec = np.ascontiguousarray(np.stack([HQ.pack(c, dims) for c in chains]))
    s = HQ.HoqpBatch(dims, nd)
    x, w, st, word = s.solve(rec)
    it = word & 0xFFFF
    xo = (word >> 16) & 3
    it0 = (word >> 20) & 0xFF
    why = (word >> 28) & 7  # the last crossover's failure: 1 too many active rows, 2 non-finite, 3 stationarity, 4 rounds, 5 an active row not met
    print("status", np.bincount(st, minlength=3))
    for l in range(it.shape[1]):
        res = it[:, l] > it0[:, l]
        print(f"level {l}: iterations mean {it[:, l].mean():.2f} max {it[:, l].max()}; first pass mean "
              f"{it0[:, l].mean():.2f} max {it0[:, l].max()}; resumed {res.sum()} (their total iterations "
              f"{np.bincount(it[res, l]).nonzero()[0].tolist()}); crossover bits {np.bincount(xo[:, l], minlength=4)}")
        print("   first-pass histogram", np.bincount(it0[:, l]).tolist())
        print("   last crossover's failure reason (levels not verified: 1 rows, 2 non-finite, 3 stationarity, 4 rounds, 5 active row not met)",
              np.bincount(why[xo[:, l] == 1, l], minlength=6).tolist())
        print("   total histogram     ", np.bincount(it[:, l]).tolist())
    tot = it.sum(1)
    print(f"iterations per chain: mean {tot.mean():.2f} p99 {np.percentile(tot, 99):.0f} max {tot.max()}")
    cyc = None
    from legged_mpc_control_amd import _native as N
    L = N.lib()
    if hasattr(L, "lmpc_debug_hoqp_stamps"):  # a -DLMPC_STAMPS build: per-chain cycles
        import ctypes
        L.lmpc_debug_hoqp_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        buf = np.zeros((nd, 8), dtype=np.uint64)
        n = L.lmpc_debug_hoqp_stamps(buf.ctypes.data, nd)
        cyc = buf[:n].sum(1).astype(float)
        print(f"cycles per chain: mean {cyc.mean():.0f} p99 {np.percentile(cyc, 99):.0f} max {cyc.max():.0f}")
        res_any = (it > it0).any(1)[:n]
        print(f"  chains that resumed some level: {res_any.sum()}, their cycles mean {cyc[res_any].mean():.0f}; "
              f"the others {cyc[~res_any].mean():.0f}")
        # the bench tiles the distinct chains to 4096 over 1024 slots (4 per CU): list scheduling in index order
        for slots, tile in ((1024, 4096),):
            c = np.resize(cyc, tile)
            free = np.zeros(slots)
            for v in c:
                k = np.argmin(free)
                free[k] += v
            print(f"  {tile} chains on {slots} slots, index order: makespan {free.max():.0f} cycles = "
                  f"{free.max() / (c.sum() / slots):.3f} x the mean load")
    if hasattr(L, "lmpc_debug_hoqp_nnls"):  # NNLS calls / successes per chain (cumulative over launches)
        import ctypes
        L.lmpc_debug_hoqp_nnls.argtypes = [ctypes.c_void_p, ctypes.c_int]
        nb = np.zeros(nd, dtype=np.int32)
        L.lmpc_debug_hoqp_nnls(nb.ctypes.data, nd)
        calls, succ = nb % 64, nb // 64
        print(f"NNLS: chains calling it {int((calls > 0).sum())}, calls {int(calls.sum())}, successes {int(succ.sum())}")
        unver = np.nonzero((xo == 1).any(1))[0]
        print("  unverified chains:", [(int(b), int(calls[b]), int(succ[b])) for b in unver])
    order = np.argsort(-(cyc if cyc is not None else tot))
    for b in order[:12]:
        extra = f" {cyc[b]:.0f} cycles" if cyc is not None else ""
        print(f"  chain {b}:{extra} " + "  ".join(f"L{l} {it0[b, l]}/{it[b, l]} xo{xo[b, l]}" for l in range(it.shape[1])))


if __name__ == "__main__":
    main()

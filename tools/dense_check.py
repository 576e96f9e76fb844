#!/usr/bin/env python3
"""Dev tool (GPU): the condensed dense path vs the Riccati path vs the oracle, and their kernel times."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.init()
from legged_mpc_control_amd import BatchedConvexQPSolver, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


MODES = {"gi": "gi", "ipm": "ipm", "riccati": "off"}


def solver(p, H, B, mode):
    return BatchedConvexQPSolver(p, H, B, dense_path=MODES[mode])


def main():
    for cid, cnt in ((2, 256), (4, 256), (1, 1)):
        p, H, rec, con = synth.config_batch(cid, count=cnt)
        nrm = synth.config_normals(cid, count=cnt)
        ref, _, _ = O.solve_batch(O.params_from(p), H, rec, con, n_threads=8, normals=nrm)
        for dense in ("gi", "ipm", "riccati"):
            g, st, it = solver(p, H, cnt, dense).solve(rec, con, normals=nrm)
            err = np.max(np.abs(g - ref) / np.maximum(1.0, np.abs(ref)))
            nls = (con.sum((1, 2)))
            print(f"config {cid} dense={dense}: max err {err:.2e} status {np.bincount(st, minlength=3)} "
                  f"ipm {np.mean(it & 0xffff):.2f} rounds {np.mean(it >> 16):.2f} "
                  f"(dense-eligible {(nls <= 20).sum()}/{cnt})", flush=True)
            if err > 1e-6:
                bad = np.argsort(-np.max(np.abs(g - ref).reshape(cnt, -1), 1))[:3]
                for b in bad:
                    print("   worst", b, "nls", nls[b], "err", np.max(np.abs(g[b] - ref[b])), "status", st[b], "it", it[b] & 0xffff, it[b] >> 16)
    # timing, config 2 full batch
    p, H, rec, con = synth.config_batch(2)
    dev = torch.device("cuda", 0)
    for dense in ("gi", "ipm", "riccati", "gi"):
        s = solver(p, H, len(rec), dense)
        d = [torch.from_numpy(rec).to(dev), torch.from_numpy(con).to(dev),
             torch.empty((len(rec), H, 12), dtype=torch.float64, device=dev),
             torch.empty(len(rec), dtype=torch.int32, device=dev), torch.empty(len(rec), dtype=torch.int32, device=dev)]
        stream = torch.cuda.Stream(dev)
        for _ in range(3):
            s.solve_device(*d, stream=stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            s.solve_device(*d, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        print(f"config 2 B=1024 dense={dense}: {e0.elapsed_time(e1) / 20:.4f} ms per solve", flush=True)




def stamps():
    """Per-phase cycles of the dense kernel (needs the -DLMPC_STAMPS library: build.build_stamps())."""
    import ctypes

    from legged_mpc_control_amd import _native as N
    p, H, rec, con = synth.config_batch(2)
    s = solver(p, H, len(rec), "ipm")
    g, st, it = s.solve(rec, con)
    L = N.lib()
    L.lmpc_debug_dense_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((1024, 14), dtype=np.uint64)
    n = L.lmpc_debug_dense_stamps(buf.ctypes.data, 1024)
    names = ["prologue", "condense", "ipm leg-step + rhs", "M tiles (ipm)", "factor (MFMA part)", "solve", "diag tiles",
             "M tiles (polish)", "predictor step", "corrector step", "polish verify", "polish set-up + rhs",
             "ipm: wave_sum of s'z", "ipm: D blocks + weights"]
    tot = buf[:n, :14].sum(1).astype(float)
    print(f"dense config 2: mean cycles/QP {tot.mean():.0f} (ipm {np.mean(it & 0xffff):.2f} rounds {np.mean(it >> 16):.2f})")
    for i, nm in enumerate(names):
        v = buf[:n, i].astype(float).mean()
        print(f"  {nm:20s} {v:10.0f} ({100 * v / tot.mean():5.1f}%)")
    print(f"  max cycles/QP {tot.max():.0f}, p99 {np.percentile(tot, 99):.0f}")
    if os.environ.get("LMPC_STAMPS_OUT"):  # per-QP phase cycles and iteration words, for comparing builds
        np.savez(os.environ["LMPC_STAMPS_OUT"], stamps=buf[:n], iters=it[:n])
    for q in np.argsort(-tot)[:6]:
        print(f"    slow QP {q}: {tot[q]:.0f} cycles, ipm {it[q] & 0xffff} rounds {it[q] >> 16}, "
              f"diag {buf[q, 6]:.0f} solve {buf[q, 5]:.0f}")
    L.lmpc_debug_condense_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    cb = np.zeros((1024, 5), dtype=np.uint64)
    n = L.lmpc_debug_condense_stamps(cb.ctypes.data, 1024)
    for i, nm in enumerate(["free response", "adjoint + gradient", "P~ recursion", "H zero + identity", "H columns"]):
        print(f"    condense: {nm:20s} {cb[:n, i].astype(float).mean():10.0f}")
    return tot


def gi_stamps():
    """Per-phase cycles of the GI kernel (needs the -DLMPC_STAMPS library)."""
    import ctypes

    from legged_mpc_control_amd import _native as N
    p, H, rec, con = synth.config_batch(2)
    s = solver(p, H, len(rec), "gi")
    g, st, it = s.solve(rec, con)
    L = N.lib()
    L.lmpc_debug_gi_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((1024, 8), dtype=np.uint64)
    n = L.lmpc_debug_gi_stamps(buf.ctypes.data, 1024)
    names = ["prologue+condense", "cholesky+x0+J", "violation search", "d = J'n", "z, r", "step+add",
             "step+drop", "output"]
    tot = buf[:n, :8].sum(1).astype(float)
    steps = it[:n] & 0xffff
    print(f"gi config 2: mean cycles/QP {tot.mean():.0f} max {tot.max():.0f} (steps mean {steps.mean():.1f} max {steps.max()})")
    for i, nm in enumerate(names):
        v = buf[:n, i].astype(float)
        print(f"  {nm:20s} mean {v.mean():10.0f} ({100 * v.mean() / tot.mean():5.1f}%) max {v.max():10.0f}")
    w = int(np.argmax(tot))
    print(f"  slowest QP {w}: {tot[w]:.0f} cycles, {steps[w]} steps, {it[w] >> 16} drops: " +
          ", ".join(f"{nm} {buf[w, i]}" for i, nm in enumerate(names)))
    per = buf[:n, 2:7].sum(1).astype(float) / np.maximum(steps, 1)
    print(f"  cycles per active-set step: mean {per.mean():.0f}")
    return tot


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "stamps":
        from legged_mpc_control_amd import build as B
        os.environ["LMPC_LIB"] = os.environ.get("LMPC_STAMPS_LIB") or B.build_stamps()
        ti = stamps()
        tg = gi_stamps()
        both = np.minimum(ti, tg)
        print(f"per-QP min(ipm, gi): max {both.max():.0f} p99 {np.percentile(both, 99):.0f} mean {both.mean():.0f}; "
              f"corr(ipm, gi) {np.corrcoef(ti, tg)[0, 1]:.2f}; gi faster on {(tg < ti).sum()}/{len(ti)}")
        for cap in (300000, 400000, 500000, 600000):
            c = np.where(tg <= cap, tg, cap + ti)
            print(f"  gi capped at {cap} cycles then ipm: max {c.max():.0f} mean {c.mean():.0f}")
    else:
        main()

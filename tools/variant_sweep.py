"""Dev tool: run parity + iteration statistics + timing for diagnostic library variants.

    python tools/variant_sweep.py TAG [TAG ...]      (libraries tools/build/liblmpc_TAG.so, built beforehand)
Each variant runs in its own subprocess (the ctypes library is bound per process)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def opts():
    """Default options, overridden by LMPC_TOL_MU / LMPC_MAX_ROUNDS when set."""
    import ctypes

    from legged_mpc_control_amd import _native as N

    o = N.LmpcOptions()
    N.lib().lmpc_options_default(ctypes.byref(o))
    if os.environ.get("LMPC_TOL_MU"):
        o.tol_mu = float(os.environ["LMPC_TOL_MU"])
    if os.environ.get("LMPC_MAX_ROUNDS"):
        o.max_rounds = int(os.environ["LMPC_MAX_ROUNDS"])
    return o


def child(tag):
    sys.path.insert(0, ROOT)
    import time

    import numpy as np
    import torch

    torch.cuda.init()  # torch's HIP runtime first (as bench.py does), then the ctypes library

    from legged_mpc_control_amd import BatchedConvexQPSolver, synth
    from oracle import oracle as O

    out = {"tag": tag}
    for (H, gait, B) in ((10, 0, 256), (10, -1, 256), (30, -1, 32)):
        p = synth.params("go1")
        rec, con = synth.fill(p, synth.synth_cfg("go1", gait), H, B, seed=911 + H - gait)
        s = BatchedConvexQPSolver(p, H, B, options=opts())
        grf, st, it = s.solve(rec, con)
        op = O.params_from(p)
        ref = np.stack([O.solve(op, H, rec[b], con[b])[0] for b in range(B)])
        err = float(np.max(np.abs(grf - ref) / np.maximum(1.0, np.abs(ref))))
        ipm, rd = it & 0xFFFF, it >> 16
        out[f"H{H}g{gait}"] = dict(err=err, bad=int((st != 0).sum()), ipm=float(ipm.mean()), ipm_max=int(ipm.max()),
                                   rd=float(rd.mean()), rd_max=int(rd.max()), fac_max=int((ipm + rd).max()))
    p, H, rec, con = synth.config_batch(2)
    s = BatchedConvexQPSolver(p, H, len(rec), options=opts())

    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(rec).to(dev), torch.from_numpy(con).to(dev), torch.empty((len(rec), H, 12), dtype=torch.float64, device=dev),
         torch.empty(len(rec), dtype=torch.int32, device=dev), torch.empty(len(rec), dtype=torch.int32, device=dev)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    for _ in range(3):
        s.solve_device(*d, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(20):
        s.solve_device(*d, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    out["cfg2_kernel_ms"] = e0.elapsed_time(e1) / 20
    it = d[4].cpu().numpy()
    out["cfg2_ipm"] = float((it & 0xFFFF).mean())
    out["cfg2_fac_max"] = int(((it & 0xFFFF) + (it >> 16)).max())
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    for spec in sys.argv[1:]:
        # TAG or TAG:tol_mu
        tag, _, tol = spec.partition(":")
        env = dict(os.environ, LMPC_LIB=os.path.join(ROOT, "tools", "build", f"liblmpc_{tag}.so"))
        if tol:
            env["LMPC_TOL_MU"] = tol
            tag = spec
        r = subprocess.run([sys.executable, __file__, "--child", tag], env=env, capture_output=True, text=True,
                           timeout=300)
        sys.stdout.write(r.stdout if r.returncode == 0 else f'{{"tag": "{tag}", "rc": {r.returncode}, "err": {json.dumps(r.stderr[-800:])}}}\n')
        sys.stdout.flush()
        if r.returncode != 0:
            break


if __name__ == "__main__":
    main()

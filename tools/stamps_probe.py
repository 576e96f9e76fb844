"""Dev tool: per-phase cycle breakdown from the -DLMPC_STAMPS diagnostic build (run under gpurun)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from legged_mpc_control_amd import build as B
os.environ["LMPC_LIB"] = B.build_stamps()
import numpy as np
from legged_mpc_control_amd import BatchedConvexQPSolver, synth
from legged_mpc_control_amd import _native as N

cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
p, H, rec, con = synth.config_batch(cid, count=count)
s = BatchedConvexQPSolver(p, H, max_batch=count)
for _ in range(2):
    grf, st, it = s.solve(rec, con)
L = N.lib()
L.lmpc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((min(count, 4096), 8), dtype=np.uint64)
n = L.lmpc_debug_stamps(buf.ctypes.data, buf.shape[0])
names = ["prologue", "leg/ipm", "factor", "solve", "adjoint", "epilogue"]
tot = buf[:n, :6].sum(1).astype(float)
print(f"config {cid} H={H} B={count}: mean cycles/QP {tot.mean():.0f}  ipm_it {np.mean(it & 0xffff):.2f} rounds {np.mean(it >> 16):.2f}")
for i, nm in enumerate(names):
    print(f"  {nm:9s} {buf[:n, i].astype(float).mean():12.0f}  ({100 * buf[:n, i].astype(float).mean() / tot.mean():5.1f}%)")

# sub-phase stamps (accumulated over every launch above: 2 runs)
L.lmpc_debug_substamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
sb = np.zeros((min(count, 4096), 24), dtype=np.uint64)
n = L.lmpc_debug_substamps(sb.ctypes.data, sb.shape[0])
sb = sb[:n].astype(float) / 2.0
ipm = (it[:n] & 0xffff).astype(float)
rnd = (it[:n] >> 16).astype(float)
nfac = ipm + rnd  # one factorisation per IPM iteration (+ the final check) and per polish round (approx.)
nsol = 2 * ipm + rnd
sub = {0: "solve:pre", 1: "solve:backward", 2: "solve:mid", 3: "solve:forward", 4: "solve:post",
       5: "factor:pre-MFMA", 9: "factor:elim blk0", 10: "factor:elim blk1", 11: "factor:elim blk2", 12: "factor:elim blk3",
       7: "factor:elim out", 8: "factor:post-MFMA", 13: "leg:top-of-loop", 14: "leg:prep+rhs",
       16: "leg:leg_u", 17: "leg:pred-post", 18: "leg:corr-post"}
print(f"sub-phases (cycles per QP, per call; H={H})")
for i, nm in sub.items():
    per_qp = sb[:, i].mean()
    calls = (nsol if (i < 5 or i >= 13) else nfac).mean()
    calls = ipm.mean() if i in (17, 18) else calls
    print(f"  {nm:16s} {per_qp:12.0f}  per call {per_qp / calls:9.0f}  per stage {per_qp / calls / H:8.0f}")

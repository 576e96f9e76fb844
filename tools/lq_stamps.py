"""Dev tool: per-phase cycles of the LDS-resident Riccati kernel (lmpc_lq.hip) from the -DLMPC_STAMPS build, beside
the global-workspace kernel's (lmpc_kernels.hip) on the same QPs.  Run under gpurun:
    python tools/lq_stamps.py CONFIG [COUNT]      (dense path off: every QP on the Riccati kernel)"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from legged_mpc_control_amd import build as B
os.environ["LMPC_LIB"] = os.environ.get("LMPC_STAMPS_LIB") or B.build_stamps()
import numpy as np
from legged_mpc_control_amd import BatchedConvexQPSolver, synth
from legged_mpc_control_amd import _native as N

cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
p, H, rec, con = synth.config_batch(cid, count=count)
L = N.lib()
n = min(count, 4096)

s = BatchedConvexQPSolver(p, H, max_batch=count, dense_path="off", riccati_path="lds")
grf, st, it = s.solve(rec, con)
L.lmpc_debug_lq_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((n, 16), dtype=np.uint64)
L.lmpc_debug_lq_stamps(buf.ctypes.data, n)
buf = buf.astype(float)
ipm = (it[:n] & 0xffff).astype(float)
rnd = (it[:n] >> 16).astype(float)
calls = {0: np.ones(n), 1: 2 * ipm + rnd, 2: ipm, 3: ipm + rnd, 4: 2 * ipm + rnd, 5: 2 * ipm + rnd, 6: ipm, 7: ipm,
         8: rnd, 9: rnd, 10: np.ones(n), 11: ipm + rnd, 12: ipm + rnd, 13: ipm + rnd, 14: ipm + rnd, 15: rnd}
names = ["prologue", "leg-step work", "corr backward", "factorisation", "forward sweep", "inputs", "pred step",
         "corr step", "adjoint", "polish check", "epilogue", " f:C,PA,G", " f:leg blocks", " f:KH", " f:KZ,P", " f:polish (incl.)"]
tot = buf[:, :15].sum(1)
if os.environ.get("LQ_STAMPS_DUMP"):  # per-QP cycles and iteration words, for a cost-predictor study on the CPU
    np.savez(os.environ["LQ_STAMPS_DUMP"], cycles=tot, it=it[:n], config=cid, count=count)
print(f"LDS kernel: config {cid} H={H} B={count}: mean cycles/QP {tot.mean():.0f} max {tot.max():.0f}  "
      f"ipm {ipm.mean():.2f} rounds {rnd.mean():.2f}")
for i, nm in enumerate(names):
    m = buf[:, i].mean()
    c = calls[i].mean()
    print(f"  {nm:14s} {m:11.0f} ({100 * m / tot.mean():5.1f}%)  per call {m / max(c, 1e-9):8.0f}  per stage {m / max(c, 1e-9) / H:6.0f}")

# Dispatch tail (round 6): the launch's QPs run on `slots` wave slots (4 per CU at H > 16 and at H <= 16 with one
# wave per SIMD, 8 at two waves per SIMD), each slot taking the next QP when it frees -- list scheduling in index
# order, which is what the dispatcher does.  Against the mean load per slot and against longest-first order.
import heapq  # noqa: E402


def makespan(costs, m):
    h = [0.0] * m
    for c in costs:
        heapq.heappush(h, heapq.heappop(h) + c)
    return max(h)


slots = 256 * (8 if (4 * H <= 64 and count > 1024) else 4)
if count > slots:
    ms_list, ms_lpt, mean_load = makespan(tot, slots), makespan(np.sort(tot)[::-1], slots), tot.sum() / slots
    print(f"dispatch tail on {slots} slots: mean load {mean_load:.0f} cycles, index order {ms_list:.0f} "
          f"({ms_list / mean_load:.3f}x), longest first {ms_lpt:.0f} ({ms_lpt / mean_load:.3f}x)")

s2 = BatchedConvexQPSolver(p, H, max_batch=count, dense_path="off", riccati_path="scratch")
grf2, st2, it2 = s2.solve(rec, con)
L.lmpc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
b2 = np.zeros((n, 8), dtype=np.uint64)
L.lmpc_debug_stamps(b2.ctypes.data, n)
b2 = b2.astype(float)
ipm2 = (it2[:n] & 0xffff).astype(float)
rnd2 = (it2[:n] >> 16).astype(float)
tot2 = b2[:, :6].sum(1)
print(f"scratch kernel: mean cycles/QP {tot2.mean():.0f} max {tot2.max():.0f}  ipm {ipm2.mean():.2f} rounds {rnd2.mean():.2f}")
c2 = {0: 1.0, 1: 1.0, 2: (ipm2 + rnd2).mean(), 3: (2 * ipm2 + rnd2).mean(), 4: rnd2.mean(), 5: 1.0}
for i, nm in enumerate(["prologue", "leg/ipm", "factor", "solve", "adjoint", "epilogue"]):
    m = b2[:, i].mean()
    print(f"  {nm:14s} {m:11.0f} ({100 * m / tot2.mean():5.1f}%)  per call {m / max(c2[i], 1e-9):8.0f}  per stage {m / max(c2[i], 1e-9) / H:6.0f}")

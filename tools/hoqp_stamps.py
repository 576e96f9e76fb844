"""Dev tool: per-phase cycle breakdown of lmpc_hoqp_kernel from the -DLMPC_STAMPS diagnostic build (run under
gpurun): WBC batch of tools/bench_hoqp.py, one launch, mean / max cycles per phase over the instances."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from legged_mpc_control_amd import build as B  # noqa: E402

os.environ["LMPC_LIB"] = B.build_stamps()
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from legged_mpc_control_amd import _native as N  # noqa: E402
from legged_mpc_control_amd import hoqp as HQ  # noqa: E402
from legged_mpc_control_amd import wbc as W  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
chains = [W.synth_wbc_tasks(1_000_000 + i) for i in range(min(batch, 1024))]
dims = HQ.dims_of(chains[0])
rec = np.resize(np.stack([HQ.pack(c, dims) for c in chains]), (batch, HQ.record_len(dims)))
x, w, st, it = HQ.HoqpBatch(dims, batch).solve(rec)
L = N.lib()
L.lmpc_debug_hoqp_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((min(batch, 4096), 8), dtype=np.uint64)
n = L.lmpc_debug_hoqp_stamps(buf.ctypes.data, buf.shape[0])
names = ["setup", "lu+basis", "rows", "resid", "K mfma", "chol", "newton", "output"]
tot = buf[:n].sum(axis=1).astype(float)
print(f"instances {n}, status counts {np.bincount(st, minlength=3)}, iters mean {it.mean(axis=0)} max {it.max(axis=0)}")
print(f"total cycles mean {tot.mean():.0f} max {tot.max():.0f}")
for i, nm in enumerate(names):
    v = buf[:n, i].astype(float)
    print(f"  {nm:9s} mean {v.mean():10.0f} ({100 * v.mean() / tot.mean():5.1f} %) max {v.max():10.0f}")
its = it[:n].sum(axis=1)
print(f"per iteration: chol {np.mean(buf[:n, 5] / its):.0f}  K {np.mean(buf[:n, 4] / its):.0f}  "
      f"newton {np.mean(buf[:n, 6] / its):.0f}  resid {np.mean(buf[:n, 3] / its):.0f}")
L.lmpc_debug_hoqp_substamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
sb = np.zeros((min(batch, 4096), 8), dtype=np.uint64)
L.lmpc_debug_hoqp_substamps(sb.ctypes.data, sb.shape[0])
for i, nm in enumerate(["q", "R'q", "substitutions", "R dy + dirs", "step length", "mu_aff+targets", "update"]):
    print(f"  newton/{nm:15s} per iteration {np.mean(sb[:n, i] / its):8.0f}")

#!/usr/bin/env python3
"""Dev tool (GPU box): kernel time of the Riccati path for a Go1 trot batch at a given horizon (device-resident
inputs, one event pair over K launches), for the library in LMPC_LIB.
    python tools/h_sweep_time.py H BATCH [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from legged_mpc_control_amd import BatchedConvexQPSolver, synth  # noqa: E402

H, B = int(sys.argv[1]), int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda", 0)
p, _, rec, con = synth.config_batch(5, count=B, first_index=0, H=H)
s = BatchedConvexQPSolver(p, H, max_batch=0, device=0, dense_path="off")
d_rec, d_con = torch.from_numpy(rec).to(dev), torch.from_numpy(con).to(dev)
g = torch.empty((B, H, 12), dtype=torch.float64, device=dev)
st = torch.empty(B, dtype=torch.int32, device=dev)
for _ in range(3):
    s.solve_device(d_rec, d_con, g, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    s.solve_device(d_rec, d_con, g, st)
e1.record()
torch.cuda.synchronize()
print(f"{os.path.basename(os.environ.get('LMPC_LIB', 'liblmpc.so'))} H {H} B {B}: {e0.elapsed_time(e1) / K:.4f} ms, "
      f"status ok {(st == 0).sum().item()}/{B}")

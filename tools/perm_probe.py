#!/usr/bin/env python3
"""Dev tool (GPU): solve a config batch in natural and permuted order and report the QPs whose
results differ (stance count, status, iterations of both runs, error of each vs the oracle)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from legged_mpc_control_amd import BatchedConvexQPSolver, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(s, d_rec, d_con, B, H, dev):
    out = torch.full((B, H, 12), float("nan"), dtype=torch.float64, device=dev)
    st = torch.full((B,), -7, dtype=torch.int32, device=dev)
    it = torch.full((B,), -7, dtype=torch.int32, device=dev)
    s.solve_device(d_rec, d_con, out, st, it)
    torch.cuda.synchronize()
    return out, st, it


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cnt = int(sys.argv[2]) if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0)
    p, H, rec, con = synth.config_batch(cid, count=cnt)
    B = rec.shape[0]
    s = BatchedConvexQPSolver(p, H, max_batch=0)
    d_rec, d_con = torch.from_numpy(rec).to(dev), torch.from_numpy(con).to(dev)
    o1, s1, i1 = run(s, d_rec, d_con, B, H, dev)
    o2, s2, i2 = run(s, d_rec, d_con, B, H, dev)
    print("repeat equal:", torch.equal(o1, o2), "status", np.bincount(s1.cpu().numpy() + 7))
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(1)).to(dev)
    o3, s3, i3 = run(s, d_rec[perm].contiguous(), d_con[perm].contiguous(), B, H, dev)
    ref = o1[perm]
    diff = (o3 != ref).reshape(B, -1).any(1) | (o3 != o3).reshape(B, -1).any(1)
    bad = torch.nonzero(diff).flatten().cpu().numpy()
    print(f"permuted mismatches: {len(bad)} of {B}; status perm {np.bincount(s3.cpu().numpy() + 7)}")
    pc = perm.cpu().numpy()
    nls = con.sum((1, 2))
    s1n, i1n, s3n, i3n = s1.cpu().numpy(), i1.cpu().numpy(), s3.cpu().numpy(), i3.cpu().numpy()
    op = O.params_from(p)
    for k in bad[:12]:
        g = pc[k]
        r, _, _ = O.solve(op, H, rec[g], con[g])
        e1 = np.max(np.abs(o1[g].cpu().numpy() - r) / np.maximum(1, np.abs(r)))
        e3 = np.max(np.abs(o3[k].cpu().numpy() - r) / np.maximum(1, np.abs(r)))
        print(f"  slot {k} <- qp {g}: nls {nls[g]} | natural st {s1n[g]} it {i1n[g] & 0xffff}/{i1n[g] >> 16} err {e1:.2e}"
              f" | permuted st {s3n[k]} it {i3n[k] & 0xffff}/{i3n[k] >> 16} err {e3:.2e}")
    if len(bad):
        print("nls histogram of mismatches:", np.bincount(nls[pc[bad]]))
        print("slot mod 8 histogram:", np.bincount(bad % 8, minlength=8), "slot range", bad.min(), bad.max())


if __name__ == "__main__":
    main()

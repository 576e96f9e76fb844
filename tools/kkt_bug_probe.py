#!/usr/bin/env python3
"""Dev tool (GPU box): the re-injected-bug variants (build.py TEST_VARIANTS) on the tests' workloads -- status counts,
how many wrong answers carry status 0, and the largest error among them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import test_gpu_kkt as T  # noqa: E402
from legged_mpc_control_amd import build as B  # noqa: E402

wl = T._workloads()
for tag in B.TEST_VARIANTS:
    L = T._variant(tag)
    for name, p, H, rec, con, ref in wl:
        g, st, _ = T._solve_with(L, p, H, rec, con)
        err = T._per_qp_err(g, ref)
        bad = (st == 0) & (err > 1e-5)
        print(f"{tag:14s} {name:16s} status {np.bincount(st, minlength=3)} status0&err>1e-5 {int(bad.sum())} "
              f"max err {err.max():.3g} max err(status0) {err[st == 0].max() if (st == 0).any() else 0:.3g}", flush=True)

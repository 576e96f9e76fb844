#!/usr/bin/env python3
"""Dev tool (CPU): compare two per-QP dense stamp dumps (tools/dense_check.py stamps with LMPC_STAMPS_OUT).
    python tools/stamps_cmp.py A.npz B.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
ta, tb = a["stamps"][:, :14].sum(1).astype(float), b["stamps"][:, :14].sum(1).astype(float)
print(f"mean {ta.mean():.0f} vs {tb.mean():.0f}; max {ta.max():.0f} vs {tb.max():.0f}; "
      f"p99 {np.percentile(ta, 99):.0f} vs {np.percentile(tb, 99):.0f}")
for q in np.argsort(-np.maximum(ta, tb))[:12]:
    ia, ib = int(a["iters"][q]), int(b["iters"][q])
    print(f"  QP {q}: {ta[q]:.0f} vs {tb[q]:.0f}  (ipm {ia & 0xffff} rounds {ia >> 16}; ipm {ib & 0xffff} rounds {ib >> 16})"
          f"  solve {a['stamps'][q, 5]:.0f}/{b['stamps'][q, 5]:.0f} setup {a['stamps'][q, 11]:.0f}/{b['stamps'][q, 11]:.0f}"
          f" diag {a['stamps'][q, 6]:.0f}/{b['stamps'][q, 6]:.0f}")

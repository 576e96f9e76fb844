#!/bin/bash
# Round 6: Gondzio centrality correctors in the dense interior point (LMPC_GONDZIO builds)
# against the product -- iteration words, errors and config-2 kernel time (three alternating runs).
OUT=gpurun_out/gz
mkdir -p $OUT
for lib in prod6 gz1 gz2 gz1s; do
  timeout -k 10 120 python tools/polish_err_probe.py tools/build/liblmpc_$lib.so $OUT/err_$lib.npy 1024 0 >> $OUT/err.log 2>&1 || exit 3
done
python tools/polish_err_probe.py cmp $OUT/err_prod6.npy $OUT/err_gz1.npy $OUT/err_gz2.npy $OUT/err_gz1s.npy >> $OUT/err.log
python - >> $OUT/err.log << 'PY'
import numpy as np
for t in ("prod6", "gz1", "gz2", "gz1s"):
    a = np.load(f"gpurun_out/gz/err_{t}.npy"); it = a[2].astype(np.int64)
    ipm, rd = it & 0xFFFF, it >> 16
    print(t, "ipm hist", dict(zip(*np.unique(ipm, return_counts=True))), "rounds hist", dict(zip(*np.unique(rd, return_counts=True))))
PY
for rep in 1 2 3; do
  AB_SPECS="2:100" tools/ab_bench.sh prod6 gz1 gz2 gz1s >> $OUT/ab.log 2>&1 || exit 4
done
grep -v "^  qp" $OUT/err.log | grep -v amdgpu; cat $OUT/ab.log

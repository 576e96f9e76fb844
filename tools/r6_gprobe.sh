#!/bin/bash
# Round 6: the n64 golden group per chain and level at the first-pass stop 1e-9 (product) and 1e-8 (diagnostic builds).
export TMPDIR=/tmp
mkdir -p gpurun_out/gprobe
for t in itd9 itd8; do
  echo "== $t" >> gpurun_out/gprobe/n64.log
  LMPC_LIB=tools/build/liblmpc_$t.so timeout -k 10 120 python -u tools/hoqp_golden_probe.py n64 >> gpurun_out/gprobe/n64.log 2>&1 || exit 3
done
cat gpurun_out/gprobe/n64.log

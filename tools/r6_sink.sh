#!/bin/bash
# Round 6: -mllvm -sink-insts-to-avoid-spills (tools/build/liblmpc_sink.so: every kernel) against the product
# (prod6b), configs 2/3/4/5, two alternating rounds.
export TMPDIR=/tmp
mkdir -p gpurun_out/sink
for r in 1 2; do
  AB_SPECS="2:50 3:10 4:4 5:10" tools/ab_bench.sh prod6b sink >> gpurun_out/sink/ab.log 2>&1 || { cat gpurun_out/sink/ab.log; exit 3; }
done
cat gpurun_out/sink/ab.log

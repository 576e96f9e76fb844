#!/bin/bash
# Round 6: stamps + N=2 rehearsal, then the LS=2 two-wave Riccati instance (LMPC_AB_LS2W2) against the product on
# configs 3 and 5, two alternating runs.  Output under gpurun_out/st/ and gpurun_out/ls2w2/.
bash tools/r6_stamps_n2.sh || exit $?
mkdir -p gpurun_out/ls2w2
for rep in 1 2; do
  AB_SPECS="3:10 5:5" tools/ab_bench.sh prod6 ls2w2 >> gpurun_out/ls2w2/ab.log 2>&1 || exit 7
done
cat gpurun_out/ls2w2/ab.log

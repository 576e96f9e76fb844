#!/bin/bash
# Dev tool (GPU box): A/B of the range-space polish rules (LMPC_SCHUR_SLOPE, LMPC_POLISH_BORDER) on config 2.
mkdir -p gpurun_out/border
for r in 1 2 3; do AB_SPECS="2:50" tools/ab_bench.sh ${AB_TAGS:-s0 s1 s2 s3 nb nbs1} || exit 4; done | tee gpurun_out/border/ab_slope.log

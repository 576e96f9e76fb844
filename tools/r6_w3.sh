#!/bin/bash
# Round 6: the LDS Riccati kernel on config 4 (65536 QPs, H = 10, terrain) -- the product (closed-loop rows in LDS,
# 20.1 KB per QP: eight per CU, two waves per SIMD), without the closed-loop rows (14.4 KB, still two waves), and
# without them at three waves per SIMD (168 registers: eleven QPs per CU).  Two alternating runs.
OUT=gpurun_out/w3
mkdir -p $OUT
for rep in 1 2; do
  AB_SPECS="4:5 2off:20" tools/ab_bench.sh prod6 kz0 kz0w3 >> $OUT/ab.log 2>&1 || exit 3
done
cat $OUT/ab.log

#!/bin/bash
# Round 6: the WBC kernel's first interior-point pass capped at 8 / 10 / 12 iterations ahead of the crossover
# (LMPC_HQ_XO_EARLY, tools/build/liblmpc_xe*.so) against the product (prod6): launch time over the 4096-chain bench
# batch (two alternating rounds), crossover outcome per level on the golden chains, and the GPU HoQp tests.
export TMPDIR=/tmp
OUT=gpurun_out/xe
mkdir -p $OUT
HQ_AB_ROUNDS=2 tools/hoqp_ab.sh prod6 xe8 xe10 xe12 > $OUT/ab.log 2>&1 || exit 3
for tag in prod6 xe8 xe10 xe12; do
  echo "== $tag" >> $OUT/xo.log
  LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 120 python tools/hoqp_xo_check.py >> $OUT/xo.log 2>&1 || exit 4
done
for tag in xe8 xe10 xe12; do
  LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hoqp.py -x -q -m gpu \
    --timeout 120 --timeout-method thread > $OUT/tests_$tag.log 2>&1 || { echo "$tag tests failed" >> $OUT/xo.log; }
done
cat $OUT/ab.log $OUT/xo.log
tail -2 $OUT/tests_*.log

#!/bin/bash
# Round 6: the dense polish's accuracy with the (conditional) refinement of range-space rounds
# against round 5's library, and its cost (config 2, alternating library builds on one box), then the GPU tests.
# Output under gpurun_out/refine/.
OUT=gpurun_out/refine
mkdir -p $OUT
for lib in r5 refine; do
  for w in 0 1024 2048 3072; do
    timeout -k 10 120 python tools/polish_err_probe.py tools/build/liblmpc_$lib.so $OUT/err_${lib}_$w.npy 1024 $w >> $OUT/err.log 2>&1 || exit 3
  done
done
for w in 0 1024 2048 3072; do
  python tools/polish_err_probe.py cmp $OUT/err_r5_$w.npy $OUT/err_refine_$w.npy >> $OUT/err.log
done
for rep in 1 2 3; do
  AB_SPECS="2:100" tools/ab_bench.sh r5 refine >> $OUT/ab.log 2>&1 || exit 4
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "differ|max err|range-space" $OUT/gpu_tests.log | head; tail -3 $OUT/gpu_tests.log
cat $OUT/err.log | grep -v "^  qp" ; cat $OUT/ab.log
exit $rc

#!/bin/bash
# Round 6: the WBC's level 0 started at its unconstrained minimiser (LMPC_HQ_LS_START, tools/build/liblmpc_ls0.so)
# against the product (prod6d): launch time over the 4096-chain bench batch (two alternating rounds), crossover
# outcome and golden deviations, the GPU HoQp tests.
export TMPDIR=/tmp
OUT=gpurun_out/ls0
mkdir -p $OUT
for r in 1 2; do
  for tag in prod6d ls0; do
    LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 180 python tools/bench_hoqp.py --steps 20 --warmup 2 --no-cpu \
      --parity-sample 32 > $OUT/b_${tag}_$r.json 2>/dev/null || exit 3
    python -c "import json; d=json.load(open('$OUT/b_${tag}_$r.json')); print('$tag', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], d['parity']['final_x_rel_err'], d['parity']['level_Ax_abs_err'], d['crossover_verified_per_level'], d['ipm_iters_per_level_mean'], d['ipm_iters_per_level_max'], d['status'])" >> $OUT/ab.log
  done
done
echo "== ls0" >> $OUT/xo.log
LMPC_LIB=tools/build/liblmpc_ls0.so timeout -k 10 120 python tools/hoqp_xo_check.py >> $OUT/xo.log 2>&1 || exit 4
LMPC_LIB=tools/build/liblmpc_ls0.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hoqp.py -q -m gpu \
    --timeout 120 --timeout-method thread > $OUT/tests_ls0.log 2>&1 || echo "ls0 tests failed" >> $OUT/xo.log
LMPC_LIB=tools/build/liblmpc_ls0.so timeout -k 10 200 python -u tools/hoqp_dump.py 1024 $OUT/gpu_ls0.npz >> $OUT/xo.log 2>&1 || exit 5
cat $OUT/ab.log $OUT/xo.log; tail -n 3 $OUT/tests_ls0.log; grep "^FAILED\|^E  .*differs" $OUT/tests_ls0.log | head

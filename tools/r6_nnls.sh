#!/bin/bash
# Round 6: non-negative multipliers for the WBC crossover's degenerate active sets (LMPC_HQ_XO_NNLS, tools/build/
# liblmpc_nnls.so) against the product without them (prod6b): launch time over the 4096-chain bench batch (two
# alternating rounds), crossover outcome per level on the golden chains and on the bench chains, GPU HoQp tests.
export TMPDIR=/tmp
OUT=gpurun_out/nnls
mkdir -p $OUT
for r in 1 2; do
  for tag in prod6b nnls; do
    LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 180 python tools/bench_hoqp.py --steps 20 --warmup 2 --no-cpu \
      --parity-sample 32 > $OUT/b_${tag}_$r.json 2>/dev/null || exit 3
    python -c "import json; d=json.load(open('$OUT/b_${tag}_$r.json')); print('$tag', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], d['parity'], d['crossover_verified_per_level'], d['ipm_iters_per_level_max'], d['status'])" >> $OUT/ab.log
  done
done
echo "== nnls" >> $OUT/xo.log
LMPC_LIB=tools/build/liblmpc_nnls.so timeout -k 10 120 python tools/hoqp_xo_check.py >> $OUT/xo.log 2>&1 || exit 4
LMPC_LIB=tools/build/liblmpc_itdst.so timeout -k 10 180 python -u tools/hoqp_tail_probe.py 1024 > $OUT/tail.log 2>&1 || exit 5
LMPC_LIB=tools/build/liblmpc_nnls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hoqp.py -x -q -m gpu \
    --timeout 120 --timeout-method thread > $OUT/tests_nnls.log 2>&1 || echo "nnls tests failed" >> $OUT/xo.log
cat $OUT/ab.log $OUT/xo.log; head -20 $OUT/tail.log; tail -n 2 $OUT/tests_nnls.log

#!/bin/bash
# Round 6: the WBC first-pass stop ahead of the crossover (LMPC_HQ_XO_TOL 1e-8 / 1e-7) with the NNLS multipliers and the
# active-row check, against the product (prod6c, 1e-9): launch time (two alternating rounds), golden chains, tests.
export TMPDIR=/tmp
OUT=gpurun_out/nt
mkdir -p $OUT
for r in 1 2; do
  for tag in prod6c nt8 nt7; do
    LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 180 python tools/bench_hoqp.py --steps 20 --warmup 2 --no-cpu \
      --parity-sample 32 > $OUT/b_${tag}_$r.json 2>/dev/null || exit 3
    python -c "import json; d=json.load(open('$OUT/b_${tag}_$r.json')); print('$tag', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], d['parity']['final_x_rel_err'], d['parity']['level_Ax_abs_err'], d['crossover_verified_per_level'], d['ipm_iters_per_level_mean'], d['status'])" >> $OUT/ab.log
  done
done
for tag in nt8 nt7; do
  echo "== $tag" >> $OUT/xo.log
  LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 120 python tools/hoqp_xo_check.py >> $OUT/xo.log 2>&1 || exit 4
  LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_hoqp.py -q -m gpu \
    --timeout 120 --timeout-method thread > $OUT/tests_$tag.log 2>&1 || echo "$tag tests failed" >> $OUT/xo.log
done
cat $OUT/ab.log $OUT/xo.log
for f in $OUT/tests_*.log; do echo "$f: $(tail -n 1 $f)"; grep "^FAILED\|^E  .*differs" $f | head -8; done

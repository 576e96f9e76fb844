#!/bin/bash
# Round 6: the interior point's default stop at 2e-4 (was 1e-4): the GPU test suite, the bench lines of configs
# 2-5, and a randomised parity sweep at two batch sizes.  Output under gpurun_out/tol/.
export TMPDIR=/tmp
OUT=gpurun_out/tol
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
for c in 3 4 5; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 3; done &&
timeout -k 10 300 python -u tools/fuzz_parity.py --seconds 120 --batch 512 --out $OUT/fuzz_b512.json > $OUT/fuzz_b512.log 2>&1 &&
timeout -k 10 300 python -u tools/fuzz_parity.py --seconds 120 --batch 1024 --out $OUT/fuzz_b1024.json > $OUT/fuzz_b1024.log 2>&1
rc=$?
tail -n 1 $OUT/gpu_tests.log
for c in 2 3 4 5; do python -c "import json; d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]); print('c$c', d['ms_per_step'], d['roofline']['kernel_ms'], d['max_grf_err'], d['qp_status'], d['ipm_iters_mean'], d['polish_rounds_mean'])"; done
tail -n 1 $OUT/fuzz_b512.log $OUT/fuzz_b1024.log
echo "r6_tol rc=$rc"
exit $rc

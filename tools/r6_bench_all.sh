#!/bin/bash
# Round 6: bench lines of configs 2-5 (product), CPU baselines on config 2 only.  Output under gpurun_out/bench/.
OUT=gpurun_out/bench
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 3
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit 4
done
for c in 2 3 4 5; do
  python -c "import json; d=json.loads(open('$OUT/bench_c$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('config $c', 'ms/step %.4f kernel %.4f QP/s %.3e frac %.3f useful %.4f err %.2e' % (d['ms_per_step'], r['kernel_ms'], d['value'], r['frac'], r['useful_frac'], d['max_grf_err']), d['iteration_histogram'])"
done

#!/bin/bash
# GPU box: the round's bench lines (configs 2-5 with the bounded CPU baseline, the WBC HoQp bench) into
# gpurun_out/bench/, each step under its own limit, stopping at the first failure
mkdir -p gpurun_out/bench
for c in 2 3 4 5; do
  steps=20; [ $c = 4 ] && steps=5; [ $c = 3 ] && steps=10; [ $c = 5 ] && steps=10
  timeout -k 10 300 python bench.py --config $c --steps $steps --warmup 3 > gpurun_out/bench/bench_c$c.json 2> gpurun_out/bench/bench_c$c.err || { echo "config $c failed"; tail -n 20 gpurun_out/bench/bench_c$c.err; exit 1; }
  echo "config $c: $(python -c "import json; d=json.load(open('gpurun_out/bench/bench_c$c.json')); print(round(d['ms_per_step'],4), 'ms', '%.3e QP/s' % d['value'], 'frac', round(d['roofline']['frac'],4), d['roofline'].get('frac_source'))")"
done
timeout -k 10 300 python tools/bench_hoqp.py > gpurun_out/bench/bench_hoqp.json 2> gpurun_out/bench/bench_hoqp.err || { tail -n 20 gpurun_out/bench/bench_hoqp.err; exit 1; }
tail -c 600 gpurun_out/bench/bench_hoqp.json

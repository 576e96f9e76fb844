#!/bin/bash
# Round 6 check on the GPU box: the GPU test suite, smoke(), the default bench line (config 2) and the step overhead
# probe.  Each step has its own limit; the chain stops at the first failure.  Output under gpurun_out/r6/.
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
timeout -k 10 120 python tools/step_overhead.py 300 2 > $OUT/overhead.log 2>&1
rc=$?
tail -2 $OUT/gpu_tests.log; cat $OUT/smoke.log; cat $OUT/overhead.log
python -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','max_grf_err')}, d['roofline']['kernel_ms'], d['roofline']['frac'], d['cpu_baseline'].get('max_abs_dev_u0_N'), d['cpu_baseline'].get('p50_abs_dev_u0_N'), d['iteration_histogram'])"
echo "r6_check rc=$rc"
exit $rc

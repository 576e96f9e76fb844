#!/bin/bash
# Round 6: GPU tests after the HoQp C-ABI's lazy ordering event, and the WBC bench line (one event pair, time-based
# warm-up).  Output under gpurun_out/hq/.
OUT=gpurun_out/hq
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_hoqp.py > $OUT/bench_hoqp.json 2> $OUT/bench_hoqp.err
rc=$?
tail -2 $OUT/gpu_tests.log
python -c "import json; d=json.loads(open('$OUT/bench_hoqp.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','warmup_steps_run')}, d['roofline']['kernel_ms'])"
exit $rc

#!/bin/bash
# Round 6: config 2's bench line against the timed-step count and the warm-up (the driver runs --steps 20 --warmup 5);
# --warmup-ms 0 is the round-5 warm-up (W steps only).  Output under gpurun_out/steps/.
OUT=gpurun_out/steps
mkdir -p $OUT
for a in "20 5 0" "20 5 30" "20 5 0" "20 5 30" "50 5 30" "200 50 30"; do
  set -- $a
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --warmup-ms $3 --no-cpu > $OUT/b.json 2>/dev/null || exit 3
  python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('steps $1 warmup $2 warmup-ms $3 (run %d)' % d['warmup_steps_run'], 'ms/step %.4f kernel %.4f' % (d['ms_per_step'], d['roofline']['kernel_ms']))" | tee -a $OUT/steps.log
done

#!/bin/bash
# Dev tool (GPU box): the WBC bench batch with the crossover on and off, alternating (time, parity, crossover stats).
for m in 1 0 1 0; do timeout -k 10 120 python3 tools/bench_hoqp.py --steps 20 --warmup 2 --no-cpu --crossover $m | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=d['parity']; print('xo', $m, 'kernel_ms %.4f'%r['kernel_ms'], 'x %.1e w %.1e ax %.1e'%(p['final_x_rel_err'], p['slack_abs_err'], p['level_Ax_abs_err']), d['status'], d['crossover_verified_per_level'])"; done

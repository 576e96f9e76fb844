#!/bin/bash
# Dev tool (GPU box): the WBC hierarchies' interior-point stop (lmpc_hoqp_options.tol_mu) with the exact crossover
# on: launch time, parity on a sample against the restatement, status and iterations per level.
for t in ${HT_TOLS:-1e-13 1e-11 1e-9 1e-7}; do
  timeout -k 10 200 python tools/bench_hoqp.py --steps 20 --warmup 3 --no-cpu --parity-sample ${HT_SAMPLE:-32} --tol-mu $t 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tol $t', 'ms %.3f'%d['ms_per_step'], d['parity'], d['status'], d['ipm_iters_per_level_mean'], d['ipm_iters_per_level_max'])" || exit 1
done

#!/bin/bash
# Dev tool (GPU box): A/B of the interior point's stop (tol_mu) and the polish budget (max_rounds) on the
# bench path.  AB_TOLS / AB_ROUNDS / AB_CFGS ("config:dense:steps") pick the grid; two alternating passes.
for r in 1 2; do
for spec in ${AB_CFGS:-2:ipm:100 4:gi:20 3:ipm:20 5:ipm:20}; do IFS=: read c d steps <<< "$spec"
 for t in ${AB_TOLS:-1e-8 1e-6}; do
 for mr in ${AB_ROUNDS:-8}; do
  timeout -k 10 120 python bench.py --config $c --dense $d --steps $steps --warmup 3 --no-cpu --opt tol_mu=$t --opt max_rounds=$mr 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c/$d tol $t rounds $mr', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'err %.1e'%d['max_grf_err'], d['qp_status'], 'ipm %.2f rounds %.2f'%(d['ipm_iters_mean'], d['polish_rounds_mean']))" || exit 1
 done
 done
done
done

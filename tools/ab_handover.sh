#!/bin/bash
# Dev tool (GPU box): the dense path's hand-over to the polish -- tol_mu x dense_polish_iter grid on config 2,
# two alternating passes (runtime options, the product library).
mkdir -p gpurun_out/border
for r in 1 2; do
 for t in ${AB_TOLS:-1e-4 3e-4 1e-3}; do
  for pi in ${AB_PI:-40 6 5}; do
   timeout -k 10 120 python bench.py --config 2 --steps 50 --warmup 3 --no-cpu --opt tol_mu=$t --opt dense_polish_iter=$pi 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tol $t polish_iter $pi', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'err %.1e'%d['max_grf_err'], d['qp_status'], 'ipm %.2f rounds %.2f'%(d['ipm_iters_mean'], d['polish_rounds_mean']))" || exit 1
  done
 done
done | tee gpurun_out/border/ab_handover.log

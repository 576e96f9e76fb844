#!/bin/bash
# Dev tool (GPU box): config 4 kernel time against the interior point hand-over tolerance (lmpc_options.tol_mu).
for t in 1e-4 3e-4 3e-5 1e-4; do
  out=$(timeout -k 10 120 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu --opt tol_mu=$t 2>/dev/null) || { echo "tol $t FAILED"; exit 1; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tol_mu', '$t', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'err %.1e'%d['max_grf_err'], d['qp_status'], d.get('mean_ipm_iters'), d.get('mean_polish_rounds'))"
done

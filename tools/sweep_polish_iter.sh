for rep in 1 2; do for k in 40 11 10 9 8; do
LMPC_DENSE_POLISH_ITER=$k timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('polish_iter $k', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'ipm %.2f/%d'%(d['ipm_iters_mean'],d['ipm_iters_max']), 'rounds %.2f/%d'%(d['polish_rounds_mean'],d['polish_rounds_max']), 'err %.1e'%d['max_grf_err'], d['qp_status'])" || exit 1
done; done

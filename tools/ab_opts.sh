#!/bin/bash
# Dev tool (GPU box): A/B of lmpc_options settings on the bench path, two alternating passes.
#   AB_LIBS="product TAG ..." (tools/build/liblmpc_TAG.so)  AB_OFFSETS="0 1024 ..." (bench --index-offset: other samples)  AB_CFGS="config:dense:steps ..."  AB_SETS="opt=v,opt=v;opt=v ..." (';'-separated option sets, ',' within a set)
IFS=';' read -ra SETS <<< "${AB_SETS:-tol_mu=1e-6}"
for r in 1 2; do
for off in ${AB_OFFSETS:-0}; do
for lib in ${AB_LIBS:-product}; do
 if [ "$lib" = product ]; then unset LMPC_LIB; else export LMPC_LIB=tools/build/liblmpc_$lib.so; fi
for spec in ${AB_CFGS:-2:ipm:100}; do IFS=: read c d steps <<< "$spec"
 for set in "${SETS[@]}"; do
  args=""; IFS=',' read -ra kv <<< "$set"; for x in "${kv[@]}"; do args="$args --opt $x"; done
  timeout -k 10 120 python bench.py --config $c --dense $d --steps $steps --warmup 3 --no-cpu --index-offset $off $args 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib cfg $c/$d off $off [$set]', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'err %.1e'%d['max_grf_err'], d['qp_status'], 'ipm %.2f rounds %.2f'%(d['ipm_iters_mean'], d['polish_rounds_mean']))" || exit 1
 done
done
done
done
done

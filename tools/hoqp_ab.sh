#!/bin/bash
# Dev tool (GPU box): A/B launch times of diagnostic HoQp library builds (tools/build/liblmpc_TAG.so, built
# beforehand with build.build_variant), alternating the tags ROUNDS times over the WBC bench batch.
#   tools/hoqp_ab.sh TAG [TAG ...]     (HQ_AB_ROUNDS, HQ_AB_STEPS, HQ_AB_BATCH)
for r in $(seq ${HQ_AB_ROUNDS:-2}); do
  for tag in "$@"; do
    out=$(LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 180 python tools/bench_hoqp.py --steps ${HQ_AB_STEPS:-20} \
          --warmup 2 --batch ${HQ_AB_BATCH:-4096} --no-cpu --parity-sample 4 2>/dev/null) || { echo "$tag FAILED"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; p=d['parity']; print('$tag', 'kernel_ms %.4f'%r['kernel_ms'], 'x %.1e w %.1e ax %.1e'%(p['final_x_rel_err'], p['slack_abs_err'], p['level_Ax_abs_err']), d['status'], d['ipm_iters_per_level_mean'], d['ipm_iters_per_level_max'])"
  done
done

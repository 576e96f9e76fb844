#!/bin/bash
# Dev tool (GPU box): the two Riccati kernels side by side (bench.py --riccati lds / scratch).
#   LQ_SPECS="4:3 3:5" picks configs:steps (suffix off on the config: dense path off, every QP on the Riccati kernel)
for spec in ${LQ_SPECS:-2off:20 3:5 5:5 4:3}; do
  set -- ${spec/:/ }
  cfg=${1%off}; steps=$2
  dense=""
  case "$1" in *off) dense="--dense off";; esac
  for path in lds scratch; do
    out=$(timeout -k 10 180 python bench.py $dense --riccati $path --config $cfg --steps $steps --warmup 2 --no-cpu 2>/dev/null) || { echo "config $1 $path FAILED"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config', '$1', '$path', 'ms %.4f'%d['ms_per_step'], 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'QP/s %.3e'%d['value'], 'err %.1e'%d['max_grf_err'], d['qp_status'])"
  done
done

#!/bin/bash
# Dev tool (GPU box): A/B kernel times of diagnostic library builds over the bench configs.
#   tools/ab_bench.sh TAG [TAG ...]   (libraries tools/build/liblmpc_TAG.so, built beforehand)
#   AB_SPECS="2:50 4:3" picks configs:steps (suffix gi / off on the config: that dense path); AB_ARGS adds bench.py
#   options (e.g. "--riccati lds")
for tag in "$@"; do
  for spec in ${AB_SPECS:-2:20 2gi:20 2off:20 3:5 4:3 5:5}; do
    set -- ${spec/:/ }
    cfg=${1%gi}; cfg=${cfg%off}; steps=$2
    dense=""
    case "$1" in *gi) dense="--dense gi";; *off) dense="--dense off";; esac
    out=$(LMPC_LIB=tools/build/liblmpc_$tag.so timeout -k 10 120 python bench.py $AB_ARGS $dense --config $cfg --steps $steps --warmup 2 --no-cpu 2>/dev/null) || { echo "$tag config $1 FAILED"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'config', '$1', 'kernel_ms %.4f'%d['roofline']['kernel_ms'], 'QP/s %.3e'%d['value'], 'err %.1e'%d['max_grf_err'], d['qp_status'])"
  done
done

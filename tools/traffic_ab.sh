#!/bin/bash
# Dev tool (GPU box): FETCH_SIZE / WRITE_SIZE per QP of diagnostic library builds on one config, one --pmc pass each.
#   tools/traffic_ab.sh "BENCH ARGS" TAG [TAG ...]   (libraries tools/build/liblmpc_TAG.so)
export TMPDIR=/tmp
OUT=gpurun_out/traffic
mkdir -p $OUT
args=$1; shift
for tag in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LMPC_LIB=tools/build/liblmpc_$tag.so timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/$tag$c -o $tag$c --output-format csv -- python3 bench.py $args --steps 2 --warmup 1 --no-cpu > $OUT/$tag$c.log 2>&1 || { echo "$tag $c FAILED"; exit 1; }
  done
done
echo "traffic_ab done"

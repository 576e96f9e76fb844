#!/bin/bash
# GPU box: config-2 evidence after a dense-path change -- rocprof/PMC passes (tools/profile_round.sh 2), the bench
# line with the bounded CPU baseline, and the dense phase stamps; each step under its own limit.
tools/profile_round.sh 2 > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
mkdir -p gpurun_out/bench gpurun_out/st
timeout -k 10 300 python bench.py --config 2 --steps 20 --warmup 3 > gpurun_out/bench/bench_c2.json 2> gpurun_out/bench/bench_c2.err || exit 2
cat gpurun_out/bench/bench_c2.json
LMPC_STAMPS_OUT=gpurun_out/st/dense_stamps.npz LMPC_STAMPS_LIB=tools/build/liblmpc_stamps.so timeout -k 10 200 python -u tools/dense_check.py stamps > gpurun_out/st/dense_stamps.log 2>&1 || exit 3
grep -A4 "max cycles" gpurun_out/st/dense_stamps.log

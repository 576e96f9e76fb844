#!/bin/bash
# GPU box: parity + certificate tests on the product, then A/B kernel times of tools/build/liblmpc_{A,B}.so
#   SW_TESTS="tests/..." (default: parity, kkt, lq), AB_TAGS="base new", AB_SPECS (tools/ab_bench.sh)
mkdir -p gpurun_out/sw
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${SW_TESTS:-tests/test_gpu_parity.py tests/test_gpu_kkt.py tests/test_gpu_lq.py} > gpurun_out/sw/tests.log 2>&1 || { tail -n 30 gpurun_out/sw/tests.log; exit 1; }
tail -n 3 gpurun_out/sw/tests.log
AB_SPECS="${AB_SPECS:-2:20 2gi:20 4:3}" tools/ab_bench.sh ${AB_TAGS:-base new} > gpurun_out/sw/ab.log 2>&1
cat gpurun_out/sw/ab.log

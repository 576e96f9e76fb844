#!/bin/bash
mkdir -p gpurun_out/fl
for t in rcp nsz rcpnsz; do
  LMPC_LIB=tools/build/liblmpc_$t.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lq.py tests/test_gpu_kkt.py > gpurun_out/fl/tests_$t.log 2>&1; echo "$t tests rc=$? $(tail -n 1 gpurun_out/fl/tests_$t.log)"
done
AB_SPECS="2:30 4:3 5:5" tools/ab_bench.sh base rcp nsz rcpnsz base rcp nsz rcpnsz

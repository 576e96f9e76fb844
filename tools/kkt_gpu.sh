#!/bin/bash
# Round-5 certificate check on the GPU box: the KKT tests (re-injected bug with and without the certificate), the
# per-leg phase tests, the certificate residual distribution (diagnostic build) and an A/B of the round-4 library
# against this one.
OUT=gpurun_out/kkt
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_prep.py -x -v -s --timeout 300 --timeout-method thread > $OUT/kkt_tests.log 2>&1; rc1=$?
grep -E "passed|failed|certificate,|no certificate" $OUT/kkt_tests.log | tail -12
[ $rc1 -le 1 ] || exit $rc1
LMPC_LIB=tools/build/liblmpc_kktdiag.so timeout -k 10 300 python -u tools/kkt_diag.py --out $OUT/kkt_diag.json > $OUT/kkt_diag.log 2>&1 || exit 3
AB_SPECS="${AB_SPECS:-2:50 2off:20 3:5 4:5 5:5}" timeout -k 10 500 tools/ab_bench.sh r4 kkt r4 kkt > $OUT/ab.log 2>&1 || exit 4
cat $OUT/ab.log
exit $rc1

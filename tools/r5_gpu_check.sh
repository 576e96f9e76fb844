#!/bin/bash
# Round-5 GPU check: the whole -m gpu suite, smoke(), and the randomised parity sweep with the product library at two
# batch sizes (512: lone-wave instances; 2048: the two-wave instance at H <= 16).  Each step has its own
# limit; the chain stops at the first failure.
OUT=gpurun_out/r5
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -4 $OUT/gpu_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error|assert" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $OUT/smoke.log 2>&1 || exit 5
tail -3 $OUT/smoke.log
timeout -k 10 300 python -u tools/fuzz_parity.py --seconds 120 --batch 512 --out $OUT/fuzz_b512.json > $OUT/fuzz_b512.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/fuzz_parity.py --seconds 120 --batch 2048 --out $OUT/fuzz_b2048.json > $OUT/fuzz_b2048.log 2>&1 || exit 7
tail -n 2 $OUT/fuzz_b512.log $OUT/fuzz_b2048.log

#!/bin/bash
# Dev tool (GPU box): range-space polish rounds that drop faces (LMPC_POLISH_BORDER) -- iteration words against the
# refactorising build on 1024 config-2 QPs, three alternating config-2 A/B runs, then the dense-path GPU tests.
OUT=gpurun_out/border
mkdir -p $OUT
for t in border noschur noborder; do
  timeout -k 10 120 python tools/schur_check.py tools/build/liblmpc_$t.so $OUT/it_$t.npy 1024 777 || exit 3
done
python tools/schur_check.py cmp $OUT/it_border.npy $OUT/it_noschur.npy | tee $OUT/cmp.log
python tools/schur_check.py cmp $OUT/it_noborder.npy $OUT/it_noschur.npy | tee -a $OUT/cmp.log
for r in 1 2 3; do AB_SPECS="2:50" tools/ab_bench.sh border noborder || exit 4; done | tee $OUT/ab.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_parity.log 2>&1; rc=$?
tail -3 $OUT/gpu_parity.log
exit $rc

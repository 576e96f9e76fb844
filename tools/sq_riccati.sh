#!/bin/bash
# SQ wave-state counters (issue vs. waiting) of the Riccati kernel on configs 4 and 5 and of config 2 on the
# Riccati kernel only (--dense off); one --pmc pass each (8 SQ counters).  Run via gpurun from the repo root.
export TMPDIR=/tmp
OUT=gpurun_out/sqr
rm -rf $OUT; mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS"
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/s4 -o s4 --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $OUT/s4.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/s5 -o s5 --output-format csv -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu > $OUT/s5.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $OUT/s2 -o s2 --output-format csv -- python3 bench.py --dense off --steps 3 --warmup 1 --no-cpu > $OUT/s2.log 2>&1
rc=$?; echo "sq_riccati rc=$rc"; exit $rc

#!/bin/bash
# SQ counters of the two Riccati kernels side by side (bench.py --riccati lds / scratch): wave states (issue vs
# waiting) and the instruction mix, one --pmc pass per set and kernel path.  Run via gpurun from the repo root.
#   SQ_CFG="--dense off" (default: config 2, every QP on the Riccati kernel) or e.g. SQ_CFG="--config 4"
export TMPDIR=/tmp
OUT=gpurun_out/sqlq
rm -rf $OUT; mkdir -p $OUT
CFG=${SQ_CFG:---dense off}
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES"
B="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_MOPS_F64"
rc=0
for path in ${SQ_PATHS:-lds scratch}; do
  for set in A B; do
    C=${!set}
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/$path$set -o $path$set --output-format csv -- python3 bench.py $CFG --riccati $path --steps 2 --warmup 1 --no-cpu > $OUT/$path$set.log 2>&1 || { rc=$?; break 2; }
  done
done
echo "sq_lq rc=$rc"
[ $rc = 0 ] && python3 tools/sq_lq_summary.py $OUT
exit $rc

#!/bin/bash
# Collect the round's rocprofv3 evidence on the GPU box (run via gpurun from the repo root):
#   kernel-trace + stats for configs 2 and 4 (default dense path), config 2 with the dual active-set
#   kernel and configs 3 and 5 (Riccati kernel); separate FETCH_SIZE / WRITE_SIZE PMC passes for configs 2-5;
#   one SQ pass per config for the fp64 flops the kernels execute (SQ_INSTS_VALU_FLOPS_FP64 and
#   SQ_INSTS_VALU_MFMA_MOPS_F64: VALU flops and matrix-core flops / 512); and the PMC calibration micro-benchmark
#   (tools/ubench/pmc_cal.hip).  Every GPU step has its own limit and the chain stops at the first failure.
#   Usage: tools/profile_round.sh [configs...]   (default: 2 4 3 5)
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT
mkdir -p $OUT
CFGS="${*:-2 4 3 5}"
rp() { timeout -k 10 300 rocprofv3 "$@"; }
pmc() { timeout -s KILL 240 rocprofv3 "$@"; }
steps_of() { case $1 in 2) echo "--steps 20 --warmup 3";; 4) echo "--steps 5 --warmup 2";; *) echo "--steps 5 --warmup 2";; esac; }
psteps_of() { case $1 in 2) echo "--steps 5 --warmup 1";; *) echo "--steps 2 --warmup 1";; esac; }
rc=0
for c in $CFGS; do
  rp --kernel-trace --stats -d $OUT/c$c -o c$c --output-format csv -- python3 bench.py --config $c $(steps_of $c) --no-cpu > $OUT/c${c}_bench.log 2>&1 || { rc=$?; break; }
  pmc --pmc FETCH_SIZE --kernel-trace -d $OUT/f$c -o f$c --output-format csv -- python3 bench.py --config $c $(psteps_of $c) --no-cpu > $OUT/f$c.log 2>&1 || { rc=$?; break; }
  pmc --pmc WRITE_SIZE --kernel-trace -d $OUT/w$c -o w$c --output-format csv -- python3 bench.py --config $c $(psteps_of $c) --no-cpu > $OUT/w$c.log 2>&1 || { rc=$?; break; }
  pmc --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_MFMA_MOPS_F64 --kernel-trace -d $OUT/q$c -o q$c --output-format csv -- python3 bench.py --config $c $(psteps_of $c) --no-cpu > $OUT/q$c.log 2>&1 || { rc=$?; break; }
  if [ "$c" = 2 ]; then
    rp --kernel-trace --stats -d $OUT/c2gi -o c2gi --output-format csv -- python3 bench.py --dense gi --steps 20 --warmup 3 --no-cpu > $OUT/c2gi_bench.log 2>&1 || { rc=$?; break; }
  fi
done
if [ $rc = 0 ]; then
  pmc --pmc FETCH_SIZE --kernel-trace -d $OUT/calf -o calf --output-format csv -- tools/ubench/pmc_cal > $OUT/calf.log 2>&1 &&
  pmc --pmc WRITE_SIZE --kernel-trace -d $OUT/calw -o calw --output-format csv -- tools/ubench/pmc_cal > $OUT/calw.log 2>&1 &&
  pmc --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_MFMA_MOPS_F64 --kernel-trace -d $OUT/calq -o calq --output-format csv -- tools/ubench/pmc_cal > $OUT/calq.log 2>&1
  rc=$?
fi
echo "profile_round rc=$rc"
find $OUT -name "*.csv" | head -60
exit $rc

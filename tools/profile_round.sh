#!/bin/bash
# Collect the round's rocprofv3 evidence on the GPU box (run via gpurun from the repo root):
#   kernel-trace + stats for configs 2 and 4 (default dense path), config 2 with the dual active-set
#   kernel and configs 3 and 5 (Riccati kernel), separate FETCH_SIZE / WRITE_SIZE PMC passes, and the PMC calibration micro-benchmark
#   (tools/ubench/pmc_cal.hip).  Every GPU step has its own limit and the chain stops at the first failure.
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT
mkdir -p $OUT
rp() { timeout -k 10 300 rocprofv3 "$@"; }
rp --kernel-trace --stats -d $OUT/c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/c2_bench.log 2>&1 &&
rp --kernel-trace --stats -d $OUT/c4 -o c4 --output-format csv -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu > $OUT/c4_bench.log 2>&1 &&
LMPC_DENSE=gi rp --kernel-trace --stats -d $OUT/c2gi -o c2gi --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/c2gi_bench.log 2>&1 &&
rp --kernel-trace --stats -d $OUT/c3 -o c3 --output-format csv -- python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu > $OUT/c3_bench.log 2>&1 &&
rp --kernel-trace --stats -d $OUT/c5 -o c5 --output-format csv -- python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu > $OUT/c5_bench.log 2>&1 &&
rp --pmc FETCH_SIZE --kernel-trace -d $OUT/f2 -o f2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/f2.log 2>&1 &&
rp --pmc WRITE_SIZE --kernel-trace -d $OUT/w2 -o w2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/w2.log 2>&1 &&
rp --pmc FETCH_SIZE --kernel-trace -d $OUT/f4 -o f4 --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $OUT/f4.log 2>&1 &&
rp --pmc WRITE_SIZE --kernel-trace -d $OUT/w4 -o w4 --output-format csv -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $OUT/w4.log 2>&1 &&
rp --pmc FETCH_SIZE --kernel-trace -d $OUT/calf -o calf --output-format csv -- tools/ubench/pmc_cal > $OUT/calf.log 2>&1 &&
rp --pmc WRITE_SIZE --kernel-trace -d $OUT/calw -o calw --output-format csv -- tools/ubench/pmc_cal > $OUT/calw.log 2>&1
rc=$?
echo "profile_round rc=$rc"
find $OUT -name "*.csv" | head -40
exit $rc

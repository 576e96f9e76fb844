#!/bin/bash
# rocprofv3 evidence for the hierarchical-QP kernel (run via gpurun from the repo root): kernel-trace + stats of
# tools/bench_hoqp.py, then separate FETCH_SIZE and WRITE_SIZE PMC passes.  Each step has its own limit; the
# chain stops at the first failure.  tools/pmc_summary.py <tag> hoqp turns gpurun_out/prof_hoqp into profiles/.
export TMPDIR=/tmp
OUT=gpurun_out/prof_hoqp
rm -rf $OUT
mkdir -p $OUT
rp() { timeout -k 10 300 rocprofv3 "$@"; }
rp --kernel-trace --stats -d $OUT/hq -o hq --output-format csv -- python3 tools/bench_hoqp.py --steps 20 --warmup 3 --no-cpu $HOQP_ARGS > $OUT/hq_bench.log 2>&1 &&
rp --pmc FETCH_SIZE --kernel-trace -d $OUT/fhq -o fhq --output-format csv -- python3 tools/bench_hoqp.py --steps 3 --warmup 1 --no-cpu $HOQP_ARGS > $OUT/fhq.log 2>&1 &&
rp --pmc WRITE_SIZE --kernel-trace -d $OUT/whq -o whq --output-format csv -- python3 tools/bench_hoqp.py --steps 3 --warmup 1 --no-cpu $HOQP_ARGS > $OUT/whq.log 2>&1
rc=$?
echo "profile_hoqp rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc

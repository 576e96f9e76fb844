#!/bin/bash
# One gpurun call for a HoQp kernel change (run from the repo root on the GPU box): the HoQp GPU tests, the
# bench line (tools/bench_hoqp.py) and the rocprofv3 evidence (tools/profile_hoqp.sh: kernel stats + FETCH_SIZE /
# WRITE_SIZE passes).  Stops at the first failure.  Then, here: tools/pmc_summary.py <tag> hoqp.
mkdir -p gpurun_out/hqx && timeout -k 10 300 python -u -m pytest tests/test_gpu_hoqp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hqx/tests.log 2>&1 && timeout -k 10 200 python3 tools/bench_hoqp.py --steps 30 --warmup 3 --no-cpu > gpurun_out/hqx/bench.json 2>gpurun_out/hqx/bench.err && bash tools/profile_hoqp.sh > gpurun_out/hqx/prof.log 2>&1; rc=$?; tail -2 gpurun_out/hqx/tests.log; exit $rc

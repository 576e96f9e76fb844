#!/bin/bash
# Round-end check on the GPU box (run from the repo root via gpurun): the GPU test suite, smoke(), the default
# bench line (config 2, CPU baselines included), the HoQp bench line, and a 2-rank rehearsal of the N > 1 path on
# the one GPU (gloo for the bookkeeping collectives: RCCL refuses two ranks on one device).  Each step has its own
# limit; the chain stops at the first failure.  Output under gpurun_out/rc/.
OUT=gpurun_out/rc
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
timeout -k 10 300 python tools/bench_hoqp.py > $OUT/bench_hoqp.json 2> $OUT/bench_hoqp.err &&
LMPC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > $OUT/n2_rehearsal.json 2> $OUT/n2_rehearsal.err
rc=$?
tail -3 $OUT/gpu_tests.log
echo "round_check rc=$rc"
exit $rc

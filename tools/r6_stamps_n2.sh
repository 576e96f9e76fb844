#!/bin/bash
# Round 6: phase stamps of the dense kernel (config 2) and the LDS Riccati kernel (configs 4, 5) on the current
# sources, then a 2-rank rehearsal of bench.py's N > 1 path on the one GPU (gloo for the bookkeeping collectives).
rm -rf gpurun_out/st
bash tools/stamps_round.sh || exit $?
LMPC_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu > gpurun_out/st/n2_rehearsal.json 2> gpurun_out/st/n2_rehearsal.err || exit 9
tail -1 gpurun_out/st/n2_rehearsal.json | cut -c1-300

#!/bin/bash
# Dev tool (GPU box): lmpc_hoqp_kernel launch time and throughput against the batch size (WBC chains).
for b in ${HQ_BATCHES:-1 64 256 1024 2048 4096 8192}; do
  d=$(( b < 512 ? b : 512 ))
  out=$(timeout -k 10 200 python tools/bench_hoqp.py --batch $b --distinct $d --steps 20 --warmup 3 --no-cpu --parity-sample 2 2>/dev/null) || { echo "batch $b FAILED"; exit 1; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch', $b, 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'ms_per_step %.3f' % d['ms_per_step'], 'chains/s %.0f' % d['value'], d['status'])"
done

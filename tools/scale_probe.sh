#!/bin/bash
# Dev tool: kernel time vs batch size (is the launch latency-bound or serialised?)
for b in 16 64 256 1024 4096; do
  timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu --batch $b | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch', d['config']['batch_per_gpu'], 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'QP/s', round(d['value']))"
done

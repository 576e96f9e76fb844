#!/bin/bash
# Round 6: the product after the LS=2 two-wave Riccati instance -- GPU tests, smoke, randomised parity sweeps at
# batch 512 and 2048 (tools/fuzz_parity.py), and the config-3 bench line.  Output under gpurun_out/fc/.
OUT=gpurun_out/fc
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as G; G.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python tools/fuzz_parity.py --seconds 75 --batch 512 --out $OUT/fuzz_b512.json > $OUT/fuzz_b512.log 2>&1 &&
timeout -k 10 200 python tools/fuzz_parity.py --seconds 75 --batch 2048 --out $OUT/fuzz_b2048.json > $OUT/fuzz_b2048.log 2>&1 &&
timeout -k 10 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu > $OUT/bench_c3.json 2> $OUT/bench_c3.err
rc=$?
tail -2 $OUT/gpu_tests.log; cat $OUT/smoke.log | grep -v amdgpu
python -c "
import json
for b in (512, 2048):
    try:
        d = json.load(open('$OUT/fuzz_b%d.json' % b))
        print(b, {k: d[k] for k in d if not isinstance(d[k], (list, dict))})
    except Exception as e: print(b, e)
d=json.loads(open('$OUT/bench_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['roofline']['kernel_ms'], d['max_grf_err'])"
echo "final_check rc=$rc"
exit $rc

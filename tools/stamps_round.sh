mkdir -p gpurun_out/st
timeout -k 10 300 python -u tools/dense_check.py stamps > gpurun_out/st/dense_stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/lq_stamps.py 4 4096 > gpurun_out/st/lq_stamps_c4.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/lq_stamps.py 5 4096 > gpurun_out/st/lq_stamps_c5.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/lq_stamps.py 3 4096 > gpurun_out/st/lq_stamps_c3.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/st/bench_c2.json 2>gpurun_out/st/bench_c2.err || exit 4
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/st/bench_c4.json 2>gpurun_out/st/bench_c4.err || exit 5
grep -v amdgpu.ids gpurun_out/st/dense_stamps.log | head -40

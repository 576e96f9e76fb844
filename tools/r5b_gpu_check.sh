#!/bin/bash
# Round-5 check after the bordered range-space rounds: iteration words against the refactorising build, then the
# whole GPU check (tools/r5_gpu_check.sh).
mkdir -p gpurun_out/border
timeout -k 10 120 python tools/schur_check.py legged_mpc_control_amd/lib/liblmpc.so gpurun_out/border/it_prod.npy 1024 777 || exit 3
timeout -k 10 120 python tools/schur_check.py tools/build/liblmpc_noschur.so gpurun_out/border/it_noschur.npy 1024 777 || exit 3
python tools/schur_check.py cmp gpurun_out/border/it_prod.npy gpurun_out/border/it_noschur.npy | tee gpurun_out/border/cmp_prod.log
tools/r5_gpu_check.sh

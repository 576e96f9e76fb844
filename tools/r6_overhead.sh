#!/bin/bash
# Round 6: config 2's per-step overhead outside the kernel (tools/step_overhead.py): the product (the context's
# ordering event recorded only at a stream switch), round 5's code without its per-call event (LMPC_NO_CTX_EVENT) and
# round 5's library.  Alternating.
# Output under gpurun_out/overhead/.
OUT=gpurun_out/overhead
mkdir -p $OUT
for rep in 1 2; do
  for lib in legged_mpc_control_amd/lib/liblmpc.so tools/build/liblmpc_noctxev.so tools/build/liblmpc_r5.so; do
    echo "== $lib" >> $OUT/ab.log
    LMPC_LIB=$lib timeout -k 10 120 python tools/step_overhead.py 300 1 >> $OUT/ab.log 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $OUT/ab.log

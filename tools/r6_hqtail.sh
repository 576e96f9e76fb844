#!/bin/bash
# Round 6: the WBC bench batch's long chains (tools/hoqp_tail_probe.py on a -DLMPC_HQ_ITDIAG -DLMPC_STAMPS build).
export TMPDIR=/tmp
mkdir -p gpurun_out/hqtail
for t in itdst; do echo "== $t" >> gpurun_out/hqtail/tail.log; LMPC_LIB=tools/build/liblmpc_$t.so timeout -k 10 180 python -u tools/hoqp_tail_probe.py 1024 >> gpurun_out/hqtail/tail.log 2>&1 || break; done
rc=$?; cat gpurun_out/hqtail/tail.log; exit $rc

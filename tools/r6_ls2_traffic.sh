#!/bin/bash
# Round 6: the LS=2 two-wave Riccati instance's spills -- kernel time (two alternating runs) and FETCH / WRITE bytes
# per config-3 launch for the lane-map hoisting variants (LMPC_LQ_HOIST_LS2W2 = 0 / 2 / 3) and the lone-wave
# instance (round 5's choice).  Output under gpurun_out/ls2t/.
export TMPDIR=/tmp
OUT=gpurun_out/ls2t
mkdir -p $OUT
for rep in 1 2; do
  AB_SPECS="3:10" tools/ab_bench.sh ls2h3 ls2h2 ls2h0 prod6 >> $OUT/ab.log 2>&1 || exit 3
done
for tag in ls2h3 ls2h2 ls2h0 prod6; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    LMPC_LIB=tools/build/liblmpc_$tag.so timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/${tag}_$ctr -o p --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --warmup-ms 0 --no-cpu > $OUT/${tag}_$ctr.log 2>&1 || exit 4
  done
done
python3 - << 'PY'
import csv, glob, os
OUT = "gpurun_out/ls2t"
for tag in ("ls2h3", "ls2h2", "ls2h0", "prod6"):
    res = []
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{OUT}/{tag}_{ctr}/**/p_counter_collection.csv", recursive=True) or glob.glob(f"{OUT}/{tag}_{ctr}/p_counter_collection.csv")
        rows = [r for r in csv.DictReader(open(f[0])) if "lmpc_lq_kernel" in r["Kernel_Name"]]
        v = [float(r["Counter_Value"]) for r in rows]
        res.append(sum(v) / len(v) if v else float("nan"))
    print(tag, "FETCH_SIZE %.1f MB (x2 for reads, gfx950)  WRITE_SIZE %.1f MB per launch" % (res[0] / 1e3, res[1] / 1e3))
PY
cat $OUT/ab.log

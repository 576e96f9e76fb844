"""Summarise tools/sq_lq.sh: per Riccati kernel, counters per wave (= per QP that ran the kernel body; waves
that exit at once on a dense-path hand-over are counted too) summed over the profiled dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
for path in ("lds", "scratch"):
    tot = defaultdict(float)
    for s in ("A", "B"):
        for f in glob.glob(os.path.join(out, f"{path}{s}", "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row.get("Kernel_Name", "")
                if "lmpc_lq_kernel" not in k and "lmpc_qp_kernel" not in k:
                    continue
                name = row["Counter_Name"]
                if name == "SQ_WAVES":
                    name = f"SQ_WAVES_{s}"
                tot[name] += float(row["Counter_Value"])
    print(f"== {path}")
    for name in sorted(tot):
        w = tot.get("SQ_WAVES_A" if name in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                              "SQ_ACTIVE_INST_VALU", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_INST_LDS")
                    else "SQ_WAVES_B", 1.0)
        print(f"  {name:28s} {tot[name]:16.0f}  per wave {tot[name] / max(w, 1.0):12.0f}")

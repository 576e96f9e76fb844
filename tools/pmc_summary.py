#!/usr/bin/env python3
"""Turn the output of tools/profile_round.sh (gpurun_out/prof) into the committed evidence:
profiles/<tag>/c{2,2gi,3,4,5}_kernel_stats.csv, pmc_per_dispatch.json, pmc_calibration.json,
profiles/pmc_traffic.json (bytes per launch for bench.py's roofline.traffic) and profiles/pmc_flops.json
(the fp64 flops the solve kernels execute per QP, for bench.py's roofline.executed):
SQ_INSTS_VALU_FLOPS_FP64 (VALU flops) + 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 (matrix-core flops).
The flop counters are calibrated the same way (pmc_cal's fma64 / mfma64 kernels, known counts): on gfx950
SQ_INSTS_VALU_FLOPS_FP64 counts an instruction's flops once per wave, whatever its exec mask (x64 = the
lane-flops the wave issues, an upper bound on the useful ones), and a 16x16x4 f64 MFMA is 4 MOPS (x512 = 2048).

Calibration (tools/ubench/pmc_cal.hip, 512 MiB past the Infinity Cache): for 8-byte-per-lane
coalesced accesses, the access width the solve kernels use, FETCH_SIZE reports half the bytes read
and WRITE_SIZE reports the bytes written exactly.  The read factor is applied to FETCH_SIZE."""
import csv
import json
import os
import shutil
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof")
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01_final"
DST = os.path.join(ROOT, "profiles", TAG)


def rows(name):
    return list(csv.DictReader(open(os.path.join(SRC, name, f"{name}_counter_collection.csv"))))


# one solve launch = a dense-path kernel + the Riccati kernel, or the fused dense + Riccati kernel (round 5)
SOLVE_KERNELS = ("lmpc_dense_kernel", "lmpc_gi_kernel", "lmpc_qp_kernel", "lmpc_lq_kernel", "lmpc_dense_lq_kernel")


def per_kernel(name, kern, counter=None):
    r = [x for x in rows(name) if kern in x["Kernel_Name"] and (counter is None or x["Counter_Name"] == counter)]
    return [float(x["Counter_Value"]) for x in r], [int(x["End_Timestamp"]) - int(x["Start_Timestamp"]) for x in r]


def main_hoqp():
    """tools/profile_hoqp.sh output (gpurun_out/prof_hoqp) -> profiles/<tag>/hoqp_kernel_stats.csv,
    hoqp_pmc_per_dispatch.json and profiles/pmc_traffic.json["wbc_hoqp_3level_n42"]."""
    global SRC
    SRC = os.path.join(ROOT, "gpurun_out", "prof_hoqp")
    os.makedirs(DST, exist_ok=True)
    cal = json.load(open(os.path.join(DST, "pmc_calibration.json")))
    rf, wf = cal["read_factor"], cal["write_factor"]
    f, fd = per_kernel("fhq", "lmpc_hoqp_kernel")
    w, wd = per_kernel("whq", "lmpc_hoqp_kernel")
    fb, wb = st.mean(f) * 1024 * rf, st.mean(w) * 1024 * wf
    B = 4096
    json.dump(dict(fetch_kib_raw=f, write_kib_raw=w, fetch_bytes=fb, write_bytes=wb, dispatch_ns_fetch_pass=fd,
                   dispatch_ns_write_pass=wd), open(os.path.join(DST, "hoqp_pmc_per_dispatch.json"), "w"), indent=1)
    traffic = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    traffic["wbc_hoqp_3level_n42"] = {
        "bytes_per_launch": fb + wb, "bytes_per_qp": (fb + wb) / B, "fetch_bytes": fb, "write_bytes": wb,
        "source": f"profiles/{TAG}/hoqp_pmc_per_dispatch.json",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of tools/bench_hoqp.py "
                  f"(B = {B}); FETCH_SIZE x {rf:.3f}, WRITE_SIZE x {wf:.3f} from profiles/{TAG}/pmc_calibration.json"}
    json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    shutil.copy(os.path.join(SRC, "hq", "hq_kernel_stats.csv"), os.path.join(DST, "hoqp_kernel_stats.csv"))
    shutil.copy(os.path.join(SRC, "hq_bench.log"), os.path.join(DST, "hoqp_prof_bench.log"))
    print("wbc_hoqp_3level_n42", round((fb + wb) / 1e6, 1), "MB/launch", round((fb + wb) / B), "B/hierarchy")


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "hoqp":
        return main_hoqp()
    os.makedirs(DST, exist_ok=True)
    cal = {}
    for tag, ctr in (("calf", "FETCH_SIZE"), ("calw", "WRITE_SIZE")):
        for x in rows(tag):
            cal[f"{x['Kernel_Name'].split('(')[0]}:{ctr}_KiB"] = float(x["Counter_Value"])
    truth_kib = 512 * 1024
    read_factor = truth_kib / cal["read8:FETCH_SIZE_KiB"]
    write_factor = truth_kib / cal["write8:WRITE_SIZE_KiB"]
    cal.update(read_factor=read_factor, write_factor=write_factor, bytes_moved=truth_kib * 1024,
               note="8 B/lane coalesced; FETCH_SIZE x read_factor and WRITE_SIZE x write_factor = bytes")
    # fp64 flop counters: fma64 (1024 waves x 4 chains x 4096 FMAs, all lanes) and mfma64 (1024 x 1024 MFMAs)
    qf = {x["Counter_Name"]: float(x["Counter_Value"]) for x in rows("calq") if x["Kernel_Name"].startswith("fma64")}
    qm = {x["Counter_Name"]: float(x["Counter_Value"]) for x in rows("calq") if x["Kernel_Name"].startswith("mfma64")}
    valu_factor = (2.0 * 4 * 4096 * 64 * 1024) / qf["SQ_INSTS_VALU_FLOPS_FP64"]
    mfma_factor = (2048.0 * 1024 * 1024) / qm["SQ_INSTS_VALU_MFMA_MOPS_F64"]
    cal.update(valu_flop_factor=valu_factor, mfma_flop_factor=mfma_factor,
               flop_note="SQ_INSTS_VALU_FLOPS_FP64 x valu_flop_factor = lane-flops issued (exec mask ignored by the "
                         "counter); SQ_INSTS_VALU_MFMA_MOPS_F64 x mfma_flop_factor = matrix-core flops")
    json.dump(cal, open(os.path.join(DST, "pmc_calibration.json"), "w"), indent=1)

    per = {}
    traffic = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    fpath = os.path.join(ROOT, "profiles", "pmc_flops.json")
    flops = json.load(open(fpath)) if os.path.exists(fpath) else {}
    for c, wl, qps in (("2", "go1_trot_h10_b1024", 1024), ("4", "go1_mixed_h10_b65536+terrain", 65536),
                       ("3", "go1_trot_h20_b8192", 8192), ("5", "go1_trot_h30_b4096", 4096)):
        if not os.path.isdir(os.path.join(SRC, f"f{c}")):
            continue
        valu = mfma = 0.0
        for kern in SOLVE_KERNELS:
            v, _ = per_kernel(f"q{c}", kern, "SQ_INSTS_VALU_FLOPS_FP64")
            m, _ = per_kernel(f"q{c}", kern, "SQ_INSTS_VALU_MFMA_MOPS_F64")
            if v:
                valu += valu_factor * st.mean(v)
                mfma += mfma_factor * st.mean(m)
        flops[wl] = {
            "flop_per_qp": (valu + mfma) / qps, "valu_flop_per_qp": valu / qps, "mfma_flop_per_qp": mfma / qps,
            "source": f"profiles/{TAG}/q{c}_counter_collection.csv",
            "method": f"rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_MFMA_MOPS_F64 over bench.py (config {c}, "
                      f"--no-cpu); per-dispatch means summed over the launch's solve kernels; VALU = {valu_factor:.1f} x "
                      f"FLOPS_FP64 (lane-flops issued: the counter ignores the exec mask), MFMA = {mfma_factor:.1f} x MOPS; "
                      f"factors from profiles/{TAG}/pmc_calibration.json",
        }
        shutil.copy(os.path.join(SRC, f"q{c}", f"q{c}_counter_collection.csv"),
                    os.path.join(DST, f"q{c}_counter_collection.csv"))
        fb = wb = 0.0
        per[wl] = {}
        for kern in SOLVE_KERNELS:
            f, fd = per_kernel(f"f{c}", kern)
            w, wd = per_kernel(f"w{c}", kern)
            if not f:
                continue
            kf, kw = st.mean(f) * 1024 * read_factor, st.mean(w) * 1024 * write_factor
            fb, wb = fb + kf, wb + kw
            per[wl][kern] = dict(fetch_kib_raw=f, write_kib_raw=w, fetch_bytes=kf, write_bytes=kw,
                                 dispatch_ns_fetch_pass=fd, dispatch_ns_write_pass=wd)
        traffic[wl] = {
            "bytes_per_launch": fb + wb,
            "bytes_per_qp": (fb + wb) / qps,
            "fetch_bytes": fb,
            "write_bytes": wb,
            "source": f"profiles/{TAG}/pmc_per_dispatch.json",
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of bench.py "
                      f"(config {c}, --no-cpu); per-dispatch means of the launch's dense-path kernel + Riccati kernel (lmpc_lq_kernel by default); FETCH_SIZE x {read_factor:.3f}, "
                      f"WRITE_SIZE x {write_factor:.3f} from profiles/{TAG}/pmc_calibration.json",
        }
    json.dump(per, open(os.path.join(DST, "pmc_per_dispatch.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    json.dump(flops, open(fpath, "w"), indent=1)
    for c in ("c2", "c4", "c2gi", "c3", "c5"):
        if not os.path.isdir(os.path.join(SRC, c)):
            continue
        shutil.copy(os.path.join(SRC, c, f"{c}_kernel_stats.csv"), os.path.join(DST, f"{c}_kernel_stats.csv"))
        shutil.copy(os.path.join(SRC, f"{c}_bench.log"), os.path.join(DST, f"{c}_bench.log"))
    for k, v in traffic.items():
        print(k, round(v["bytes_per_launch"] / 1e6, 1), "MB/launch", round(v["bytes_per_qp"]), "B/QP")
    for k, v in flops.items():
        print(k, round(v["flop_per_qp"] / 1e6, 3), "Mflop/QP executed,", round(v["mfma_flop_per_qp"] / v["flop_per_qp"], 3),
              "on the matrix cores")


if __name__ == "__main__":
    main()

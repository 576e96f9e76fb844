"""Dev tool: per-region instruction mix of a device function in a gfx950 .s dump.

Regions are delimited by '; wave barrier' markers (single-wave __syncthreads).  Counts are
static (straight-line code; loops/branches are not weighted)."""
import re
import sys


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_") and ("f64" in op or "_b64" in op and op.startswith("v_mov_b64")):
        return "v64"
    if op.startswith("v_"):
        return "v32"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "mem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, func):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(rf"^{re.escape(func)}.*:", l))
    regions, cur = [], {}
    for l in lines[start + 1:]:
        if "s_setpc_b64" in l or "s_endpgm" in l:
            break
        if "; wave barrier" in l:
            regions.append(cur)
            cur = {}
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = classify(op)
        cur[c] = cur.get(c, 0) + 1
    regions.append(cur)
    keys = ["v64", "v32", "lds", "mem", "salu", "wait", "mfma", "other"]
    print("region " + " ".join(f"{k:>5s}" for k in keys) + "  total")
    for i, r in enumerate(regions):
        print(f"{i:6d} " + " ".join(f"{r.get(k, 0):5d}" for k in keys) + f"  {sum(r.values()):5d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

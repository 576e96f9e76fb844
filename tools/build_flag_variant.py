#!/usr/bin/env python3
"""Dev tool: a diagnostic library (tools/build/liblmpc_TAG.so) where the named sources get extra compiler flags on
top of the product's (legged_mpc_control_amd/build.py HIP_FLAGS + SCHED_FLAGS); every other object is reused from
the product build (legged_mpc_control_amd/lib/obj).  For A/B runs of compiler flags (tools/ab_bench.sh).
    python tools/build_flag_variant.py TAG "lmpc_dense.hip,lmpc_gi.hip" -mllvm -misched-cyclicpath [--replace-sched]
--replace-sched: the extra flags replace the file's SCHED_FLAGS instead of adding to them."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from legged_mpc_control_amd import build as B  # noqa: E402


def main():
    tag, files = sys.argv[1], sys.argv[2].split(",")
    extra = [a for a in sys.argv[3:] if a != "--replace-sched"]
    replace = "--replace-sched" in sys.argv[3:]
    B.build_native()
    objdir = os.path.join(B.LIBDIR, "obj")
    vdir = os.path.join(B.ROOT, "tools", "build")
    os.makedirs(vdir, exist_ok=True)
    objs = []
    for s in B.SOURCES:
        if s not in files:
            objs.append(os.path.join(objdir, s + ".o"))
            continue
        obj = os.path.join(vdir, f"{tag}_{s}.o")
        sched = [] if replace else B.SCHED_FLAGS.get(s, [])
        cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
               "-I", os.path.join(B.ROOT, "include"), "-I", B.CSRC, "-c", "-o", obj] + B.HIP_FLAGS + sched + extra + \
            [os.path.join(B.CSRC, s)]
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        objs.append(obj)
    out = os.path.join(vdir, f"liblmpc_{tag}.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    for o in objs:
        if o.startswith(vdir):
            os.remove(o)
    print(out)


if __name__ == "__main__":
    main()

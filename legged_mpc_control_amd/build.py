"""In-tree build of the HIP library (hipcc, gfx950 only) and the C++ host mirror test."""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "liblmpc.so")
ARCH = "gfx950"
# MFMA accumulators in the VGPR file (gfx950's register file is unified): without it the compiler parks the
# fp64 MFMA results in AGPRs and moves every element the VALU touches with v_accvgpr_read/write.  Measured:
# config 2 0.342 -> 0.329 ms, config 4 22.4 -> 22.0 ms (profiles/r02/diag_ab_configs.log).
HIP_FLAGS = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
# Per-file machine scheduler (round 3, tools/ab_bench.sh / tools/hoqp_ab.sh, alternating runs, bit-identical
# results): the kernels are lone-wave, issue-in-order chains, and the ILP-oriented strategies interleave their
# independent work better than the default occupancy-oriented one -- max-ilp: config 2 0.2254-0.2284 ->
# 0.2198-0.2212 ms, config 4 19.61 -> 19.07-19.18 ms; iterative-ilp: the dual active set (config 2 --dense gi)
# 0.469 -> 0.459-0.461 ms, the WBC hierarchies 4.89 -> 4.78 ms.  (iterative-ilp crashes the compiler on
# lmpc_prep.hip, which keeps the default.)
# Floating-point contract of the dense path and the LDS Riccati kernel (the dense body is compiled into both
# lmpc_dense.hip and lmpc_lq.hip):
#   -ffp-contract=on: a * b + c becomes an fma only within one source expression (HIP's default contracts across
#     statements in the backend, where the result depends on how the surrounding code happens to split into basic
#     blocks).  A QP's bits must not depend on the kernel instance or launch that solves it (one- or two-wave
#     Riccati instance, the fused dense + Riccati launch); round 5 found the default broke that identity once the
#     kernel bodies became shared device functions.  0.6-1.4 % faster on configs 2-5 (tools/ab_bench.sh).
#   -fno-signed-zeros: lets the compiler drop additions of and multiplications into structural zeros of the unrolled
#     lane patterns (x + 0.0 = x up to the sign of a zero result; nothing here reads a zero's sign, and NaNs still
#     propagate to the NaN guard): config 4 9.74 -> 9.48 ms, config 5 3.33 -> 3.28 ms, config 2 within noise, every
#     GPU test at its tolerance (profiles/r05/fused/ab_math_flags.log; -freciprocal-math gained < 1 %, not adopted).
KERNEL_FP = ["-ffp-contract=on", "-fno-signed-zeros"]
SCHED_FLAGS = {
    "lmpc_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "lmpc_dense.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"] + KERNEL_FP,
    # the LDS Riccati kernel re-measured in round 5 (profiles/r05/fused/ab_sched.log): iterative-ilp config 4
    # 9.46 -> 9.26 ms, config 5 3.29 -> 3.12 ms; the dense body prefers max-ilp (config 2 +1.2 % under iterative-ilp),
    # so the fused dense + Riccati kernel has a file of its own
    "lmpc_lq.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"] + KERNEL_FP,
    "lmpc_fused.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"] + KERNEL_FP,
    "lmpc_gi.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "lmpc_hoqp.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
}

SOURCES = ["lmpc_kernels.hip", "lmpc_lq.hip", "lmpc_fused.hip", "lmpc_dense.hip", "lmpc_gi.hip", "lmpc_prep.hip", "lmpc_hoqp.hip", "lmpc_wbc.hip", "lmpc_capi.cpp",
           "hoqp_capi.cpp", "lmpc_host.cpp", "ConvexQPSolver.cpp"]
HEADERS = ["lmpc_device.h", "lmpc_common.h", "lmpc_kernel_common.h", "lmpc_dense_common.h", "lmpc_dense_kernel.h", "lmpc_lq_kernel.h",
           "lmpc_hoqp_device.h"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile_lib(out: str, objdir: str, defines=(), flags=(), verbose: bool = False, only=None) -> str:
    """liblmpc from SOURCES: one compile per source (HIP_FLAGS + that file's SCHED_FLAGS + `flags`, -D`defines`),
    run in parallel, then one link; written to `out` atomically.  `only`: compile just these sources and link the
    product's objects (lib/obj, built first) for the rest."""
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    procs, objs = [], []
    for s in SOURCES:
        if only is not None and s not in only:
            objs.append(os.path.join(LIBDIR, "obj", s + ".o"))
            continue
        obj = os.path.join(objdir, s + ".o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
               "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c", "-o", obj] + HIP_FLAGS + \
            SCHED_FLAGS.get(s, []) + list(flags) + [f"-D{d}" for d in defines] + [os.path.join(CSRC, s)]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    for cmd, pr in procs:
        if pr.wait() != 0:
            raise subprocess.CalledProcessError(pr.returncode, cmd)
    tmp = out + ".tmp"
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    os.replace(tmp, out)
    return out


def build_native(force: bool = False, verbose: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [
        os.path.join(ROOT, "include", "lmpc", "lmpc.h"), os.path.join(ROOT, "include", "lmpc", "lmpc_hoqp.h"),
        os.path.join(ROOT, "include", "lmpc", "ConvexQPSolver.hpp"),
        os.path.abspath(__file__)]
    if not force and not _stale(LIB, deps):
        return LIB
    return _compile_lib(LIB, os.path.join(LIBDIR, "obj"), verbose=verbose)


MULTI_LIB = os.path.join(LIBDIR, "liblmpc_multi.so")


def build_multi(force: bool = False, verbose: bool = False) -> str:
    """liblmpc_multi.so (include/lmpc/lmpc_multi.h): several devices from one process, RCCL for the batch
    scatter / gather.  Links liblmpc.so (found next to it at run time) and librccl."""
    src = os.path.join(CSRC, "lmpc_multi.cpp")
    deps = [src, LIB, os.path.join(ROOT, "include", "lmpc", "lmpc_multi.h"), os.path.join(ROOT, "include", "lmpc", "lmpc.h"),
            os.path.abspath(__file__)]
    if not force and not _stale(MULTI_LIB, deps):
        return MULTI_LIB
    tmp = MULTI_LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O2", "-fPIC", "-shared", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", tmp, src,
           "-L", LIBDIR, "-llmpc", "-Wl,-rpath,$ORIGIN", "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, MULTI_LIB)
    return MULTI_LIB


def build_stamps(force: bool = False) -> str:
    """Diagnostic library with in-kernel phase cycle stamps (tools/stamps_probe.py); never shipped as the product."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    out = os.path.join(ROOT, "tools", "build", "liblmpc_stamps.so")
    if not force and not _stale(out, srcs + [os.path.join(CSRC, h) for h in HEADERS]):
        return out
    return _compile_lib(out, os.path.join(ROOT, "tools", "build", "obj_stamps"), defines=["LMPC_STAMPS"])


def build_variant(tag: str, defines, force: bool = False, flags=()) -> str:
    """Diagnostic library variant (extra -D flags, extra compiler flags) under tools/build/; never shipped as the
    product."""
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    out = os.path.join(ROOT, "tools", "build", f"liblmpc_{tag}.so")
    if not force and not _stale(out, srcs + [os.path.join(CSRC, h) for h in HEADERS]):
        return out
    return _compile_lib(out, os.path.join(ROOT, "tools", "build", f"obj_{tag}"), defines=defines, flags=flags)


TEST_BUILD = os.path.join(ROOT, "tests", "build")
# Test-only library variants (tests/test_gpu_kkt.py), never the product: bugs re-injected into the LDS Riccati
# kernel's forward sweep -- round 4's lost "+ za", and the next stage's yaw read for A_k -- with the polish's KKT
# certificate (the product's verification) and without it (LMPC_KKT_OFF: round 4's verification).
TEST_VARIANTS = {
    "bugza": (["LMPC_BUG_ZA"], ("lmpc_lq.hip", "lmpc_fused.hip")),
    "bugza_nokkt": (["LMPC_BUG_ZA", "LMPC_KKT_OFF"], ("lmpc_lq.hip", "lmpc_fused.hip")),
    "bugyaw": (["LMPC_BUG_YAW"], ("lmpc_lq.hip", "lmpc_fused.hip")),
    "bugyaw_nokkt": (["LMPC_BUG_YAW", "LMPC_KKT_OFF"], ("lmpc_lq.hip", "lmpc_fused.hip")),
    # the dense polish with every round refactorised (no range-space updates): tests/test_gpu_kkt.py checks that the
    # product's updates reach the same iteration words and forces
    "noschur": (["LMPC_POLISH_SCHUR=0"], ("lmpc_dense.hip", "lmpc_lq.hip", "lmpc_fused.hip")),
}


def build_test_variants(force: bool = False) -> dict:
    """The TEST_VARIANTS libraries under tests/build/ (only the named sources recompiled; the rest are the product's
    objects, so build_native() first)."""
    build_native()
    out = {}
    for tag, (defines, only) in TEST_VARIANTS.items():
        path = os.path.join(TEST_BUILD, f"liblmpc_{tag}.so")
        deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(CSRC, h) for h in HEADERS] + [LIB]
        if force or _stale(path, deps):
            _compile_lib(path, os.path.join(TEST_BUILD, f"obj_{tag}"), defines=defines, only=only)
        out[tag] = path
    return out


def build_cpp_test(force: bool = False) -> str:
    """C++ program that drives legged::ConvexQPSolver exactly like ConvexMpc::grf_update."""
    src = os.path.join(ROOT, "tests", "cpp", "grf_update_test.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "build", "grf_update_test")
    if not force and not _stale(out, [src, LIB]):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", out, src,
           "-L", LIBDIR, "-llmpc", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True)
    return out


def build_cpp_multi_test(force: bool = False) -> str:
    """C++ host over the multi-device C-ABI (tests/cpp/multi_test.cpp): shards a batch without PyTorch."""
    src = os.path.join(ROOT, "tests", "cpp", "multi_test.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "build", "multi_test")
    if not force and not _stale(out, [src, LIB, MULTI_LIB]):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", out, src,
           "-L", LIBDIR, "-llmpc_multi", "-llmpc", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True)
    return out


def build_cpp_eigen_test(force: bool = False) -> str:
    """The reference's ConvexMpc lines over include/lmpc/ConvexQPSolverEigen.hpp (tests/cpp/eigen_dropin_test.cpp),
    compiled against the test stand-ins in tests/cpp/eigen_dropin/ (no Eigen / ROS in this image)."""
    src = os.path.join(ROOT, "tests", "cpp", "eigen_dropin_test.cpp")
    stub = os.path.join(ROOT, "tests", "cpp", "eigen_dropin")
    out = os.path.join(ROOT, "tests", "cpp", "build", "eigen_dropin_test")
    hdr = os.path.join(ROOT, "include", "lmpc", "ConvexQPSolverEigen.hpp")
    if not force and not _stale(out, [src, hdr, LIB]):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), "-O2", "-std=c++17", "-Wall", "-I", stub, "-I", os.path.join(ROOT, "include"), "-o", out, src,
           "-L", LIBDIR, "-llmpc", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True)
    return out


def build_cpp_hoqp_test(force: bool = False) -> str:
    """C++ program running the reference's HoQp test (ho_qp_test.cpp) against legged::HoQp (include/lmpc/HoQp.hpp)."""
    src = os.path.join(ROOT, "tests", "cpp", "ho_qp_test.cpp")
    out = os.path.join(ROOT, "tests", "cpp", "build", "ho_qp_test")
    hdr = os.path.join(ROOT, "include", "lmpc", "HoQp.hpp")
    if not force and not _stale(out, [src, hdr, LIB]):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", out, src,
           "-L", LIBDIR, "-llmpc", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True)
    return out


def build_tool_cpp(name: str, force: bool = False) -> str:
    """Dev tool program over liblmpc.so (tools/<name>.cpp -> tools/build/<name>); never shipped."""
    src = os.path.join(ROOT, "tools", f"{name}.cpp")
    out = os.path.join(ROOT, "tools", "build", name)
    if not force and not _stale(out, [src, LIB]):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [hipcc(), "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", out, src,
           "-L", LIBDIR, "-llmpc", f"-Wl,-rpath,{LIBDIR}"]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
    print(build_multi(force=True, verbose=True))

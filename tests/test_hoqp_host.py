"""CPU tests of the hierarchical-QP boundary (include/lmpc/lmpc_hoqp.h): exports, record
layout, argument checks without a GPU, the WBC task formulation (wbc.cpp:102-259) and its padding rule against
the CPU restatement, the golden fixture's certificates."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

from legged_mpc_control_amd import _native as N
from legged_mpc_control_amd import hoqp as HQ
from legged_mpc_control_amd import wbc as W

HEADER = os.path.join(ROOT, "include", "lmpc", "lmpc_hoqp.h")


def declared():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(lmpc_[a-z0-9_]+)\s*\(", src)))


def test_header_declarations_are_exported_with_c_linkage():
    lib = N.lib()
    assert sorted(N.HOQP_SYMBOLS) == declared()
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for name in declared():
        assert hasattr(lib, name) and name in syms


def test_dims_record_layout_and_limits():
    lib = N.lib()
    d = N.LmpcHoqpDims()
    lib.lmpc_hoqp_dims_wbc(ctypes.byref(d))
    assert (d.num_vars, d.num_levels) == (42, 3)
    assert list(d.eq_rows[:3]) == list(W.WBC_EQ_ROWS) and list(d.ineq_rows[:3]) == list(W.WBC_INEQ_ROWS)
    assert lib.lmpc_hoqp_record_len(ctypes.byref(d)) == (30 + 44 + 18 + 12) * 43
    assert lib.lmpc_hoqp_slack_len(ctypes.byref(d)) == 44
    chain = W.synth_wbc_tasks(3)
    dd = HQ.dims_of(chain)
    assert HQ.record_len(dd) == 4472
    rec = HQ.pack(chain, dd)
    a0 = rec[:30 * 42].reshape(30, 42)
    assert np.array_equal(a0, chain[0].a)
    assert np.array_equal(rec[30 * 43:30 * 43 + 44 * 42].reshape(44, 42), chain[0].d)
    bad = N.LmpcHoqpDims()
    bad.num_vars, bad.num_levels = 65, 1
    assert lib.lmpc_hoqp_record_len(ctypes.byref(bad)) == -1
    bad.num_vars, bad.num_levels = 8, 5
    assert lib.lmpc_hoqp_record_len(ctypes.byref(bad)) == -1
    bad.num_levels = 3
    bad.ineq_rows[0] = bad.ineq_rows[1] = bad.ineq_rows[2] = 60  # 180 stacked rows > 128
    assert lib.lmpc_hoqp_record_len(ctypes.byref(bad)) == -1
    assert lib.lmpc_hoqp_lds_bytes(ctypes.byref(d)) == 40448  # the WBC: four chains per CU
    big = N.LmpcHoqpDims()  # 64 variables with 128 stacked rows: 107 KB of LDS, over one workgroup's 64 KB
    big.num_vars, big.num_levels = 64, 2
    big.eq_rows[0] = big.eq_rows[1] = 64
    big.ineq_rows[0] = big.ineq_rows[1] = 64
    assert lib.lmpc_hoqp_lds_bytes(ctypes.byref(big)) > 65536
    assert lib.lmpc_hoqp_record_len(ctypes.byref(big)) == -1
    o = N.LmpcHoqpOptions()
    lib.lmpc_hoqp_options_default(ctypes.byref(o))
    assert o.max_iter == 60 and o.tol_mu == 1e-13 and o.tol_res == 1e-7 and o.crossover == 1


def test_create_and_solve_reject_bad_arguments_without_gpu():
    import torch

    lib = N.lib()
    d = N.LmpcHoqpDims()
    lib.lmpc_hoqp_dims_wbc(ctypes.byref(d))
    ctx = ctypes.c_void_p()
    assert lib.lmpc_hoqp_create(ctypes.byref(d), 0, 0, ctypes.byref(ctx)) == -1
    assert lib.lmpc_hoqp_create(None, 4, 0, ctypes.byref(ctx)) == -1
    assert lib.lmpc_hoqp_solve_batch(None, None, 1, None, None, None, None) == -1
    assert lib.lmpc_hoqp_solve_device(None, None, 1, None, None, None, None, None) == -1
    assert lib.lmpc_hoqp_solve_batch_z(None, None, 1, None, None, None, None, None, None) == -1
    assert lib.lmpc_hoqp_solve_device_z(None, None, 1, None, None, None, None, None, None, None) == -1
    assert lib.lmpc_hoqp_sync(None) == -1
    if torch.cuda.device_count() == 0:
        assert lib.lmpc_hoqp_create(ctypes.byref(d), 4, 0, ctypes.byref(ctx)) == -2
        assert not ctx.value
        with pytest.raises(RuntimeError):
            HQ.HoqpBatch(d, 4)


def test_task_stacking_follows_task_h():
    a = np.ones((2, 3))
    t = HQ.Task(a, [1, 2], None, None) + HQ.Task(None, None, np.eye(3), [1, 1, 1])
    assert t.a.shape == (2, 3) and t.d.shape == (3, 3)  # 0x0 blocks absorbed (task.h:40-51)
    u = HQ.Task(2 * a, [3, 4]) + HQ.Task(a, [1, 2])
    assert np.array_equal(u.a[:2], 2 * a) and np.array_equal(u.b, [3, 4, 1, 2])  # self first
    with pytest.raises(ValueError):
        HQ.Task(np.ones((2, 3)), [1])


def test_wbc_tasks_follow_wbc_cpp():
    s = W.synth_wbc(4)
    levels = W.wbc_tasks(s["M"], s["nle"], s["J"], s["dJv"], (1, 0, 0, 1), s["base_accel"], s["swing_acc"],
                         s["forces_des"], padded=False)
    t0, t1, t2 = levels
    # level 0: EoM [M, -J', -S'] x = -nle (wbc.cpp:102-115), then swing-force rows, then stance contact rows
    assert t0.a.shape == (30, 42) and np.array_equal(t0.a[:18, :18], s["M"])
    assert np.array_equal(t0.a[:18, 18:30], -s["J"].T) and np.array_equal(t0.a[:18, 30:], -np.vstack(
        [np.zeros((6, 12)), np.eye(12)]))
    assert np.array_equal(t0.b[:18], -s["nle"])
    assert np.array_equal(t0.a[18:21, 21:24], np.eye(3)) and np.array_equal(t0.a[21:24, 24:27], np.eye(3))
    assert np.array_equal(t0.a[24:27, :18], s["J"][0:3]) and np.array_equal(t0.b[27:30], -s["dJv"][9:12])
    # inequalities: +-tau <= 33.5, pyramids of stance legs 0 and 3, then 3 zero rows per swing leg
    assert t0.d.shape == (24 + 10 + 6, 42) and np.all(t0.f[:24] == 33.5)
    assert np.array_equal(t0.d[24:29, 18:21], W.FRICTION_PYRAMID(0.3))
    assert np.array_equal(t0.d[29:34, 27:30], W.FRICTION_PYRAMID(0.3)) and not np.any(t0.d[34:])
    # level 1: base acceleration then swing legs 1, 2; level 2: contact forces
    assert t1.a.shape == (12, 42) and np.array_equal(t1.a[:6, :6], np.eye(6))
    assert np.array_equal(t1.b[6:9], s["swing_acc"][1] - s["dJv"][3:6])
    assert np.array_equal(t2.a[:, 18:30], np.eye(12)) and np.array_equal(t2.b, s["forces_des"])


def test_wbc_padding_is_inert_on_the_restatement():
    """The padded batch layout (zero rows) gives the reference layout's solution (oracle/hoqp.py): the same
    x, the same slacks on the torque and pyramid rows, zero slacks on the zero rows."""
    from oracle import hoqp as Q

    for seed in (1, 7):
        sol = []
        for padded in (False, True):
            lv = []
            for t in W.synth_wbc_tasks(seed, padded=padded):
                lv.append(Q.HoQp(Q.Task(t.a, t.b, t.d, t.f), lv[-1] if lv else None))
            sol.append((lv[-1].solution(), lv[0].w_sol))
        nc = sum(W.synth_wbc(seed)["contact"])
        live = 24 + 5 * nc
        assert np.allclose(sol[0][0], sol[1][0], atol=1e-9)
        assert np.allclose(sol[0][1][:live], sol[1][1][:live], atol=1e-12)
        assert not np.any(sol[0][1][live:]) and not np.any(sol[1][1][live:])


def test_golden_fixture_is_certified():
    """The committed expected values satisfy every level's KKT conditions (re-solved here) and the reference
    test's properties on its own data."""
    from oracle import hoqp as Q

    d = np.load(os.path.join(GOLDEN, "hoqp_golden.npz"), allow_pickle=False)
    dims = d["ref_dims"]
    assert list(dims[:2]) == [4, 2]
    t0, t1 = Q.reference_test_tasks()
    h0 = Q.HoQp(t0)
    h1 = Q.HoQp(t1, h0)
    assert np.allclose(d["ref_x"][0, 0], h0.solution(), atol=1e-12)
    assert np.allclose(d["ref_x"][0, 1], h1.solution(), atol=1e-12)
    assert np.allclose(d["ref_w"][0], h1.stacked_slack, atol=1e-12)
    assert d["wbc_rec"].shape == (16, 4472) and bool(d["wbc_pinned"])


def test_wbc_task_assembly_native_matches_formulation():
    """lmpc_wbc_tasks (C, the device kernel's restatement) == wbc.wbc_tasks packed, bitwise, for every one of
    the 16 contact patterns (flight and single-leg stance included) on synthetic dynamics."""
    assert ctypes.sizeof(N.LmpcWbcInput) == 4848
    s = W.synth_wbc(3)
    for mask in range(16):
        contact = [(mask >> i) & 1 for i in range(4)]
        tasks = W.wbc_tasks(s["M"], s["nle"], s["J"], s["dJv"], contact, s["base_accel"], s["swing_acc"],
                            s["forces_des"])
        rec = HQ.pack(tasks, HQ.dims_of(tasks))
        nat = W.record_native(W.wbc_input(s["M"], s["nle"], s["J"], s["dJv"], contact, s["base_accel"],
                                          s["swing_acc"], s["forces_des"]))
        assert np.array_equal(rec, nat), (mask, np.nonzero(rec != nat)[0][:8])
    assert N.lib().lmpc_wbc_tasks(None, None) == -1


def test_cpp_hoqp_mirror_builds():
    """include/lmpc/HoQp.hpp (the C++ mirror of task.h / HoQp.h) compiles with the reference test's program."""
    from legged_mpc_control_amd import build as B

    exe = B.build_cpp_hoqp_test()
    assert os.path.exists(exe) and os.access(exe, os.X_OK)

"""Whole-body-control task formulation for the hierarchical QP.

Mirrors `Wbc::update` (src/legged_ctrl/src/wbc_ctrl/wbc.cpp:37-100) from the point where the reference has its
dynamics terms: the mass matrix M, the nonlinear effects h, the contact Jacobians J and their time variation
times v (dJ v) come from Pinocchio there (wbc.cpp:59-91) and are inputs here.  Decision variables (wbc.h:18):
x = [qdd (18), F (12), tau (12)], n = 42.

    level 0 = floating-base EoM + torque limits + friction cone + no-contact motion   (wbc.cpp:93-94)
    level 1 = base acceleration + swing-leg acceleration                              (wbc.cpp:95)
    level 2 = contact forces                                                          (wbc.cpp:96)

Tasks are `hoqp.Task`.  Rows are the reference's, in its order.  The batch layout has fixed row counts per level (`WBC_DIMS`), so two
kinds of all-zero rows pad the variable-size blocks, both inert (a zero equality row adds nothing to A'A or
A'b and does not change the FullPivLU kernel; a zero inequality row 0 <= 0 + w has the optimal slack w = 0):
level 0's inequality block is [24 torque rows; 5 pyramid rows per stance leg; zeros] (the reference already
pads its friction block with 3 zero rows per swing leg, wbc.cpp:166-172; here with 5), and level 1's equality
block is padded to 6 + 12 rows.  Host-side NumPy (input assembly, not the hot path).
"""
from __future__ import annotations

import numpy as np

from .hoqp import Task

WBC_RECORD_LEN = 4472  # doubles per WBC chain record (lmpc_hoqp_record_len of lmpc_hoqp_dims_wbc)

NQ = 18            # generalized coordinates (6 base + 12 joints)
NF = 12            # 4 three-dof contacts
NTAU = 12          # actuated joints
WBC_N = NQ + NF + NTAU
WBC_EQ_ROWS = (30, 18, 12)
WBC_INEQ_ROWS = (44, 0, 0)
TORQUE_LIMITS = (33.5, 33.5, 33.5)  # config/task.info:226-231 (HAA HFE KFE)
FRICTION_COEFF = 0.3                # config/task.info:233-236
SWING_KP, SWING_KD = 350.0, 37.0    # config/task.info:238-242

# wbc.cpp:162-164, rows on (fx, fy, fz) of one contact
FRICTION_PYRAMID = lambda mu: np.array([[0, 0, -1], [1, 0, -mu], [-1, 0, -mu], [0, 1, -mu], [0, -1, -mu]],
                                       dtype=np.float64)


def swing_accel(p_des, p, v_des, v, kp=SWING_KP, kd=SWING_KD):
    """wbc.cpp:239: commanded swing-foot acceleration kp (p_des - p) + kd (v_des - v), per foot (4 x 3)."""
    return kp * (np.asarray(p_des) - np.asarray(p)) + kd * (np.asarray(v_des) - np.asarray(v))


def wbc_tasks(M, nle, J, dJv, contact, base_accel, swing_acc, forces_des, torque_limits=TORQUE_LIMITS,
              mu=FRICTION_COEFF, padded=True):
    """The three task levels of wbc.cpp:93-96 for one robot.  M (18x18), nle (18), J (12x18, LOCAL_WORLD_ALIGNED
    translation rows per foot), dJv (12), contact (4 bools), base_accel (6: the b of formulateBaseAccelTask,
    wbc.cpp:195-203), swing_acc (4x3, swing_accel()), forces_des (12: input_desired.head(12)).
    padded=False returns the reference's exact row counts (they vary with the contact count)."""
    contact = [bool(c) for c in contact]
    nc = sum(contact)
    n = WBC_N
    S_T = np.zeros((NQ, NTAU))
    S_T[6:, :] = np.eye(NTAU)
    # formulateFloatingBaseEomTask (wbc.cpp:102-115): [M, -J', -S'] x = -nle
    eom = Task(np.hstack([M, -J.T, -S_T]), -np.asarray(nle), None, None)
    # formulateTorqueLimitsTask (:117-131): +-tau <= limits
    d = np.zeros((2 * NTAU, n))
    d[:NTAU, NQ + NF:] = np.eye(NTAU)
    d[NTAU:, NQ + NF:] = -np.eye(NTAU)
    torque = Task(None, None, d, np.tile(np.asarray(torque_limits, dtype=np.float64), 2 * NTAU // 3))
    # formulateFrictionConeTask (:151-175): swing forces = 0; pyramid on stance forces; zero rows after
    a = np.zeros((3 * (4 - nc), n))
    j = 0
    for i in range(4):
        if not contact[i]:
            a[3 * j:3 * j + 3, NQ + 3 * i:NQ + 3 * i + 3] = np.eye(3)
            j += 1
    drows = 5 * 4 if padded else 5 * nc + 3 * (4 - nc)
    d = np.zeros((drows, n))
    j = 0
    for i in range(4):
        if contact[i]:
            d[5 * j:5 * j + 5, NQ + 3 * i:NQ + 3 * i + 3] = FRICTION_PYRAMID(mu)
            j += 1
    friction = Task(a, np.zeros(a.shape[0]), d, np.zeros(drows))
    # formulateNoContactMotionTask (:133-149): J_i qdd = -dJ_i v on stance feet
    a = np.zeros((3 * nc, n))
    b = np.zeros(3 * nc)
    j = 0
    for i in range(4):
        if contact[i]:
            a[3 * j:3 * j + 3, :NQ] = J[3 * i:3 * i + 3]
            b[3 * j:3 * j + 3] = -dJv[3 * i:3 * i + 3]
            j += 1
    nocontact = Task(a, b, None, None)
    # formulateBaseAccelTask (:177-206): qdd_base = b
    a = np.zeros((6, n))
    a[:, :6] = np.eye(6)
    base = Task(a, np.asarray(base_accel, dtype=np.float64), None, None)
    # formulateSwingLegTask (:208-246): J_i qdd = accel_i - dJ_i v on swing feet
    rows = 3 * 4 if padded else 3 * (4 - nc)
    a = np.zeros((rows, n))
    b = np.zeros(rows)
    j = 0
    sw = np.asarray(swing_acc, dtype=np.float64).reshape(4, 3)
    for i in range(4):
        if not contact[i]:
            a[3 * j:3 * j + 3, :NQ] = J[3 * i:3 * i + 3]
            b[3 * j:3 * j + 3] = sw[i] - dJv[3 * i:3 * i + 3]
            j += 1
    swing = Task(a, b, None, None)
    # formulateContactForceTask (:248-259): F = F_des
    a = np.zeros((NF, n))
    a[:, NQ:NQ + NF] = np.eye(NF)
    force = Task(a, np.asarray(forces_des, dtype=np.float64)[:NF], None, None)
    return [eom + torque + friction + nocontact, base + swing, force]


def _skew(r):
    return np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])


GAITS = ((1, 0, 0, 1), (0, 1, 1, 0), (1, 1, 1, 1), (0, 1, 1, 1), (1, 0, 1, 1), (1, 1, 0, 1), (1, 1, 1, 0))


def synth_wbc(seed: int, mass=13.0):
    """Synthetic Go1-scale dynamics terms for one robot (no Pinocchio here): SPD M with the trunk's mass and
    inertia on the base block, gravity in h, foot Jacobians [I, -skew(r_i), J_leg,i] (LOCAL_WORLD_ALIGNED
    translation rows), a trot / stand / crawl contact pattern, targets of the size the controller produces."""
    rng = np.random.default_rng(20261016 + seed)
    B = 0.08 * rng.standard_normal((NQ, NQ))
    base = np.diag([mass, mass, mass, 0.0158533, 0.0377999, 0.0456542])
    M = B.T @ B
    M[:6, :6] += base
    M[6:, 6:] += np.diag(rng.uniform(0.01, 0.05, 12))
    nle = np.concatenate([[0.0, 0.0, mass * 9.81], 0.3 * rng.standard_normal(3), 1.5 * rng.standard_normal(12)])
    J = np.zeros((12, NQ))
    feet = np.array([[0.19, 0.13, -0.3], [0.19, -0.13, -0.3], [-0.19, 0.13, -0.3], [-0.19, -0.13, -0.3]])
    for i in range(4):
        r = feet[i] + rng.uniform(-0.03, 0.03, 3)
        J[3 * i:3 * i + 3, 0:3] = np.eye(3)
        J[3 * i:3 * i + 3, 3:6] = -_skew(r)
        J[3 * i:3 * i + 3, 6 + 3 * i:9 + 3 * i] = 0.25 * rng.standard_normal((3, 3)) + np.diag([0.1, 0.2, 0.2])
    dJv = 0.5 * rng.standard_normal(12)
    contact = GAITS[int(rng.integers(0, len(GAITS)))]
    nc = sum(contact)
    base_accel = np.concatenate([1.0 * rng.standard_normal(3), 2.0 * rng.standard_normal(3)])
    swing_acc = swing_accel(rng.normal(0, 0.02, (4, 3)), np.zeros((4, 3)), rng.normal(0, 0.3, (4, 3)),
                            np.zeros((4, 3)))
    forces = np.zeros(12)
    for i in range(4):
        if contact[i]:
            forces[3 * i:3 * i + 3] = [rng.normal(0, 5), rng.normal(0, 5), mass * 9.81 / nc]
    return dict(M=M, nle=nle, J=J, dJv=dJv, contact=contact, base_accel=base_accel, swing_acc=swing_acc,
                forces_des=forces)


def synth_wbc_tasks(seed: int, padded=True):
    s = synth_wbc(seed)
    return wbc_tasks(s["M"], s["nle"], s["J"], s["dJv"], s["contact"], s["base_accel"], s["swing_acc"],
                     s["forces_des"], padded=padded)


def wbc_input(M, nle, J, dJv, contact, base_accel, swing_acc, forces_des, torque_limits=TORQUE_LIMITS,
              mu=FRICTION_COEFF):
    """The C-ABI's per-robot input block (include/lmpc/lmpc_hoqp.h lmpc_wbc_input)."""
    from ._native import LmpcWbcInput

    s = LmpcWbcInput()
    s.M[:] = list(np.asarray(M, dtype=np.float64).reshape(-1))
    s.nle[:] = list(np.asarray(nle, dtype=np.float64))
    s.J[:] = list(np.asarray(J, dtype=np.float64).reshape(-1))
    s.dJv[:] = list(np.asarray(dJv, dtype=np.float64))
    s.base_accel[:] = list(np.asarray(base_accel, dtype=np.float64))
    s.swing_acc[:] = list(np.asarray(swing_acc, dtype=np.float64).reshape(-1))
    s.forces_des[:] = list(np.asarray(forces_des, dtype=np.float64))
    s.torque_limits[:] = list(np.asarray(torque_limits, dtype=np.float64))
    s.mu = float(mu)
    s.contact[:] = [int(bool(c)) for c in contact]
    return s


def record_native(inp) -> np.ndarray:
    """One WBC record by the product's host restatement (lmpc_wbc_tasks)."""
    import ctypes

    from ._native import check, lib

    rec = np.zeros(WBC_RECORD_LEN)
    check(lib().lmpc_wbc_tasks(ctypes.byref(inp), rec.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
          "lmpc_wbc_tasks")
    return rec


def records_device(d_inputs, d_records, stream=None):
    """A batch of WBC records on the device (lmpc_wbc_tasks_device): d_inputs = uint8 torch tensor [B][sizeof
    lmpc_wbc_input] in HBM, d_records = float64 [B][4472]."""
    import ctypes

    import torch

    from ._native import LmpcWbcInput, check, lib
    from .hoqp import check_device_tensor

    s = stream if stream is not None else torch.cuda.current_stream()
    B = int(d_inputs.shape[0]) if d_inputs.dim() >= 1 else -1
    dev = d_inputs.device if getattr(d_inputs, "is_cuda", False) else torch.device("cuda", torch.cuda.current_device())
    check_device_tensor("d_inputs", d_inputs, torch.uint8, (B, ctypes.sizeof(LmpcWbcInput)), dev)
    check_device_tensor("d_records", d_records, torch.float64, (B, WBC_RECORD_LEN), dev)
    check(lib().lmpc_wbc_tasks_device(ctypes.c_void_p(d_inputs.data_ptr()), d_inputs.shape[0],
                                      ctypes.c_void_p(d_records.data_ptr()), ctypes.c_void_p(s.cuda_stream)),
          "lmpc_wbc_tasks_device")


def synth_input(seed: int):
    s = synth_wbc(seed)
    return wbc_input(s["M"], s["nle"], s["J"], s["dJv"], s["contact"], s["base_accel"], s["swing_acc"],
                     s["forces_des"])

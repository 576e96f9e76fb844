"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The oracle restates the reference's
ConvexQPSolver QP (src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexQPSolver.cpp:
16-346) and solves it exactly (dense Goldfarb-Idnani); see lmpc_oracle.h.
Parity unpinned: the reference has no fixtures for this path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liblmpc_oracle.so")
_lock = threading.Lock()
_lib = None


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("q_weights", ctypes.c_double * 12),
        ("r_weights", ctypes.c_double * 12),
        ("robot_mass", ctypes.c_double),
        ("trunk_inertia", ctypes.c_double * 9),
        ("mu", ctypes.c_double),
        ("f_max", ctypes.c_double),
        ("gravity", ctypes.c_double),
        ("dt", ctypes.c_double),
    ]


class OsqpSettings(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("eps_abs", "eps_rel", "rho", "sigma", "alpha")] + \
               [(k, ctypes.c_int) for k in ("scaling", "max_iter", "check_termination", "adaptive_rho_interval")]


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (make) into oracle/build/ (make rebuilds it when the sources changed)."""
    srcs = [os.path.join(_HERE, f) for f in ("lmpc_oracle.c", "osqp_admm.c", "lmpc_oracle.h")]
    stale = not os.path.exists(_LIB_PATH) or any(
        os.path.exists(s) and os.path.getmtime(s) > os.path.getmtime(_LIB_PATH) for s in srcs)
    if force or stale:
        subprocess.run(["make", "-s", "-C", _HERE] + (["-B"] if force else []), check=True)
    return _LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = ctypes.CDLL(_LIB_PATH)
            dp = ctypes.POINTER(ctypes.c_double)
            u8p = ctypes.POINTER(ctypes.c_uint8)
            i32p = ctypes.POINTER(ctypes.c_int32)
            ip = ctypes.POINTER(ctypes.c_int)
            pp = ctypes.POINTER(OracleParams)
            L.oracle_build_sparse_qp.argtypes = [pp, ctypes.c_int, dp, u8p, dp, dp, dp, dp, dp]
            L.oracle_build_sparse_qp.restype = None
            L.oracle_update_A.argtypes = [ctypes.c_double, ctypes.c_double, dp]
            L.oracle_update_B.argtypes = [pp, dp, dp, dp]
            L.oracle_condense.argtypes = [ctypes.c_int, dp, dp, dp, dp, dp, dp, dp, dp]
            L.oracle_condense.restype = ctypes.c_int
            L.oracle_solve.argtypes = [pp, ctypes.c_int, dp, u8p, dp, dp, ip]
            L.oracle_solve.restype = ctypes.c_int
            L.oracle_solve_batch.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, u8p, dp, i32p, ctypes.c_int]
            L.oracle_solve_batch.restype = ctypes.c_int
            L.oracle_terrain_frame.argtypes = [dp, dp]
            L.oracle_terrain_frame.restype = None
            L.oracle_build_sparse_qp_ex.argtypes = [pp, ctypes.c_int, dp, u8p, dp, dp, dp, dp, dp, dp]
            L.oracle_build_sparse_qp_ex.restype = None
            L.oracle_solve_ex.argtypes = [pp, ctypes.c_int, dp, u8p, dp, dp, dp, ip]
            L.oracle_solve_ex.restype = ctypes.c_int
            L.oracle_solve_batch_ex.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, u8p, dp, dp, i32p, ctypes.c_int]
            L.oracle_solve_batch_ex.restype = ctypes.c_int
            L.oracle_foot_position.argtypes = [dp, dp, dp, dp]
            L.oracle_foot_position.restype = None
            L.oracle_foot_jacobian.argtypes = [dp, dp, dp, dp]
            L.oracle_foot_jacobian.restype = None
            L.oracle_grf_to_torque.argtypes = [dp, dp, dp, dp, dp, dp]
            L.oracle_grf_to_torque.restype = None
            L.oracle_gi_solve.argtypes = [ctypes.c_int, dp, dp, ctypes.c_int, dp, dp, dp, dp, ip]
            L.oracle_gi_solve.restype = ctypes.c_int
            L.oracle_predict_contact.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double]
            L.oracle_predict_contact.restype = ctypes.c_int
            L.oracle_current_contact.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
            L.oracle_current_contact.restype = ctypes.c_int
            sp = ctypes.POINTER(OsqpSettings)
            L.oracle_osqp_settings_default.argtypes = [sp]
            L.oracle_osqp_settings_default.restype = None
            L.oracle_osqp_solve.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, sp, dp, ip, ip, dp]
            L.oracle_osqp_solve.restype = ctypes.c_int
            L.oracle_osqp_grf_batch.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, u8p, dp, sp, dp, i32p, i32p,
                                                ctypes.c_int]
            L.oracle_osqp_grf_batch.restype = ctypes.c_int
            _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def make_params(q_weights, r_weights, robot_mass=13.0, trunk_inertia=None, mu=0.3, f_max=180.0,
                gravity=9.8, dt=0.01) -> OracleParams:
    p = OracleParams()
    for i in range(12):
        p.q_weights[i] = float(q_weights[i])
        p.r_weights[i] = float(r_weights[i])
    p.robot_mass = float(robot_mass)
    I = np.diag([0.0158533, 0.0377999, 0.0456542]) if trunk_inertia is None else np.asarray(trunk_inertia)
    for i, v in enumerate(np.asarray(I, dtype=np.float64).reshape(9)):
        p.trunk_inertia[i] = float(v)
    p.mu, p.f_max, p.gravity, p.dt = float(mu), float(f_max), float(gravity), float(dt)
    return p


def params_from(struct) -> OracleParams:
    """Copy any ctypes struct with the lmpc_params field layout."""
    p = OracleParams()
    ctypes.memmove(ctypes.byref(p), ctypes.byref(struct), ctypes.sizeof(OracleParams))
    return p


def _normals(normals, lead=()):
    """None (flat ground, the reference) or a contiguous float64 [..., 4, 3] array."""
    if normals is None:
        return None, None
    a = np.ascontiguousarray(normals, dtype=np.float64).reshape(tuple(lead) + (4, 3))
    return a, _dp(a)


def terrain_frame(n) -> np.ndarray:
    """Contact frame R (columns t1, t2, n) of a ground normal; R = I for n = e_z."""
    n = np.ascontiguousarray(n, dtype=np.float64).reshape(3)
    R = np.zeros(9)
    lib().oracle_terrain_frame(_dp(n), _dp(R))
    return R.reshape(3, 3)


def build_sparse_qp(p: OracleParams, H: int, rec: np.ndarray, contact: np.ndarray, normals=None):
    n, m = 24 * H, 32 * H
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    nrm, nrm_p = _normals(normals)
    P = np.zeros(n); q = np.zeros(n); A = np.zeros((m, n)); l = np.zeros(m); u = np.zeros(m)
    lib().oracle_build_sparse_qp_ex(ctypes.byref(p), H, _dp(rec), _u8p(contact), nrm_p,
                                    _dp(P), _dp(q), _dp(A), _dp(l), _dp(u))
    return P, q, A, l, u


def condense(H: int, P, q, A, l):
    N = 12 * H
    Hc = np.zeros((N, N)); g = np.zeros(N); T = np.zeros((12 * H, N)); c = np.zeros(12 * H)
    rc = lib().oracle_condense(H, _dp(np.ascontiguousarray(P)), _dp(np.ascontiguousarray(q)),
                               _dp(np.ascontiguousarray(A)), _dp(np.ascontiguousarray(l)),
                               _dp(Hc), _dp(g), _dp(T), _dp(c))
    if rc != 0:
        raise RuntimeError(f"oracle_condense failed: {rc}")
    return Hc, g, T, c


def solve(p: OracleParams, H: int, rec: np.ndarray, contact: np.ndarray, normals=None):
    """Exact optimum of one instance -> (grf[H,12], kkt[4], n_active).  normals[4,3] or None (flat)."""
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    nrm, nrm_p = _normals(normals)
    grf = np.zeros(12 * H); kkt = np.zeros(4); na = ctypes.c_int(0)
    rc = lib().oracle_solve_ex(ctypes.byref(p), H, _dp(rec), _u8p(contact), nrm_p, _dp(grf), _dp(kkt),
                               ctypes.byref(na))
    if rc != 0:
        raise RuntimeError(f"oracle_solve failed: {rc}")
    return grf.reshape(H, 12), kkt, na.value


def solve_batch(p: OracleParams, H: int, rec: np.ndarray, contact: np.ndarray, n_threads: int = 1, normals=None):
    B = rec.shape[0]
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    nrm, nrm_p = _normals(normals, (B,))
    grf = np.zeros((B, H, 12)); status = np.zeros(B, dtype=np.int32)
    fails = lib().oracle_solve_batch_ex(ctypes.byref(p), H, B, _dp(rec), _u8p(contact), nrm_p, _dp(grf),
                                        status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n_threads)
    return grf, status, fails


def gi_solve(G, g0, CI, ci0):
    """min 1/2 x'Gx + g0'x  s.t. CI x + ci0 >= 0 (CI rows = constraints)."""
    G = np.ascontiguousarray(G, dtype=np.float64)
    n = G.shape[0]
    CI = np.ascontiguousarray(CI, dtype=np.float64)
    m = CI.shape[0]
    x = np.zeros(n); lam = np.zeros(max(m, 1)); na = ctypes.c_int(0)
    rc = lib().oracle_gi_solve(n, _dp(G), _dp(np.ascontiguousarray(g0, dtype=np.float64)), m, _dp(CI),
                               _dp(np.ascontiguousarray(ci0, dtype=np.float64)), _dp(x), _dp(lam), ctypes.byref(na))
    return rc, x, lam[:m], na.value


def predict_contact(gait: int, leg: int, phase: float, speed: float, dt: float) -> int:
    return lib().oracle_predict_contact(gait, leg, phase, speed, dt)


def current_contact(gait: int, leg: int, phase: float) -> int:
    return lib().oracle_current_contact(gait, leg, phase)


def _f64(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if n is None else a.reshape(n)


def foot_position(rho_fix, rho_opt, q) -> np.ndarray:
    p = np.zeros(3)
    lib().oracle_foot_position(_dp(_f64(rho_fix, 5)), _dp(_f64(rho_opt, 3)), _dp(_f64(q, 3)), _dp(p))
    return p


def foot_jacobian(rho_fix, rho_opt, q) -> np.ndarray:
    J = np.zeros(9)
    lib().oracle_foot_jacobian(_dp(_f64(rho_fix, 5)), _dp(_f64(rho_opt, 3)), _dp(_f64(q, 3)), _dp(J))
    return J.reshape(3, 3)


def grf_to_torque(rho_fix, rho_opt, rot, joint_pos, grf0) -> np.ndarray:
    """rho_fix [4,5], rho_opt [4,3], rot [3,3] row-major, joint_pos [12], grf0 [12] -> tau [12]."""
    tau = np.zeros(12)
    rf, ro = _f64(rho_fix, 20), _f64(rho_opt, 12)
    lib().oracle_grf_to_torque(_dp(rf), _dp(ro), _dp(_f64(rot, 9)), _dp(_f64(joint_pos, 12)), _dp(_f64(grf0, 12)),
                               _dp(tau))
    return tau


def osqp_settings(**kw) -> OsqpSettings:
    """The reference's OSQP settings (ConvexQPSolver.cpp:182-194 + OSQP 0.6 defaults), fields overridable."""
    s = OsqpSettings()
    lib().oracle_osqp_settings_default(ctypes.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def osqp_solve(P_diag, q, A, l, u, **kw):
    """C restatement of OSQP's ADMM (osqp_admm.c) on one QP -> (x, iters, converged, [prim, dual, rho])."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    m, n = A.shape
    x = np.zeros(n); info = np.zeros(3); it = ctypes.c_int(0); cv = ctypes.c_int(0)
    rc = lib().oracle_osqp_solve(n, m, _dp(_f64(P_diag)), _dp(_f64(q)), _dp(A), _dp(_f64(l)), _dp(_f64(u)),
                                 ctypes.byref(osqp_settings(**kw)), _dp(x), ctypes.byref(it), ctypes.byref(cv), _dp(info))
    if rc != 0:
        raise RuntimeError(f"oracle_osqp_solve failed: {rc}")
    return x, it.value, bool(cv.value), info


def osqp_grf_batch(p: OracleParams, H: int, rec, contact, n_threads: int = 1, normals=None, **kw):
    """The reference's compute_grfs (OSQP ADMM at its settings) over a batch -> (grf [B,H,12], iters, converged)."""
    B = rec.shape[0]
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    nrm, nrm_p = _normals(normals, (B,))
    grf = np.zeros((B, H, 12)); it = np.zeros(B, dtype=np.int32); cv = np.zeros(B, dtype=np.int32)
    i32 = ctypes.POINTER(ctypes.c_int32)
    lib().oracle_osqp_grf_batch(ctypes.byref(p), H, B, _dp(rec), _u8p(contact), nrm_p, ctypes.byref(osqp_settings(**kw)),
                                _dp(grf), it.ctypes.data_as(i32), cv.ctypes.data_as(i32), n_threads)
    return grf, it, cv.astype(bool)

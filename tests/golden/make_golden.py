#!/usr/bin/env python3
"""Generate and certify the golden fixtures in tests/golden/ (run in the build
container; the fixtures are committed, the GPU box only reads them).

For every instance:
  1. inputs come from the product's seeded generator (lmpc_synth_fill) or are
     hand-built edge cases;
  2. an INDEPENDENT numpy restatement of the reference's sparse OSQP problem
     (ConvexQPSolver.cpp:16-346, written here from the reference text, not
     from the C oracle) must equal the oracle's assembly exactly;
  3. the oracle's solution (dense Goldfarb-Idnani on the condensed QP) is
     certified optimal for the SPARSE reference form by a KKT certificate:
     multipliers y with the OSQP sign pattern from a bounded least-squares fit,
     stationarity residual || P z + q + A'y || / scale <= 1e-8;
  4. inputs, expected GRFs and the certificate are written to golden_*.npz.

The reference itself cannot be built or run here (Eigen3, OsqpEigen, OSQP and
ROS are absent), so parity is pinned by this certificate, not by reference
outputs ("parity unpinned" with respect to reference-produced vectors).
"""
from __future__ import annotations

import os
import sys

import numpy as np
from scipy.optimize import lsq_linear

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from legged_mpc_control_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

INF = 1e30


# ---------------------------------------------------------------------------
# independent numpy restatement of the reference QP (ConvexQPSolver.cpp)
# ---------------------------------------------------------------------------
def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def rodrigues_frame(n):
    """Terrain extension: rotation about axis e_z x n by angle acos(n_z) (Rodrigues' formula),
    the independent restatement of lmpc_terrain_frame / oracle_terrain_frame."""
    n = np.asarray(n, dtype=np.float64) / np.linalg.norm(n)
    ax = np.cross([0.0, 0.0, 1.0], n)
    s = np.linalg.norm(ax)
    if s == 0.0:
        return np.eye(3)
    k = ax / s
    K = skew(k)
    th = np.arctan2(s, n[2])
    return np.eye(3) + np.sin(th) * K + (1.0 - np.cos(th)) * (K @ K)


def ref_sparse_qp(q_w, r_w, mass, Ib, mu, fmax, g, dt, H, rec, contact, normals=None):
    nx = nu = 12
    n, m = (nx + nu) * H, (nx + 16 + 4) * H
    dyn, fric = nx * H, 16 * H
    x0 = rec[0:12]
    R = rec[12:21].reshape(3, 3)
    feet = rec[21:33].reshape(4, 3).T  # 3 x 4 like foot_pos_abs
    xref = rec[33:].reshape(H, 12)
    P = np.zeros(n)
    for i in range(H):
        P[24 * i:24 * i + 12] = r_w
        P[24 * i + 12:24 * i + 24] = q_w
    q = np.zeros(n)
    A = np.zeros((m, n))
    l = np.zeros(m)
    u = np.zeros(m)
    # B (update_B_matrix)
    Iw = R @ Ib @ R.T
    Bc = np.zeros((12, 12))
    for j in range(4):
        Bc[6:9, 3 * j:3 * j + 3] = np.linalg.inv(Iw) @ skew(feet[:, j])
        Bc[9:12, 3 * j:3 * j + 3] = np.eye(3) / mass
    Bd = Bc * dt
    for i in range(H):
        yaw = xref[i, 2]
        Ac = np.zeros((12, 12))
        Ac[0:3, 6:9] = np.array([[np.cos(yaw), np.sin(yaw), 0], [-np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
        Ac[3:6, 9:12] = np.eye(3)
        Ad = np.eye(12) + Ac * dt
        A[12 * i:12 * i + 12, 24 * i:24 * i + 12] = Bd
        A[12 * i:12 * i + 12, 24 * i + 12:24 * i + 24] = -np.eye(12)
        if i == 0:
            u[0:12] = -Ad @ x0
            u[11] += g * dt
            l[0:12] = u[0:12]
        else:
            A[12 * i:12 * i + 12, 24 * i - 12:24 * i] = Ad
            l[12 * i + 11] = u[12 * i + 11] = g * dt
        q[24 * i + 12:24 * i + 24] = -q_w * xref[i]
        for j in range(4):
            rr = dyn + 16 * i + 4 * j
            c = 24 * i + 3 * j
            # pyramid rows on the contact-frame force g = Rn' f (Rn = I: the reference rows)
            Rn = np.eye(3) if normals is None else rodrigues_frame(normals[j])
            C = np.array([[1, 0, mu], [1, 0, -mu], [0, 1, mu], [0, 1, -mu], [0, 0, 1.0]]) @ Rn.T
            A[rr:rr + 4, c:c + 3] = C[:4]
            l[rr:rr + 4] = [0, -INF, 0, -INF]
            u[rr:rr + 4] = [INF, 0, INF, 0]
            b = dyn + fric + 4 * i + j
            A[b, c:c + 3] = C[4]
            l[b] = 0
            u[b] = fmax * contact[i, j]
    return P, q, A, l, u


def kkt_certificate(P, q, A, l, u, grf, H):
    """Certify z (states from the dynamics rows) for the sparse QP; returns scaled residual."""
    n = P.shape[0]
    dyn = 12 * H
    z = np.zeros(n)
    # states from the dynamics: A_dyn z = l_dyn, solve for x given u
    for i in range(H):
        z[24 * i:24 * i + 12] = grf[i]
    for i in range(H):
        rows = A[12 * i:12 * i + 12]
        rhs = l[12 * i:12 * i + 12] - rows[:, 24 * i:24 * i + 12] @ z[24 * i:24 * i + 12]
        if i > 0:
            rhs -= rows[:, 24 * i - 12:24 * i] @ z[24 * i - 12:24 * i]
        z[24 * i + 12:24 * i + 24] = -rhs  # coefficient of x_{i+1} is -I
    Az = A @ z
    tol = 1e-7 * (1 + np.abs(Az))
    lo = np.full(A.shape[0], 0.0)
    hi = np.full(A.shape[0], 0.0)
    for i in range(A.shape[0]):
        at_u = u[i] < INF / 2 and Az[i] >= u[i] - tol[i]
        at_l = l[i] > -INF / 2 and Az[i] <= l[i] + tol[i]
        if i < dyn or (at_u and at_l):
            lo[i], hi[i] = -np.inf, np.inf
        elif at_u:
            lo[i], hi[i] = 0.0, np.inf
        elif at_l:
            lo[i], hi[i] = -np.inf, 0.0
        else:
            lo[i], hi[i] = -1e-300, 1e-300
    # primal feasibility
    viol = max(0.0, float(np.max(np.where(u < INF / 2, Az - u, -np.inf))),
               float(np.max(np.where(l > -INF / 2, l - Az, -np.inf))))
    g = P * z + q
    active = hi - lo > 1e-200
    At = A[active].T
    res = lsq_linear(At, -g, bounds=(lo[active], hi[active]), lsmr_tol="auto", method="bvls", tol=1e-14)
    stat = np.max(np.abs(At @ res.x + g)) / max(1.0, np.max(np.abs(g)))
    return stat, viol / max(1.0, np.max(np.abs(grf)))


# ---------------------------------------------------------------------------
def make_set(name, p, H, rec, con, meta, normals=None):
    op = O.params_from(p)
    qw, rw = np.array(p.q_weights[:]), np.array(p.r_weights[:])
    Ib = np.array(p.trunk_inertia[:]).reshape(3, 3)
    grfs, kkts, nacts, certs = [], [], [], []
    for b in range(rec.shape[0]):
        nb = None if normals is None else normals[b]
        Po, qo, Ao, lo, uo = O.build_sparse_qp(op, H, rec[b], con[b], normals=nb)
        Pn, qn, An, ln, un = ref_sparse_qp(qw, rw, p.robot_mass, Ib, p.mu, p.f_max, p.gravity, p.dt, H, rec[b], con[b],
                                           normals=nb)
        for a, c, what in ((Po, Pn, "P"), (qo, qn, "q"), (Ao, An, "A"), (lo, ln, "l"), (uo, un, "u")):
            err = np.max(np.abs(a - c) / np.maximum(1.0, np.abs(c)))
            assert err < 1e-13, f"{name}[{b}]: oracle assembly differs from numpy restatement in {what}: {err}"
        grf, kkt, na = O.solve(op, H, rec[b], con[b], normals=nb)
        stat, viol = kkt_certificate(Pn, qn, An, ln, un, grf, H)
        assert stat < 1e-8 and viol < 1e-9, f"{name}[{b}]: KKT certificate failed stat={stat} viol={viol}"
        grfs.append(grf)
        kkts.append(kkt)
        nacts.append(na)
        certs.append([stat, viol])
    out = os.path.join(HERE, f"golden_{name}.npz")
    params = np.concatenate([p.q_weights[:], p.r_weights[:], [p.robot_mass], p.trunk_inertia[:],
                             [p.mu, p.f_max, p.gravity, p.dt]])
    extra = {} if normals is None else {"normals": np.asarray(normals, dtype=np.float64)}
    np.savez_compressed(out, H=np.int64(H), params=params, rec=rec, contact=con, grf=np.array(grfs),
                        kkt=np.array(kkts), n_active=np.array(nacts), certificate=np.array(certs),
                        meta=np.array(meta), **extra)
    print(f"{out}: {rec.shape[0]} instances, max certificate {np.max(certs):.2e}")


def edge_cases(p, H):
    """Hand-built edge cases: swing steps, all-swing, stand, single stance leg,
    friction-boundary push, f_max-bound push, lift-off."""
    cfg = synth.synth_cfg("go1", 0)
    rec, con = synth.fill(p, cfg, H, 8, seed=4242)
    rec = rec.copy()
    con = con.copy()
    meta = []
    con[0, 3:5, :] = 0; meta.append("all-swing steps 3,4")
    con[1, :, :] = 0; meta.append("all legs swing over the whole horizon -> u = 0")
    con[2, :, :] = 1; meta.append("stand (all stance)")
    con[3, :, :] = 0; con[3, :, 1] = 1; meta.append("single stance leg (FR)")
    # lateral push: large desired lateral velocity -> friction cone active
    R = rec[4, 12:21].reshape(3, 3)
    vd = R @ np.array([0.0, 3.0, 0.0])
    for i in range(H):
        rec[4, 33 + 12 * i + 4] = rec[4, 3 + 1] + vd[1] * p.dt * i
        rec[4, 33 + 12 * i + 9:33 + 12 * i + 11] = vd[:2]
    con[4, :, :] = 1
    meta.append("lateral push, stance: friction pyramid active")
    # upward push: far-too-low body with downward velocity -> fz = f_max active
    rec[5, 5] = 0.10
    rec[5, 11] = -2.0
    for i in range(H):
        rec[5, 33 + 12 * i + 5] = 0.60
    con[5, :, :] = 1
    meta.append("upward push: fz = f_max active")
    # lift-off: body too high and moving up -> legs want to pull -> f = 0 apex
    rec[6, 5] = 0.60
    rec[6, 11] = 1.5
    for i in range(H):
        rec[6, 33 + 12 * i + 5] = 0.20
    meta.append("lift-off: pyramid apex (f = 0) on stance legs")
    meta.append("regular trot instance")
    return rec, con, meta


def main():
    # config 1: A1 standing, H=10, batch 1 (CPU plumbing config)
    p1, H1, rec1, con1 = synth.config_batch(1)
    make_set("config1_a1_standing_h10", p1, H1, rec1, con1, ["A1 standing, FSM reset, trot prediction for i>=1"])
    # configs 2/3/5 (Go1 trot) and 4 (mixed gaits), 16 instances each, global indices 0..15
    for cid, cnt in ((2, 16), (3, 12), (4, 16), (5, 8)):
        p, H, rec, con = synth.config_batch(cid, count=cnt)
        make_set(f"config{cid}_{synth.CONFIGS[cid]['name']}", p, H, rec, con,
                 [f"{synth.CONFIGS[cid]['name']} global index {i}" for i in range(cnt)])
    # config 4 with its terrain normals (extension; parity vs this build's oracle only)
    p4, H4, rec4, con4 = synth.config_batch(4, count=16)
    nrm4 = synth.config_normals(4, count=16)
    for n in nrm4.reshape(-1, 3):  # the product's frame equals the Rodrigues restatement
        assert np.max(np.abs(synth.terrain_frame(n) - rodrigues_frame(n))) < 1e-15
    make_set("config4t_go1_mixed_terrain_h10", p4, H4, rec4, con4,
             [f"go1_mixed_h10_b65536 + terrain normals, global index {i}" for i in range(16)], normals=nrm4)
    # terrain edge cases: steep tilt (theta = 0.6) so friction faces bind, and flat normals (= reference)
    rec_e, con_e, meta_e = edge_cases(synth.params("go1"), 10)
    nrm_e = synth.normals(rec_e.shape[0], 777, theta_max=0.6)
    nrm_e[7] = [0.0, 0.0, 1.0]
    meta_e = [m + " + steep terrain (theta <= 0.6)" for m in meta_e[:7]] + ["regular trot, flat normals (= reference)"]
    make_set("edge_go1_terrain_h10", synth.params("go1"), 10, rec_e, con_e, meta_e, normals=nrm_e)
    p = synth.params("go1")
    for H in (10, 30):
        rec, con, meta = edge_cases(p, H)
        make_set(f"edge_go1_h{H}", p, H, rec, con, meta)


if __name__ == "__main__":
    main()

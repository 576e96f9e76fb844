"""CPU check of the dense polish's range-space (bordered) round update (lmpc_dense_kernel.h: schur_leg and the
`schur` branch of dense_body), restated in numpy: a polish round whose faces differ from the last factorised round's
is solved from that factorisation -- new free directions as columns, added faces (or u = 0 at a new apex) as rows,
K s = c - V'y0 with K = Cb - V'M^-1 V quasi-definite -- and must equal the round's direct equality-constrained solve.
Random SPD Hessians over six leg-steps; every transition kind the kernel qualifies is exercised."""
import itertools

import numpy as np

MU, FMAX = 0.6, 150.0


def rowvec(i):  # cons_rowvec (lmpc_kernel_common.h)
    return np.array([-1.0 if i == 0 else 1.0 if i == 1 else 0.0, -1.0 if i == 2 else 1.0 if i == 3 else 0.0,
                     1.0 if i == 4 else -MU])


def beta(i):
    return FMAX if i == 4 else 0.0


def is_apex(a):
    return (a & 3) == 3 or (a & 12) == 12


def leg_basis(a):
    """T (3x3, orthonormal nonzero columns first) and up (min-norm particular solution); apex: zeros."""
    T, up = np.zeros((3, 3)), np.zeros(3)
    if is_apex(a):
        return T, up, True
    faces = [i for i in range(5) if (a >> i) & 1][:3]
    if not faces:
        return np.eye(3), up, False
    R = np.array([rowvec(i) for i in faces])
    b = np.array([beta(i) for i in faces])
    up = np.linalg.lstsq(R, b, rcond=None)[0]
    _, sv, vt = np.linalg.svd(R)
    ns = vt[int(np.sum(sv > 1e-12)):].T
    T[:, :ns.shape[1]] = ns
    return T, up, False


def ncols(T):
    return int(np.sum(np.abs(T).sum(0) > 0))


def factorised(Hm, g, act):
    n = len(act)
    Tb, upv = np.zeros((3 * n, 3 * n)), np.zeros(3 * n)
    for b, a in enumerate(act):
        T, up, _ = leg_basis(a)
        Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3] = T
        upv[3 * b:3 * b + 3] = up
    M = Tb.T @ Hm @ Tb
    fixed = np.where(np.abs(Tb).sum(0) == 0)[0]
    M[fixed, fixed] += 1.0
    y = np.linalg.solve(M, -Tb.T @ (Hm @ upv + g))
    return Tb, upv, M, y


def direct(Hm, g, act):
    Tb, upv, _, y = factorised(Hm, g, act)
    return upv + Tb @ y


def schur_leg(a, b):
    """(kc, kr, ok) of one changed leg-step, as schur_leg in lmpc_dense_kernel.h."""
    bap, nap = is_apex(b), is_apex(a)
    if bap and nap:
        return 0, 0, True
    cm = a & b
    Tc, _, _ = leg_basis(cm)
    Tb, _, _ = leg_basis(b)
    Tn, _, _ = leg_basis(a)
    nb, nc, nn = ncols(Tb), ncols(Tc), ncols(Tn)
    kc = nc - nb
    kr = nc if nap else bin(a & ~b).count("1")
    ok = 0 <= kc <= 3 and kr <= 3 and (not bap or not cm & 16) and (not nap or not (a | b) & 16) and (nap or nn == nc - kr)
    return kc, kr, ok


def bordered(Hm, g, bact, act):
    """The kernel's update of the factorised round `bact` to the round `act`; None where a refactorisation runs."""
    n = len(act)
    Tb, upv, M, y0 = factorised(Hm, g, bact)
    hg = Hm @ upv + g
    ents = []  # (kind, leg, vec3, scalar)
    for b, (a, a0) in enumerate(zip(act, bact)):
        if a == a0:
            continue
        kc, kr, ok = schur_leg(a, a0)
        if not ok:
            return None
        if kc == 0 and kr == 0:
            continue
        Tl = Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3]
        Tc, _, _ = leg_basis(a & a0)
        nb = ncols(Tl)
        if nb == 0:
            tv = [Tc[:, j] for j in range(3)]
        elif kc == 0:
            tv = []
        else:
            res = [Tc[:, q] - Tl @ (Tl.T @ Tc[:, q]) for q in range(3)]
            t0 = max(res, key=lambda r: r @ r)
            t0 = t0 / np.linalg.norm(t0)
            tv = [t0, np.cross(Tl[:, 0], t0)]
        for j in range(kc):
            ents.append(("col", b, tv[j], -tv[j] @ hg[3 * b:3 * b + 3]))
        if is_apex(a):
            rows = [(Tc[:, q], 0.0) for q in range(kr)]
        else:
            rows = [(rowvec(i), beta(i)) for i in range(5) if (a >> i) & 1 and not (a0 >> i) & 1]
        up = upv[3 * b:3 * b + 3]
        for r, bv in rows:
            ents.append(("row", b, r, bv - r @ up))
    K = len(ents)
    V = np.zeros((3 * n, K))
    for e, (kind, b, v3, _) in enumerate(ents):
        if kind == "col":
            E = np.zeros(3 * n)
            E[3 * b:3 * b + 3] = v3
            V[:, e] = Tb.T @ (Hm @ E)
        else:
            V[3 * b:3 * b + 3, e] = v3 @ Tb[3 * b:3 * b + 3, 3 * b:3 * b + 3]
    Cb = np.zeros((K, K))
    for i, j in itertools.product(range(K), range(K)):
        ki, bi, vi, _ = ents[i]
        kj, bj, vj, _ = ents[j]
        if ki == "col" and kj == "col":
            Cb[i, j] = vi @ Hm[3 * bi:3 * bi + 3, 3 * bj:3 * bj + 3] @ vj
        elif ki != kj and bi == bj:
            Cb[i, j] = vi @ vj
    W = np.linalg.solve(M, V)
    Km = Cb - V.T @ W
    rhs = np.array([e[3] for e in ents]) - V.T @ y0
    # L D L' without pivoting: positive pivots on the columns, negative on the rows (quasi-definite)
    L, d = np.eye(K), np.zeros(K)
    for c in range(K):
        d[c] = Km[c, c] - np.sum(L[c, :c] ** 2 * d[:c])
        for r in range(c + 1, K):
            L[r, c] = (Km[r, c] - np.sum(L[r, :c] * L[c, :c] * d[:c])) / d[c]
    sg = np.array([1.0 if e[0] == "col" else -1.0 for e in ents])
    assert np.all(sg * d > 0), (sg, d)
    s = np.linalg.solve(Km, rhs)
    y = y0 - W @ s
    u = upv + Tb @ y
    for e, (kind, b, v3, _) in enumerate(ents):
        if kind == "col":
            u[3 * b:3 * b + 3] += v3 * s[e]
    for b, a in enumerate(act):
        if is_apex(a):
            u[3 * b:3 * b + 3] = 0.0
    return u, sum(e[0] == "col" for e in ents), K


# the active sets the polish produces: none, one or two pyramid faces (adjacent), the f_max cap with those, apexes
SETS = [0, 1, 2, 4, 8, 16, 1 | 4, 1 | 8, 2 | 4, 2 | 8, 1 | 16, 2 | 16, 4 | 16, 8 | 16, 3, 12, 15, 1 | 4 | 16,
        2 | 8 | 16]


def test_bordered_round_equals_direct_solve():
    rng = np.random.default_rng(7)
    n = 6
    kinds = {"rows only": 0, "with columns": 0, "apex": 0, "refactor": 0}
    for trial in range(400):
        A = rng.standard_normal((3 * n, 3 * n))
        Hm = A @ A.T + 0.5 * np.eye(3 * n)
        g = rng.standard_normal(3 * n) * 50.0
        bact = [int(rng.choice(SETS)) for _ in range(n)]
        act = list(bact)
        for b in rng.choice(n, size=int(rng.integers(1, 3)), replace=False):
            act[b] = int(rng.choice(SETS))
        out = bordered(Hm, g, bact, act)
        if out is None:
            kinds["refactor"] += 1
            continue
        u, ncol, K = out
        ud = direct(Hm, g, act)
        assert np.max(np.abs(u - ud)) <= 1e-8 * max(1.0, np.max(np.abs(ud))), (bact, act)
        kinds["with columns" if ncol else "rows only"] += 1
        kinds["apex"] += any(is_apex(a) != is_apex(b) for a, b in zip(act, bact))
    assert kinds["rows only"] > 20 and kinds["with columns"] > 20 and kinds["apex"] > 10, kinds

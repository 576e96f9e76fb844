"""The useful-flop models of roofline.py pinned by a counted restatement.

roofline.lq_flop (the LDS Riccati kernel) and roofline.dense_flop (the condensed dense interior point) price the
headline fractions of the bench line from hand tallies of each formulation's operations (roofline.py:24-83).  Here the
operations are restated in numpy on matrices with the kernels' nonzero structure -- every product counted as it is
executed (one multiply per structural term, FMA = 2 flops, a lone multiply or division 1, a sqrt / reciprocal 1) --
and the restatements are checked for what they compute (the Riccati step against the direct formula
P_k = Q + A'PA - A'PB (I + B'PB)^-1 B'PA, the reduced inputs against W = Bt Rr^-1 Bt', the condensed Hessian against
the dense product, the Cholesky and the solves against numpy).  The models must equal the counts within 5 % at
H = 10 / 20 / 30 and at the measured mean iterations, polish rounds and stance counts of the bench configs.
Reference for what is counted: SURVEY.md 8(d); the kernels: csrc/lmpc_lq_kernel.h (header comment), csrc/lmpc_dense.hip.
"""
import numpy as np
import pytest

from legged_mpc_control_amd import roofline

RNG = np.random.default_rng(20261018)


class Flops:
    """Executed flops of a restated computation, counted on the operands' structural nonzeros."""

    def __init__(self):
        self.n = 0

    def mm(self, A, B, lower=False, acc=False):
        """A @ B: t structural terms per output entry -> t multiplies + t - 1 adds (+1 onto an accumulator);
        lower: only the lower triangle is formed (a symmetric result)."""
        t = (A != 0).astype(np.int64) @ (B != 0).astype(np.int64)
        if lower:
            t = np.tril(t)
        self.n += int(np.sum(2 * t - (t > 0)) + (np.count_nonzero(t) if acc else 0))
        return A @ B

    def add(self, k):
        self.n += int(k)

    def chol(self, M):
        """Lower Cholesky, left-looking: per column j one sqrt + reciprocal, j FMAs for the pivot, j FMAs and a
        multiply for each entry below it."""
        n = M.shape[0]
        for j in range(n):
            self.n += 2 + 2 * j + (n - 1 - j) * (2 * j + 1)
        return np.linalg.cholesky(M)

    def trsm_lower(self, L, B):
        """L X = B by forward substitution (reciprocals of the diagonal in hand): per column, row r costs r FMAs
        on the structurally nonzero solution entries above it and one multiply."""
        n, m = B.shape
        X = np.zeros_like(B)
        for c in range(m):
            nz = np.zeros(n, bool)
            for r in range(n):
                k = int(np.count_nonzero(nz[:r] & (L[r, :r] != 0)))
                self.n += 2 * k + 1 if (k or B[r, c] != 0) else 0
                X[r, c] = (B[r, c] - L[r, :r] @ X[:r, c]) / L[r, r]
                nz[r] = k > 0 or B[r, c] != 0
        return X


def spd(n, scale=1.0):
    M = RNG.standard_normal((n, n))
    return scale * (M @ M.T + n * np.eye(n))


def dtN(yaw, dt=0.01):
    """dt N(yaw) = A_k - I (ConvexQPSolver.cpp:214-228): rows 0-2 the yaw rotation on columns 6-8, rows 3-5 the
    identity on columns 9-11 -- 8 structural nonzeros."""
    N = np.zeros((12, 12))
    c, s = np.cos(yaw), np.sin(yaw)
    N[0:3, 6:9] = dt * np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]])
    N[3:6, 9:12] = dt * np.eye(3)
    return N


def g0_block():
    """G0 = B rows 6-11 (ConvexQPSolver.cpp:198-212): dt [I_w^-1 skew(r_j); I/m] per leg."""
    G = np.zeros((6, 12))
    iw = np.linalg.inv(spd(3, 0.01))
    for j in range(4):
        r = RNG.uniform(-0.3, 0.3, 3)
        sk = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
        G[0:3, 3 * j:3 * j + 3] = 0.01 * iw @ sk
        G[3:6, 3 * j:3 * j + 3] = 0.01 / 13.0 * np.eye(3)
    return G


# ---- the LDS Riccati kernel -----------------------------------------------------------------------------------

def riccati_stage_reduced(F, Ph, yaw, U, dv, qw, qcol):
    """One factorisation stage in reduced inputs (csrc/lmpc_lq_kernel.h, interior point): value function of the
    augmented state [x; 1] in P^ (13 x 13), inputs f = U v (rows 6-11, unit cost).  Returns P^_k."""
    Bh = np.zeros((13, 7))
    Bh[6:12, 0:6] = U
    Bh[6:12, 6] = dv
    C = F.mm(Ph[:, 6:12], Bh[6:12, :])                      # C = P^ B^ (column 6: v = P d)
    Guu = np.eye(6) + F.mm(U.T, C[6:12, 0:6], lower=True)    # Guu' = I + U'P22 U
    F.add(6)
    L = F.chol(Guu)
    X = F.trsm_lower(L, U.T)                                 # X = L^-1 U'
    K = F.mm(X.T, X, lower=True)                             # K = U Guu^-1 U' (rows / columns 6-11)
    Nh = np.zeros((13, 13))
    Nh[:12, :12] = dtN(yaw)
    PA = Ph + F.mm(Ph, Nh, acc=True)                         # PA = P^ A^ (the d column from C)
    PA[:, 12] += C[:, 6]
    F.add(13)
    Z = PA[6:12, :]
    KZ = F.mm(K, Z)                                          # K Z
    APA = PA + F.mm(Nh.T, PA, acc=True)                      # A^'P^A^
    Pn = APA - F.mm(Z.T, KZ, lower=True, acc=True)           # - M'K M'
    Pn[np.arange(12), np.arange(12)] += qw
    Pn[:12, 12] += qcol
    Pn[12, :12] += qcol
    F.add(12 + 12)
    return Pn


def direct_riccati(Ph, yaw, U, dv, qw, qcol):
    A = np.eye(13)
    A[:12, :12] += dtN(yaw)
    A[6:12, 12] = dv
    B = np.zeros((13, 6))
    B[6:12] = U
    PA, PB = Ph @ A, Ph @ B
    P = A.T @ PA - (A.T @ PB) @ np.linalg.solve(np.eye(6) + B.T @ PB, PB.T @ A)
    P[np.arange(12), np.arange(12)] += qw
    P[:12, 12] += qcol
    P[12, :12] += qcol
    return P


def riccati_stage_full(F, Ph, yaw, Bt, Rr, rr, dv, qw, qcol, nlegs):
    """One polish factorisation stage in full inputs (two leg-steps per lane, H > 16): C = P^[:,6:12] [Bt | dv],
    Guu = Rr + Bt'P22 Bt, its block Cholesky (3 x 3 leg pivots) with X = L^-1 [Bt' | rr] alongside, KH = X'X."""
    m = 3 * nlegs
    Bh = np.zeros((6, m + 1))
    Bh[:, :m] = Bt[:, :m]
    Bh[:, m] = dv
    C = F.mm(Ph[:, 6:12], Bh)
    Guu = Rr[:m, :m] + F.mm(Bt[:, :m].T, C[6:12, :m], lower=True, acc=True)
    L = F.chol(Guu)
    X = F.trsm_lower(L, np.hstack([Bt[:, :m].T, rr[:m, None]]))
    KH = F.mm(X.T, X, lower=True)                             # K = Bt Guu^-1 Bt', rho = Bt Guu^-1 rr
    Nh = np.zeros((13, 13))
    Nh[:12, :12] = dtN(yaw)
    PA = Ph + F.mm(Ph, Nh, acc=True)
    PA[:, 12] += C[:, m]
    F.add(13)
    Z = PA[6:12, :]
    M = np.vstack([Z, np.eye(13)[12:13]])
    KZ = F.mm(KH, M)
    APA = PA + F.mm(Nh.T, PA, acc=True)
    Pn = APA - F.mm(M.T, KZ, lower=True, acc=True)
    F.add(24)
    return Pn, KH


def leg_ipm(F, rb, z, s, G0j, rr_prev=None, mu=0.3, fmax=180.0):
    """A stance leg-step's share of an interior-point factorisation: W = z/s, Rr = Rb + C'WC, rr = C'W(s - b),
    Rr = L L', Y = G0_j L^-T, g_j = Y L^-1 rr, W_j = Y Y' (lower)."""
    W = z / s
    F.add(5)
    wv = W * (s - np.array([0, 0, 0, 0, fmax]))
    F.add(2 * 5)
    sx, sy = W[0] + W[1], W[2] + W[3]
    Rr = rb.copy()
    Rr[0, 0] += sx
    Rr[1, 1] += sy
    Rr[0, 2] = Rr[2, 0] = Rr[0, 2] + mu * (W[0] - W[1])
    Rr[1, 2] = Rr[2, 1] = Rr[1, 2] + mu * (W[2] - W[3])
    Rr[2, 2] += mu * mu * (sx + sy) + W[4]
    F.add(2 + 2 + 2 + 2 + 5 + 3)
    rr = np.array([-wv[0] + wv[1], -wv[2] + wv[3], -mu * wv[:4].sum() + wv[4]])
    F.add(2 + 2 + 6)
    L = F.chol(Rr)
    c = F.trsm_lower(L, rr[:, None])[:, 0]
    Y = F.trsm_lower(L, G0j.T).T                              # Y = G0_j L^-T
    g = F.mm(Y, c[:, None])[:, 0]
    Wj = F.mm(Y, Y.T, lower=True)
    return Rr, rr, Wj, g


def test_reduced_riccati_stage_restatement_is_the_riccati_step():
    F = Flops()
    Ph = spd(13)
    U = np.linalg.cholesky(spd(6, 1e-3))
    dv, qw, qcol = RNG.standard_normal(6), RNG.uniform(0, 10, 12), RNG.standard_normal(12)
    Pn = riccati_stage_reduced(F, Ph, 0.7, U, dv, qw, qcol)
    Pd = direct_riccati(Ph, 0.7, U, dv, qw, qcol)
    # rows 0-11 (the value function P and, in column 12, its linear term p; row 12 is never read by the kernel)
    assert np.allclose(Pn[:12], Pd[:12], rtol=1e-10, atol=1e-10)


def test_leg_terms_restatement():
    F = Flops()
    G0 = g0_block()
    rb = np.diag([1e-4, 1e-4, 1e-4])
    z, s = RNG.uniform(0.1, 2, 5), RNG.uniform(0.1, 2, 5)
    Rr, rr, Wj, g = leg_ipm(F, rb, z, s, G0[:, 0:3])
    Ri = np.linalg.inv(Rr)
    assert np.allclose(np.tril(Wj), np.tril(G0[:, 0:3] @ Ri @ G0[:, 0:3].T), rtol=1e-10, atol=1e-14)
    assert np.allclose(g, G0[:, 0:3] @ Ri @ rr, rtol=1e-10, atol=1e-14)


def counted_lq_components():
    """Flops of each roofline.lq_flop component, from the restatements."""
    out = {}
    F = Flops()
    U = np.linalg.cholesky(spd(6, 1e-3))
    F.chol(spd(6))                                           # U = chol(W_k), once per stage and factorisation
    riccati_stage_reduced(F, spd(13), 0.3, U, RNG.standard_normal(6), np.ones(12), np.ones(12))
    out["ipm_fact"] = F.n
    F = Flops()
    # the polish's reduced stage: the same plus the linear term's column g (13 x 6 + 6 x 6)
    F.chol(spd(6))
    riccati_stage_reduced(F, spd(13), 0.3, U, RNG.standard_normal(6), np.ones(12), np.ones(12))
    F.mm(spd(13)[:, 6:12], RNG.standard_normal((6, 1)))
    F.mm(spd(6), RNG.standard_normal((6, 1)))
    out["pol_fact_red"] = F.n
    F = Flops()
    Bt = g0_block()
    Rr = np.zeros((12, 12))
    for j in range(4):
        Rr[3 * j:3 * j + 3, 3 * j:3 * j + 3] = spd(3, 1e-4)
    riccati_stage_full(F, spd(13), 0.3, Bt, Rr, RNG.standard_normal(12), RNG.standard_normal(6), np.ones(12),
                       np.ones(12), 4)
    out["pol_fact_full"] = F.n
    # one Newton system: forward sweep x' = A x + dv - KZ x - t (closed-loop rows) and the costate
    # lambda2 = Z A^-1 x' (+ za - v2)
    F = Flops()
    KZ, Z, x = RNG.standard_normal((6, 12)), RNG.standard_normal((6, 12)), RNG.standard_normal(12)
    Nk = dtN(0.3)
    F.mm(Nk, x[:, None], acc=True)
    F.mm(KZ, x[:, None], acc=True)
    F.mm(Nk, x[:, None], acc=True)
    F.mm(Z, x[:, None], acc=True)
    out["system"] = F.n
    # the corrector: h = P22 dg (P22 from Z: Z[:, 6:12] - Z[:, 0:6] dtN), rho = dg - K h, q' = q - Z'rho, the
    # backward sweep p = q' + A'y - (KZ)'y6, t = K za + rho
    F = Flops()
    dg, K6 = RNG.standard_normal(6), spd(6)
    e = F.mm(Nk[0:6, 6:12], dg[:, None])
    F.mm(Z[:, 0:6], e)
    F.mm(Z[:, 6:12], dg[:, None], acc=True)
    F.mm(K6, dg[:, None], acc=True)
    F.mm(Z.T, dg[:, None], acc=True)
    F.mm(Nk.T, x[:, None], acc=True)
    F.mm(KZ.T, dg[:, None], acc=True)
    F.mm(K6, dg[:, None], acc=True)
    out["corr"] = F.n
    # polish verification per stage: B u rows (G0 u over the stage's legs), the dynamics rows, the tracking terms
    # and the adjoint step
    F = Flops()
    F.mm(Bt[:, :6], RNG.standard_normal((6, 1)))
    F.mm(Nk, x[:, None], acc=True)
    F.add(12 + 12)
    F.mm(Nk.T, x[:, None], acc=True)
    out["verify"] = F.n
    # per stance leg-step
    F = Flops()
    leg_ipm(F, np.diag([1e-4] * 3), RNG.uniform(0.1, 2, 5), RNG.uniform(0.1, 2, 5), Bt[:, 0:3])
    out["leg_ipm"] = F.n
    F = Flops()
    # polish: a leg with one active face (the common case: two free directions), its null-space basis T (3 x 2,
    # orthonormal, from the face normal: a normalisation and a cross product, ~30 flops) and particular solution
    # up, Rr = T'Rb T, rr = T'Rb up, Bt_j = G0_j T, du = G0_j up, then in reduced inputs Rr = L L', L^-1 rr,
    # Y = Bt_j L^-T, g_j = Y L^-1 rr, W_j = Y Y' (lower); Rb = diag(r) on flat ground
    T, up, Rb = RNG.standard_normal((3, 2)), RNG.standard_normal(3), np.diag(RNG.uniform(1, 2, 3))
    F.add(30)
    RT = F.mm(Rb, T)
    Rr2 = F.mm(T.T, RT, lower=True)
    rr2 = F.mm(T.T, F.mm(Rb, up[:, None]))
    Btj = F.mm(Bt[:, 0:3], T)
    F.mm(Bt[:, 0:3], up[:, None])
    Lr = F.chol(T.T @ Rb @ T)
    cr = F.trsm_lower(Lr, rr2)
    Y = F.trsm_lower(Lr, Btj.T).T
    F.mm(Y, cr)
    F.mm(Y, Y.T, lower=True)
    out["leg_pol"] = F.n
    F = Flops()
    # per Newton system and leg-step: u = -Rr^-1 (rr + Bt' lambda2), the step-length terms
    lam = RNG.standard_normal(6)
    F.mm(Bt[:, 0:3].T, lam[:, None], acc=True)
    Lr = F.chol(spd(3))
    F.trsm_lower(Lr, np.ones((3, 1)))
    F.trsm_lower(Lr.T[::-1, ::-1].copy(), np.ones((3, 1)))
    F.add(5 * 2 + 5 * 3)                                     # constraint residuals, ds, dz and their ratios
    out["leg_system"] = F.n
    F = Flops()
    # polish verification per leg-step: G0_j u, g = R u + G0_j' lambda, the multiplier fit and its residual
    F.mm(Bt[:, 0:3], np.ones((3, 1)))
    F.mm(spd(3), np.ones((3, 1)))
    F.mm(Bt[:, 0:3].T, lam[:, None], acc=True)
    F.add(5 * 2 + 30)
    out["leg_verify"] = F.n
    out["quad"] = 21 * 3 + 6 * 3                             # quad sums of W_j and g_j over the stage's legs
    return out


def counted_lq_flop(H, ipm_iters, polish_rounds, stance_per_stage):
    c = counted_lq_components()
    s = stance_per_stage
    pol_fact = c["pol_fact_red"] if 4 * H <= 64 else c["pol_fact_full"]
    ipm_stage = c["ipm_fact"] + 2 * c["system"] + c["corr"] + s * (c["leg_ipm"] + 2 * c["leg_system"]) + c["quad"]
    pol_stage = pol_fact + c["system"] + c["verify"] + s * (c["leg_pol"] + c["leg_system"] + c["leg_verify"]) + c["quad"]
    return H * (ipm_iters * ipm_stage + polish_rounds * pol_stage)


# (config, H, mean interior-point iterations, mean polish rounds, stance leg-steps per stage) of the bench lines
# (profiles/r05/bench/bench_c*.json): the operating points the headline fractions are priced at
LQ_POINTS = [(3, 20, 5.88, 1.67, 2.0), (4, 10, 5.78, 1.66, 2.5), (5, 30, 6.15, 1.83, 2.0), ("2off", 10, 5.4, 1.6, 2.0)]


@pytest.mark.parametrize("cfg,H,it,rd,s", LQ_POINTS)
def test_lq_flop_model_matches_counted_restatement(cfg, H, it, rd, s):
    model = roofline.lq_flop(H, it, rd, s)
    counted = counted_lq_flop(H, it, rd, s)
    print(f"config {cfg}: roofline.lq_flop {model:.4g}, counted {counted:.4g} ({model / counted - 1:+.1%})")
    assert abs(model / counted - 1.0) <= 0.05


def test_lq_components_match_the_tallies():
    """Component by component (flops = 2 x the FMA constants of roofline.py), within 10 % each."""
    c = counted_lq_components()
    tallies = {"ipm_fact": roofline.LQ_IPM_FACT_FMA, "pol_fact_red": roofline.LQ_POL_FACT_RED_FMA,
               "pol_fact_full": roofline.LQ_POL_FACT_FULL_FMA, "system": roofline.LQ_SYSTEM_FMA,
               "corr": roofline.LQ_CORR_FMA, "verify": roofline.LQ_VERIFY_FMA, "leg_ipm": roofline.LQ_LEG_IPM_FMA,
               "leg_pol": roofline.LQ_LEG_POL_FMA, "leg_system": roofline.LQ_LEG_SYSTEM_FMA,
               "leg_verify": roofline.LQ_LEG_VERIFY_FMA}
    for k, fma in tallies.items():
        print(f"{k}: tally {2 * fma}, counted {c[k]} ({2 * fma / c[k] - 1:+.1%})")
        assert abs(2 * fma / c[k] - 1.0) <= 0.10, k


# ---- the condensed dense interior point ---------------------------------------------------------------------

def counted_dense_flop(H, n_stance, ipm_iters, polish_rounds):
    """The dense kernel's work restated (csrc/lmpc_dense_common.h, lmpc_dense_kernel.h) with N = 3 x stance
    leg-steps: the condensation (free response and adjoint, the cost-to-go P~ recursion on the matrix cores, one
    Hessian column per stance variable walked down the steps), then per interior-point iteration M = H + C'WC on
    the leg blocks, its Cholesky and two Newton systems of two triangular solves; per polish round T'HT, the
    Cholesky, one system and the verification's H u.  Checked: the Hessian columns against the dense product."""
    F = Flops()
    N = int(round(3 * n_stance))
    # free response c_{m+1} = A_m c_m (8 terms) and the adjoint mu_m = Q (c - xref) + A_m' mu_{m+1}, per step
    for _ in range(H):
        F.mm(dtN(0.2), np.ones((12, 1)), acc=True)
        F.add(12 * 2)
        F.mm(dtN(0.2).T, np.ones((12, 1)), acc=True)
    # cost-to-go P~_m = Q + A_m' P~_{m+1} A_m (symmetric 12 x 12) per step
    Pt = spd(12)
    for _ in range(H):
        PA = Pt + F.mm(Pt, dtN(0.2), acc=True)
        Pt = PA + F.mm(dtN(0.2).T, PA, acc=True, lower=True)
    # gradient g_i = B' mu_{i+1} per stance variable (6 terms) and the Hessian columns: per stance variable v
    # (step i), L = P~_{i+1} B e_v (12 x 6 terms), then down the steps j < i: H[j-block][v] = B' L (6 terms per
    # stance variable of step j), L <- A_j' L (8 terms)
    G0 = g0_block()
    per_step = max(1, int(round(n_stance / H)))
    F.add(N * 2 * 6)
    for v in range(N):
        step = min(H - 1, v // (3 * per_step))
        L = F.mm(Pt[:, 6:12], G0[:, v % 12:v % 12 + 1])
        for j in range(step, -1, -1):
            F.mm(G0[:, : 3 * per_step].T, L[6:12])
            L = L + F.mm(dtN(0.2).T, L, acc=True)
    cond = F.n
    # the Hessian built this way is the dense product (check on a small random instance)
    Mh = spd(N)
    F = Flops()
    D = np.zeros((N, N))
    for b in range(N // 3):                                   # C'WC on the leg blocks
        D[3 * b:3 * b + 3, 3 * b:3 * b + 3] = spd(3)
    F.add(N // 3 * 9 * 2)
    M = Mh + D
    Lm = F.chol(M)
    for _ in range(2):                                        # predictor and corrector
        y = F.trsm_lower(Lm, RNG.standard_normal((N, 1)))
        F.trsm_lower(Lm.T[::-1, ::-1].copy(), y[::-1].copy())
    F.add(N * 2 * 10)                                         # right-hand sides and the step lengths
    it = F.n
    F = Flops()
    T = np.zeros((N, N))
    for b in range(N // 3):
        T[3 * b:3 * b + 3, 3 * b:3 * b + 2] = RNG.standard_normal((3, 2))
    TH = F.mm(T.T, Mh)
    F.mm(TH, T, lower=True)
    Lp = F.chol(spd(N))
    y = F.trsm_lower(Lp, RNG.standard_normal((N, 1)))
    F.trsm_lower(Lp.T[::-1, ::-1].copy(), y[::-1].copy())
    F.mm(Mh, np.ones((N, 1)), acc=True)                       # the verification's H u + g
    F.mm(Mh, np.ones((N, 1)), acc=True)                       # the round's right-hand side H up + g
    pol = F.n
    return cond + ipm_iters * it + polish_rounds * pol


def test_dense_cholesky_and_solves_restatement():
    F = Flops()
    M = spd(12)
    L = F.chol(M)
    assert np.allclose(L @ L.T, M)
    y = F.trsm_lower(L, np.ones((12, 1)))
    assert np.allclose(L @ y, 1.0)
    # a left-looking Cholesky of order N: N^3/3 + O(N^2) flops
    assert abs(F.n - (12 ** 3 / 3 + 12 ** 2)) / (12 ** 3 / 3) < 0.5


# the dense path's QPs: a trot at H = 10 has two stance legs per step (20 leg-steps; config 2's measured means), and
# 18 where a step's plan_contacts differs from the prediction
@pytest.mark.parametrize("H,ns,it,rd", [(10, 20.0, 5.30, 1.51), (10, 20.0, 6.0, 2.0), (10, 18.0, 5.5, 1.6)])
def test_dense_flop_model_matches_counted_restatement(H, ns, it, rd):
    model = roofline.dense_flop(H, ns, it, rd)
    counted = counted_dense_flop(H, ns, it, rd)
    print(f"H {H}, {ns} stance leg-steps: roofline.dense_flop {model:.4g}, counted {counted:.4g} "
          f"({model / counted - 1:+.1%})")
    assert abs(model / counted - 1.0) <= 0.05

"""Algorithmic work models of the QP path (used by bench.py's roofline).

`survey_flop` is the contract figure for `roofline.achieved`: SURVEY.md 8(d)'s algorithmic
flops of one QP of horizon H, independent of how the build solves it --

  N = 12H, block GEMM cost c = 2 * 12^3
  F0     = c (H(H-1)/2 + H) + c H(H+1)(H+2)/6 + (N^2 + 288 H) + N^3/3   (condensation + factorisation)
  F_iter = 2 N^2 + 144 H                                            (per iteration)
  F      = F0 + K * F_iter + rounds * (N^3/3 + 2 N^2)                (polish: refactor + solve)

with K the measured mean interior-point iterations and `rounds` the mean polish rounds.
F0 = 1.544M / 10.72M / 34.44M flop at H = 10 / 20 / 30.

`lq_flop` (the LDS Riccati kernel) and `dense_flop` (the condensed dense interior point) are the useful flops of
the formulations the kernels run, reported beside it and used as the headline fraction wherever the contract's F0 (a
dense N = 12H condensation) is not the work done ("Round 6").
"""
from __future__ import annotations

FP64_PEAK_TFLOPS = 78.6             # MI355X FP64 (vector = matrix), SURVEY.md 8d / AMD spec
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md chip table (spec)


# ---- the LDS Riccati kernel (lmpc_lq.hip, round 4 on): useful flops of the formulation it runs -----------------
# (pinned in round 6)  Counted on the nonzero structure of the operands, not
# on the padded 16x16 MFMA tiles or the exec-masked lanes the PMC counters see: tests/test_flop_models.py restates
# every operation below in numpy on matrices with the kernel's structure (checked for what they compute: the Riccati
# step against the direct formula, W_j against Bt Rr^-1 Bt') and counts each product as executed (FMA = 2 flops, a
# lone multiply, division, sqrt or reciprocal 1); the constants are those counts in FMA units (flops / 2).  Round 5's
# hand tallies were 4 % (factorisations) to 2x (leg-step terms, which multiplied G0_j's structural zeros) higher, in
# all 13-15 % over the count.  Per horizon stage ("Round 6"):
#   interior-point factorisation (reduced inputs, six unit-cost inputs f = U v - g): U = chol(W), C = P^[:,6:12]
#     [U | dv], Guu' = I + U'(P22 U), chol(Guu'), X = L^-1 U', K = X'X, P^ dtN, KZ = K Z, dtN' PA, PA' KZ (symmetric)
#   polish factorisation: the same in reduced inputs where W_k is well conditioned (one leg-step per lane), plus the
#     linear term's column; full inputs (two leg-steps per lane: H > 16): C = P^[:,6:12] [Bt | dv], Guu = Rr +
#     Bt'P22 Bt, its Cholesky with X = L^-1 [Bt' | rr] alongside, KH = X'X, PA, KZ, P
#   per Newton system: forward sweep x' = A x + dv - KZ x - t, costate lambda2 = Z A^-1 x'
#   corrector: P22 dg, rho, q' = q - Z'rho, the backward sweep, t = K za + rho
#   polish verification: B u rows, dynamics rows, tracking terms, adjoint step
# per stance leg-step:
#   interior point, per factorisation: W = z/s, C'WC, Rr and its Cholesky, L^-1 rr, Y = G0_j L^-T, g_j, W_j = Y Y'
#   polish, per factorisation (one active face, the common case): null basis, T'RbT, rr, Bt = G0 T, G0 up, Y, W_j
#   per Newton system: G0_j' lambda2, the 3 x 3 solve, the step-length terms
#   polish verification: G0_j u, g = R u + G0_j' lambda, the multiplier fit and the stationarity residual
# per stage and factorisation: the quad sums of W_j and g_j (27 entries x 3 adds)
LQ_IPM_FACT_FMA = 1876
LQ_POL_FACT_RED_FMA = 1980.5
LQ_POL_FACT_FULL_FMA = 3326
LQ_SYSTEM_FMA = 160
LQ_CORR_FMA = 298
LQ_VERIFY_FMA = 49
LQ_LEG_IPM_FMA = 89
LQ_LEG_POL_FMA = 117
LQ_LEG_SYSTEM_FMA = 42
LQ_LEG_VERIFY_FMA = 48.5
LQ_QUAD_FLOP = 81


def lq_flop(H: int, ipm_iters: float, polish_rounds: float, stance_per_stage: float) -> float:
    """Useful flops of one QP on the LDS Riccati kernel given its (mean) interior-point iterations, polish rounds and
    stance leg-steps per stage (an interior-point iteration = one factorisation + predictor and corrector systems;
    a polish round = one factorisation + one system + the verification)."""
    s = stance_per_stage
    reduced_polish = 4 * H <= 64  # one leg-step per lane: reduced-input polish stages (LQ_RP)
    ipm_stage = 2 * (LQ_IPM_FACT_FMA + 2 * LQ_SYSTEM_FMA + LQ_CORR_FMA
                     + s * (LQ_LEG_IPM_FMA + 2 * LQ_LEG_SYSTEM_FMA)) + LQ_QUAD_FLOP
    pol_fact = LQ_POL_FACT_RED_FMA if reduced_polish else LQ_POL_FACT_FULL_FMA
    pol_stage = 2 * (pol_fact + LQ_SYSTEM_FMA + LQ_VERIFY_FMA
                     + s * (LQ_LEG_POL_FMA + LQ_LEG_SYSTEM_FMA + LQ_LEG_VERIFY_FMA)) + LQ_QUAD_FLOP
    return H * (ipm_iters * ipm_stage + polish_rounds * pol_stage)


def dense_flop(H: int, n_stance: float, ipm_iters: float, polish_rounds: float) -> float:
    """Useful flops of one QP on the condensed dense interior point (lmpc_dense.hip): SURVEY.md 8(d)'s formulas with
    the condensed dimension the kernel solves, N = 3 x stance leg-steps (swing leg-steps are eliminated exactly), and
    the condensation's Hessian columns priced per stance variable: free response + adjoint 2 x 12 x 12 H, cost-to-go
    c H, H columns N x (12 x 6 + H x 8 + stance variables of the later steps x 6) ~ N (72 + 8 H) + N^2 x 6 / 2;
    per interior-point iteration M = H + C'WC, its Cholesky N^3 / 3, two Newton systems of two triangular solves
    (4 x 2 N^2 / 2); per polish round T'HT (2 N^2 x 3 / 3), the Cholesky, one system and H u (2 N^2)."""
    N = 3.0 * n_stance
    c = 2 * 12 ** 3
    cond = 2 * 2 * 144 * H + c * H + 2 * N * (72 + 8 * H) + 6 * N * N
    it = N * N / 2 + N ** 3 / 3 + 4 * N * N
    pol = 2 * N * N + N ** 3 / 3 + 2 * N * N + 2 * N * N
    return cond + ipm_iters * it + polish_rounds * pol


def survey_f0(H: int) -> float:
    N = 12 * H
    c = 2 * 12 ** 3
    f_pred = c * (H * (H - 1) / 2 + H)
    f_hess = c * H * (H + 1) * (H + 2) / 6
    f_grad = N * N + 288 * H
    f_chol = N ** 3 / 3
    return f_pred + f_hess + f_grad + f_chol


def survey_f_iter(H: int) -> float:
    N = 12 * H
    return 2 * N * N + 144 * H


def survey_flop(H: int, iters: float, polish_rounds: float) -> float:
    """SURVEY.md 8(d) algorithmic flops of one QP (the contract figure for roofline.achieved)."""
    N = 12 * H
    return survey_f0(H) + iters * survey_f_iter(H) + polish_rounds * (N ** 3 / 3 + 2 * N * N)


def gi_flop(H: int, steps: float) -> float:
    """Dual active-set path (lmpc_gi.hip): SURVEY.md 8(d)'s F0 (condensation + one factorisation) plus,
    per active-set step, z = J2 d2 (2 N^2) and the Householder update of J (4 N^2) on the padded
    N = 64 dense dimension (the R^-1 product and the 3-row d = J'n are lower order)."""
    return survey_f0(H) + steps * 6 * 64 * 64


def qp_bytes(H: int) -> int:
    """HBM bytes per QP: record (33+12H doubles) + contact (4H) + GRF out (12H doubles) + status + iters."""
    return (33 + 12 * H) * 8 + 4 * H + 12 * H * 8 + 8


def hoqp_level_flop(n: int, m: int, s: int, p: int, nd: int, rank: int, iters: float) -> float:
    """Algorithmic flops of one hierarchical-QP level (lmpc_hoqp.hip), FMA = 2 flops:
    n variables, m equality / s own inequality / p frozen higher rows, nd null-space coordinates on entry,
    rank = rank(A Z), iters interior-point iterations.

      setup      G = A Z (2 m n nd) + G'G (m nd^2, symmetric) + c (2 m nd) + constraint rows R = D Z
                 (2 r n nd, r = p + s) and their bounds (2 r n)
      FullPivLU  2 sum_k (m - k - 1)(nd - k - 1) over k < min(m, nd), kernel solve rank^2 (nd - rank),
                 Z' = Z K (2 n rank (nd - rank))
      iteration  K = Hy + R' W R (r nd^2, symmetric) + Cholesky nd^3 / 3 + two solves (2 x 2 nd^2)
                 + residuals R y, R'z, Hy y (4 r nd + 2 nd^2) + two Newton systems' R'q and R dy (8 r nd)
      output     x += Z y (2 n nd) + slacks (2 s nd)
    """
    r = p + s
    k = min(m, nd)
    lu = 2.0 * sum((m - i - 1) * (nd - i - 1) for i in range(k)) if m else 0.0
    dimker = nd - rank
    setup = 2 * m * n * nd + m * nd * nd + 2 * m * nd + 2 * r * n * nd + 2 * r * n
    basis = (lu + rank * rank * dimker + 2 * n * rank * dimker) if m else 0.0
    it = r * nd * nd + nd ** 3 / 3 + 4 * nd * nd + 4 * r * nd + 2 * nd * nd + 8 * r * nd
    return setup + basis + iters * it + 2 * n * nd + 2 * s * nd


def hoqp_bytes(n: int, eq_rows, ineq_rows) -> int:
    """HBM bytes of one instance: the record in (per level a, b, d, f) + x per level + slacks out."""
    rec = sum((m + s) * (n + 1) for m, s in zip(eq_rows, ineq_rows))
    return 8 * (rec + len(eq_rows) * n + sum(ineq_rows))

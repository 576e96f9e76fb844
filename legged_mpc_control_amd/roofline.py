"""Algorithmic work models of the QP path (used by bench.py's roofline).

`survey_flop` is the contract figure for `roofline.achieved`: SURVEY.md 8(d)'s algorithmic
flops of one QP of horizon H, independent of how the build solves it --

  N = 12H, block GEMM cost c = 2 * 12^3
  F0     = c (H(H-1)/2 + H) + c H(H+1)(H+2)/6 + (N^2 + 288 H) + N^3/3   (condensation + factorisation)
  F_iter = 2 N^2 + 144 H                                            (per iteration)
  F      = F0 + K * F_iter + rounds * (N^3/3 + 2 N^2)                (polish: refactor + solve)

with K the measured mean interior-point iterations and `rounds` the mean polish rounds.
F0 = 1.544M / 10.72M / 34.44M flop at H = 10 / 20 / 30.

`qp_flop` is the build's own count of useful fp64 flops of its Riccati formulation (FMA = 2
flops), per horizon stage, reported beside it:

  Riccati factorisation stage (riccati_factor):
    Bt = G0 T (216 FMA) + G0 up (72) + PB = P[:,6:12] Bt (864) + v = P d (72)
    + Guu = T'RtT + Bt'PB[6:12] (324 + 864) + Gux = PB'A (180)
    + Cholesky(12) + L^-1 Gux + L^-1 (288 + 864 + 288)
    + P(I+dtN), (I+dtN')PA (500) + Y'Y symmetric (936)            = 5468 FMA
  Riccati vector pass stage (riccati_solve): backward 450 FMA + forward 410 = 860 FMA
  Adjoint stage (adjoint_grad): 120 FMA
  IPM iteration  = 1 factorisation + 2 vector passes (predictor + corrector)
  polish round   = 1 factorisation + 1 vector pass + 1 adjoint
"""
from __future__ import annotations

FACT_FLOP_PER_STAGE = 2 * 5468
SOLVE_FLOP_PER_STAGE = 2 * 860
ADJ_FLOP_PER_STAGE = 2 * 120
LEG_FLOP_PER_IPM_ITER = 2 * 60      # per stance leg-step: W, C'WC, C'w, step lengths
LEG_FLOP_PER_POLISH = 2 * 80        # per stance leg-step: null basis + verification

FP64_PEAK_TFLOPS = 78.6             # MI355X FP64 (vector = matrix), SURVEY.md 8d / AMD spec
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md chip table (spec)


def ipm_iter_flop(H: int) -> int:
    return H * (FACT_FLOP_PER_STAGE + 2 * SOLVE_FLOP_PER_STAGE) + 4 * H * LEG_FLOP_PER_IPM_ITER


def polish_round_flop(H: int) -> int:
    return H * (FACT_FLOP_PER_STAGE + SOLVE_FLOP_PER_STAGE + ADJ_FLOP_PER_STAGE) + 4 * H * LEG_FLOP_PER_POLISH


def qp_flop(H: int, ipm_iters: float, polish_rounds: float) -> float:
    """Algorithmic flops of one QP given its (mean) IPM iterations and polish rounds."""
    return ipm_iters * ipm_iter_flop(H) + polish_rounds * polish_round_flop(H)


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

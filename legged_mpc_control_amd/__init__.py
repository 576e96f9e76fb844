"""MI355X-native batched convex-MPC ground-reaction-force QP solver.

Drop-in for the convex-MPC QP path of zha0ming1e/legged_mpc_control
(src/legged_ctrl ConvexQPSolver / ConvexMpc::grf_update): the QP assembly and
the solve run as one fused HIP kernel for gfx950 behind the C-ABI in
include/lmpc/lmpc.h.
"""
from . import _native
from ._native import (GAIT_CRAWL, GAIT_STAND, GAIT_TROT, GAIT_TROT_WITH_STAND, LmpcCommand, LmpcLegKin,
                      LmpcOptions, LmpcParams, NativeLibraryError)
from .solver import (BatchedConvexQPSolver, ConvexQPSolver, LeggedContactFSM, LeggedCtrl, LeggedFeedback,
                     LeggedParam, LeggedState, foot_jacobian, grf_to_torque, leg_kin_default, solver_options)
from . import synth

__all__ = [
    "BatchedConvexQPSolver", "ConvexQPSolver", "LeggedContactFSM", "LeggedState", "LeggedFeedback",
    "LeggedCtrl", "LeggedParam", "LmpcParams", "LmpcOptions", "NativeLibraryError", "synth",
    "GAIT_TROT", "GAIT_CRAWL", "GAIT_TROT_WITH_STAND", "GAIT_STAND", "LmpcCommand", "LmpcLegKin",
    "leg_kin_default", "foot_jacobian", "grf_to_torque", "solver_options",
]

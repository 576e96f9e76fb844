"""Host-side mirror of the reference's convex-MPC solver interface over the C-ABI.

`ConvexQPSolver` keeps the reference's method names and call sequence
(src/legged_ctrl/src/mpc_ctrl/convex_mpc/ConvexMpc.cpp:70-72):

    solver = ConvexQPSolver(q_weights, r_weights)          # ConvexQPSolver.cpp:16
    solver.calc_mpc_reference(state, leg_fsm)              # ConvexQPSolver.cpp:254-313
    solver.update_cons_matrix()                            # ConvexQPSolver.cpp:230-239 (no-op)
    grf = solver.compute_grfs(state)                       # ConvexQPSolver.cpp:314-327 -> (12,)

`BatchedConvexQPSolver` is the batched form (host numpy or device torch
buffers).  Both run the HIP kernel; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as N


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def leg_kin_default() -> N.LmpcLegKin:
    """The reference's leg constants (BaseInterface.cpp:76-97)."""
    k = N.LmpcLegKin()
    N.lib().lmpc_leg_kin_default(ctypes.byref(k))
    return k


def foot_jacobian(kin: N.LmpcLegKin, leg: int, q) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.float64).reshape(3)
    J = np.zeros(9)
    N.lib().lmpc_foot_jacobian(ctypes.byref(kin), int(leg), _dp(q), _dp(J))
    return J.reshape(3, 3)


def grf_to_torque(kin: N.LmpcLegKin, rot, joint_pos, grf0) -> np.ndarray:
    """Host: one instance, tau [12] = -J_i'(R'u0_i) (BaseInterface::tau_ctrl_update, BaseInterface.cpp:451-459)."""
    rot = np.ascontiguousarray(rot, dtype=np.float64).reshape(9)
    q = np.ascontiguousarray(joint_pos, dtype=np.float64).reshape(12)
    f = np.ascontiguousarray(grf0, dtype=np.float64).reshape(12)
    tau = np.zeros(12)
    N.check(N.lib().lmpc_grf_to_torque(ctypes.byref(kin), _dp(rot), _dp(q), _dp(f), _dp(tau)), "lmpc_grf_to_torque")
    return tau


def solver_options(**overrides) -> N.LmpcOptions:
    """lmpc_options_default with the named fields replaced, e.g. solver_options(gi_max_steps=20)."""
    o = N.LmpcOptions()
    N.lib().lmpc_options_default(ctypes.byref(o))
    for k, v in overrides.items():
        if not hasattr(o, k):
            raise AttributeError(f"lmpc_options has no field {k!r}")
        setattr(o, k, v)
    return o


class BatchedConvexQPSolver:
    """A device context: horizon H, host staging for up to max_batch QPs."""

    DENSE_PATHS = {"off": 0, "ipm": 1, "gi": 2}
    RICCATI_PATHS = {"scratch": 0, "lds": 1}

    def __init__(self, params: N.LmpcParams, horizon: int, max_batch: int = 1, device: int = 0,
                 options: N.LmpcOptions | None = None, dense_path: str | None = None,
                 riccati_path: str | None = None):
        """dense_path: "ipm" (default), "gi" or "off" (lmpc_set_dense_path); riccati_path: "lds" (default, the
        LDS-resident kernel) or "scratch" (the global-workspace kernel) -- lmpc_set_riccati_path."""
        if not (1 <= horizon <= N.LMPC_MAX_HORIZON):
            raise ValueError(f"horizon must be in [1, {N.LMPC_MAX_HORIZON}]")
        self._L = N.lib()
        self.H = int(horizon)
        self.max_batch = int(max_batch)
        self.params = params
        self._ctx = ctypes.c_void_p()
        N.check(self._L.lmpc_create(ctypes.byref(params), self.H, self.max_batch, int(device),
                                    ctypes.byref(self._ctx)), "lmpc_create")
        if options is not None:
            self.set_options(options)
        if dense_path is not None:
            self.set_dense_path(dense_path)
        if riccati_path is not None:
            self.set_riccati_path(riccati_path)
        if self.max_batch > 0:
            # the workspace of the context's paths for max_batch QPs (after the Riccati path is chosen: the scratch
            # kernel's factors are reserved only when it runs)
            N.check(self._L.lmpc_reserve(self._ctx, self.max_batch), "lmpc_reserve")

    def reserve_warm(self, batch: int) -> None:
        """Pre-allocate the warm-start workspace (lmpc_reserve_warm) so the first warm solve does not allocate."""
        N.check(self._L.lmpc_reserve_warm(self._ctx, int(batch)), "lmpc_reserve_warm")

    def set_riccati_path(self, path: str) -> None:
        N.check(self._L.lmpc_set_riccati_path(self._ctx, self.RICCATI_PATHS[path]), "lmpc_set_riccati_path")

    @property
    def riccati_path(self) -> str:
        """The Riccati kernel of cold solves for this context."""
        return {0: "scratch", 1: "lds"}[self._L.lmpc_get_riccati_path(self._ctx)]

    def set_dense_path(self, path: str) -> None:
        N.check(self._L.lmpc_set_dense_path(self._ctx, self.DENSE_PATHS[path]), "lmpc_set_dense_path")

    @property
    def dense_path(self) -> str:
        """The dense-path kernel in effect for this context."""
        v = self._L.lmpc_get_dense_path(self._ctx)
        return {0: "off", 1: "ipm", 2: "gi"}[v]

    @property
    def record_len(self) -> int:
        return 33 + 12 * self.H

    def set_options(self, o: N.LmpcOptions) -> None:
        N.check(self._L.lmpc_set_options(self._ctx, ctypes.byref(o)), "lmpc_set_options")

    def set_params(self, p: N.LmpcParams) -> None:
        N.check(self._L.lmpc_set_params(self._ctx, ctypes.byref(p)), "lmpc_set_params")
        self.params = p

    def solve(self, rec: np.ndarray, contact: np.ndarray, normals: np.ndarray | None = None):
        """Host arrays in -> (grf [B,H,12], status [B], iters [B]); synchronous.
        normals [B,4,3] (terrain extension) or None = flat ground (the reference problem)."""
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        contact = np.ascontiguousarray(contact, dtype=np.uint8)
        B = rec.shape[0]
        if rec.shape != (B, self.record_len) or contact.shape != (B, self.H, 4):
            raise ValueError("bad record/contact shape")
        nptr = None
        if normals is not None:
            normals = np.ascontiguousarray(normals, dtype=np.float64)
            if normals.shape != (B, 4, 3):
                raise ValueError("normals must be [B, 4, 3]")
            nptr = _dp(normals)
        grf = np.zeros((B, self.H, 12), dtype=np.float64)
        status = np.zeros(B, dtype=np.int32)
        iters = np.zeros(B, dtype=np.int32)
        N.check(self._L.lmpc_solve_batch_ex(self._ctx, _dp(rec), contact.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                            nptr, B, _dp(grf), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                            iters.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), "lmpc_solve_batch_ex")
        return grf, status, iters

    def solve_warm(self, rec: np.ndarray, contact: np.ndarray, act_in: np.ndarray | None = None,
                   normals: np.ndarray | None = None):
        """Warm-started solve (lmpc_solve_batch_warm): act_in [B,H,4] u8 active sets (None = cold) ->
        (grf, status, iters, act_out [B,H,4]).  Every QP runs on the Riccati kernel's active-set polish
        from act_in, falling back to its cold interior point; the optimum is the same either way."""
        rec = np.ascontiguousarray(rec, dtype=np.float64)
        contact = np.ascontiguousarray(contact, dtype=np.uint8)
        B = rec.shape[0]
        if rec.shape != (B, self.record_len) or contact.shape != (B, self.H, 4):
            raise ValueError("bad record/contact shape")
        u8 = ctypes.POINTER(ctypes.c_uint8)
        aptr = None
        if act_in is not None:
            act_in = np.ascontiguousarray(act_in, dtype=np.uint8)
            if act_in.shape != (B, self.H, 4):
                raise ValueError("act_in must be [B, H, 4]")
            aptr = act_in.ctypes.data_as(u8)
        nptr = None
        if normals is not None:
            normals = np.ascontiguousarray(normals, dtype=np.float64)
            if normals.shape != (B, 4, 3):
                raise ValueError("normals must be [B, 4, 3]")
            nptr = _dp(normals)
        grf = np.zeros((B, self.H, 12), dtype=np.float64)
        status = np.zeros(B, dtype=np.int32)
        iters = np.zeros(B, dtype=np.int32)
        act_out = np.zeros((B, self.H, 4), dtype=np.uint8)
        i32 = ctypes.POINTER(ctypes.c_int32)
        N.check(self._L.lmpc_solve_batch_warm(self._ctx, _dp(rec), contact.ctypes.data_as(u8), nptr, B, aptr,
                                              act_out.ctypes.data_as(u8), _dp(grf), status.ctypes.data_as(i32),
                                              iters.ctypes.data_as(i32)), "lmpc_solve_batch_warm")
        return grf, status, iters, act_out

    @staticmethod
    def shift_active_set(act: np.ndarray) -> np.ndarray:
        """One MPC step later (lmpc_shift_active_set): stage k <- k+1, the last stage keeps its own."""
        act = np.ascontiguousarray(act, dtype=np.uint8)
        out = np.empty_like(act)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        N.lib().lmpc_shift_active_set(act.ctypes.data_as(u8), act.shape[0], act.shape[1], out.ctypes.data_as(u8))
        return out

    def solve_device(self, rec, contact, grf, status=None, iters=None, stream=None, normals=None) -> None:
        """Device tensors (torch, resident in HBM) in/out; asynchronous on `stream`
        (a torch.cuda.Stream or raw hipStream_t int; default = torch's current stream).
        normals: optional f64 device tensor [B,4,3] (terrain extension)."""
        import torch

        B = rec.shape[0]
        for t, dt in ((rec, torch.float64), (contact, torch.uint8), (grf, torch.float64)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
                raise ValueError("solve_device expects contiguous device tensors (f64 rec/grf, u8 contact)")
        if rec.shape != (B, self.record_len) or contact.shape != (B, self.H, 4) or grf.shape != (B, self.H, 12):
            raise ValueError("bad record/contact/grf shape")
        if normals is not None and (not normals.is_cuda or normals.dtype != torch.float64 or
                                    not normals.is_contiguous() or tuple(normals.shape) != (B, 4, 3)):
            raise ValueError("normals must be a contiguous f64 device tensor [B, 4, 3]")
        if stream is None:
            stream = torch.cuda.current_stream(rec.device)
        sptr = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        N.check(self._L.lmpc_solve_batch_device_ex(
            self._ctx, rec.data_ptr(), contact.data_ptr(), None if normals is None else normals.data_ptr(), B,
            grf.data_ptr(), None if status is None else status.data_ptr(),
            None if iters is None else iters.data_ptr(), sptr), "lmpc_solve_batch_device_ex")

    # ---- the step before the QP, on the device -------------------------------
    # Commands live in HBM as an opaque uint8 tensor [B, N.COMMAND_BYTES] (lmpc_command array).
    @staticmethod
    def _stream(stream, dev):
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(dev)
        return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)

    def synth_commands_device(self, cfg: N.LmpcSynthCfg, count: int, seed: int, first_index: int = 0, device=None,
                              stream=None):
        """Synthetic commands generated on the device from (seed, global index) -> uint8 [count, 408]."""
        import torch

        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        out = torch.empty((count, N.COMMAND_BYTES), dtype=torch.uint8, device=dev)
        N.check(self._L.lmpc_synth_commands_device(self._ctx, ctypes.byref(cfg), seed, first_index, count,
                                                   out.data_ptr(), self._stream(stream, dev)),
                "lmpc_synth_commands_device")
        return out

    def synth_normals_device(self, count: int, seed: int, first_index: int = 0, theta_max: float = 0.3, device=None,
                             stream=None):
        import torch

        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        out = torch.empty((count, 4, 3), dtype=torch.float64, device=dev)
        N.check(self._L.lmpc_synth_normals_device(self._ctx, seed, first_index, count, float(theta_max),
                                                  out.data_ptr(), self._stream(stream, dev)),
                "lmpc_synth_normals_device")
        return out

    def build_records_device(self, cmd, stream=None):
        """uint8 [B, 408] commands in HBM -> (rec [B, 33+12H] f64, contact [B, H, 4] u8) in HBM."""
        import torch

        B = cmd.shape[0]
        if not cmd.is_cuda or cmd.dtype != torch.uint8 or tuple(cmd.shape) != (B, N.COMMAND_BYTES):
            raise ValueError("commands must be a uint8 device tensor [B, COMMAND_BYTES]")
        rec = torch.empty((B, self.record_len), dtype=torch.float64, device=cmd.device)
        con = torch.empty((B, self.H, 4), dtype=torch.uint8, device=cmd.device)
        N.check(self._L.lmpc_build_records_device(self._ctx, cmd.data_ptr(), B, rec.data_ptr(), con.data_ptr(),
                                                  self._stream(stream, cmd.device)), "lmpc_build_records_device")
        return rec, con

    def solve_commands_device(self, cmd, grf, status=None, iters=None, stream=None, normals=None) -> None:
        """commands -> records (context buffers) -> solve, all on `stream`."""
        import torch

        B = cmd.shape[0]
        if not cmd.is_cuda or cmd.dtype != torch.uint8 or tuple(cmd.shape) != (B, N.COMMAND_BYTES):
            raise ValueError("commands must be a uint8 device tensor [B, COMMAND_BYTES]")
        if grf.shape != (B, self.H, 12) or grf.dtype != torch.float64 or not grf.is_cuda:
            raise ValueError("bad grf tensor")
        N.check(self._L.lmpc_solve_commands_device(
            self._ctx, cmd.data_ptr(), None if normals is None else normals.data_ptr(), B, grf.data_ptr(),
            None if status is None else status.data_ptr(), None if iters is None else iters.data_ptr(),
            self._stream(stream, cmd.device)), "lmpc_solve_commands_device")

    # ---- the step after the QP: GRF -> joint torque ------------------------------
    def grf_to_torque_device(self, kin: N.LmpcLegKin, rec, joint_pos, grf, stream=None):
        """tau [B, 12] = -J'(R'u0) per leg, from rec (R), joint_pos [B, 12] and grf [B, H, 12] in HBM."""
        import torch

        B = rec.shape[0]
        for t in (rec, joint_pos, grf):
            if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous():
                raise ValueError("grf_to_torque_device expects contiguous f64 device tensors")
        if joint_pos.shape != (B, 12) or grf.shape != (B, self.H, 12) or rec.shape != (B, self.record_len):
            raise ValueError("bad rec/joint_pos/grf shape")
        tau = torch.empty((B, 12), dtype=torch.float64, device=rec.device)
        N.check(self._L.lmpc_grf_to_torque_device(self._ctx, ctypes.byref(kin), rec.data_ptr(), joint_pos.data_ptr(),
                                                  grf.data_ptr(), B, tau.data_ptr(), self._stream(stream, rec.device)),
                "lmpc_grf_to_torque_device")
        return tau

    def sync(self) -> None:
        """Wait for everything the context has issued (lmpc_sync): its own stream and its last device-path launch on
        a caller's stream."""
        N.check(self._L.lmpc_sync(self._ctx), "lmpc_sync")

    def close(self) -> None:
        if self._ctx:
            self._L.lmpc_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# Reference-shaped single-instance API
# ---------------------------------------------------------------------------
@dataclass
class LeggedFeedback:
    """Fields of LeggedFeedback read by the path (LeggedState.h:29-34,52)."""
    root_euler: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_pos: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_ang_vel: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_lin_vel: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_rot_mat: np.ndarray = field(default_factory=lambda: np.eye(3))
    foot_pos_abs: np.ndarray = field(default_factory=lambda: np.zeros((3, 4)))  # 3 x NUM_LEG


@dataclass
class LeggedCtrl:
    """Fields of LeggedCtrl read/written by the path (LeggedState.h:79-96)."""
    root_euler_d: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_pos_d: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_lin_vel_d_rel: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_lin_vel_d_world: np.ndarray = field(default_factory=lambda: np.zeros(3))
    root_ang_vel_d_rel: np.ndarray = field(default_factory=lambda: np.zeros(3))
    plan_contacts: np.ndarray = field(default_factory=lambda: np.ones(4, dtype=bool))


@dataclass
class LeggedParam:
    q_weights: np.ndarray = field(default_factory=lambda: np.zeros(12))
    r_weights: np.ndarray = field(default_factory=lambda: np.full(12, 1e-4))
    robot_mass: float = 13.0
    a1_trunk_inertia: np.ndarray = field(default_factory=lambda: np.diag([0.0158533, 0.0377999, 0.0456542]))
    gait_counter_speed: float = 4.0


@dataclass
class LeggedState:
    fbk: LeggedFeedback = field(default_factory=LeggedFeedback)
    ctrl: LeggedCtrl = field(default_factory=LeggedCtrl)
    param: LeggedParam = field(default_factory=LeggedParam)


class LeggedContactFSM:
    """Gait-phase part of LeggedContactFSM used by the QP (LeggedContactFSM.cpp:5-36,93-212,280-294).
    Swing-trajectory generation (Bezier) is outside the QP path."""

    def __init__(self):
        self.leg_id = 0
        self.gait = N.GAIT_TROT
        self.gait_phase = 0.0
        self.gait_speed = 4.0

    def reset_params(self, state: LeggedState, leg_id: int) -> None:
        self.leg_id = leg_id
        self.gait_speed = float(state.param.gait_counter_speed)
        self.set_default_gait_pattern()

    def set_default_gait_pattern(self):
        self.gait = N.GAIT_TROT

    def set_crawl_gait_pattern(self):
        self.gait = N.GAIT_CRAWL

    def set_trot_with_stand_gait_pattern(self):
        self.gait = N.GAIT_TROT_WITH_STAND

    def set_default_stand_pattern(self):
        self.gait = N.GAIT_STAND

    def reset(self) -> None:
        self.gait_phase = 0.0

    def get_contact_state(self) -> int:
        return N.lib().lmpc_current_contact(self.gait, self.leg_id, self.gait_phase)

    def predict_contact_state(self, dt: float) -> int:
        return N.lib().lmpc_predict_contact(self.gait, self.leg_id, self.gait_phase, self.gait_speed, dt)


class ConvexQPSolver:
    """Drop-in shaped like legged::ConvexQPSolver (ConvexQPSolver.h:23-40)."""

    def __init__(self, q_weights, r_weights, horizon: int = 30, robot_mass: float = 13.0,
                 trunk_inertia=None, mu: float = 0.3, f_max: float = 180.0, gravity: float = 9.8,
                 dt: float = 0.01, device: int = 0):
        p = N.LmpcParams()
        for i in range(12):
            p.q_weights[i] = float(q_weights[i])
            p.r_weights[i] = float(r_weights[i])
        p.robot_mass = float(robot_mass)
        I = np.diag([0.0158533, 0.0377999, 0.0456542]) if trunk_inertia is None else np.asarray(trunk_inertia)
        for i, v in enumerate(np.asarray(I, dtype=np.float64).reshape(9)):
            p.trunk_inertia[i] = float(v)
        p.mu, p.f_max, p.gravity, p.dt = float(mu), float(f_max), float(gravity), float(dt)
        self.H = int(horizon)
        self._p = p
        # Same defaults as the C++ drop-in (legged::ConvexQPSolver): warm start on, so every tick runs on the
        # Riccati kernel from the previous tick's verified active set shifted one step (the reference's OSQP
        # warm-starts too, ConvexQPSolver.cpp:185); cold solves (set_warm_start(False)) take the condensed
        # interior point, since round 3 also the lower-latency dense kernel for one QP per call.
        self._dev = BatchedConvexQPSolver(p, self.H, 1, device, dense_path="ipm")
        self._dev.reserve_warm(1)
        self._rec = np.zeros((1, 33 + 12 * self.H))
        self._con = np.ones((1, self.H, 4), dtype=np.uint8)
        self._warm = True
        self._act = None  # last verified active set [1, H, 4]
        self.last_status = 0
        self.last_iterations = 0

    def set_warm_start(self, on: bool) -> None:
        self._warm = bool(on)
        self._act = None

    @property
    def warm_start(self) -> bool:
        return self._warm

    def calc_mpc_reference(self, state: LeggedState, leg_FSM) -> None:
        st = N.LmpcStateIn()
        st.root_euler[:] = list(state.fbk.root_euler)
        st.root_pos[:] = list(state.fbk.root_pos)
        st.root_ang_vel[:] = list(state.fbk.root_ang_vel)
        st.root_lin_vel[:] = list(state.fbk.root_lin_vel)
        st.root_rot_mat[:] = list(np.asarray(state.fbk.root_rot_mat, dtype=np.float64).reshape(9))
        st.foot_pos_abs[:] = list(np.asarray(state.fbk.foot_pos_abs, dtype=np.float64).T.reshape(12))
        st.root_euler_d[:] = list(state.ctrl.root_euler_d)
        st.root_pos_d[:] = list(state.ctrl.root_pos_d)
        st.root_lin_vel_d_rel[:] = list(state.ctrl.root_lin_vel_d_rel)
        st.root_ang_vel_d_rel[:] = list(state.ctrl.root_ang_vel_d_rel)
        vdw = np.zeros(3)
        N.check(N.lib().lmpc_pack_record(ctypes.byref(self._p), self.H, ctypes.byref(st), _dp(self._rec[0]),
                                         _dp(vdw)), "lmpc_pack_record")
        state.ctrl.root_lin_vel_d_world = vdw  # ConvexQPSolver.cpp:260 writes it back
        # update_bound_constraints (ConvexQPSolver.cpp:329-346)
        for j in range(4):
            self._con[0, 0, j] = 1 if state.ctrl.plan_contacts[j] else 0
        for i in range(1, self.H):
            for j in range(4):
                self._con[0, i, j] = leg_FSM[j].predict_contact_state(i * self._p.dt)

    def update_cons_matrix(self) -> None:
        """No-op: the constraint values are built on the device inside the solve."""

    def compute_grfs(self, state: LeggedState) -> np.ndarray:
        if self._warm:
            act_in = None if self._act is None else BatchedConvexQPSolver.shift_active_set(self._act)
            grf, status, iters, act = self._dev.solve_warm(self._rec, self._con, act_in)
            self._act = act if int(status[0]) == 0 else None
        else:
            grf, status, iters = self._dev.solve(self._rec, self._con)
        self.last_status = int(status[0])
        self.last_iterations = int(iters[0])
        self.last_solution = grf[0]
        return grf[0, 0].copy()  # u_0: FL, FR, RL, RR x (fx, fy, fz), world frame

"""ctypes binding of the C-ABI in include/lmpc/lmpc.h (liblmpc.so, built in-tree).

The product path has no fallback: if the HIP library is missing or the device
code cannot run, calls raise instead of silently computing on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "liblmpc.so")

LMPC_OK = 0
LMPC_QP_CONVERGED = 0
LMPC_QP_MAX_ITER = 1
LMPC_QP_NAN = 2
LMPC_MAX_HORIZON = 32
GAIT_TROT, GAIT_CRAWL, GAIT_TROT_WITH_STAND, GAIT_STAND = 0, 1, 2, 3

# every symbol include/lmpc/lmpc.h declares (checked by tests/test_capi.py)
EXPORTED_SYMBOLS = (
    "lmpc_params_go1", "lmpc_params_a1", "lmpc_options_default", "lmpc_record_len",
    "lmpc_abi_version", "lmpc_strerror", "lmpc_create", "lmpc_destroy", "lmpc_set_options",
    "lmpc_set_params", "lmpc_reserve", "lmpc_solve_batch", "lmpc_solve_batch_device", "lmpc_sync",
    "lmpc_predict_contact", "lmpc_current_contact", "lmpc_contact_schedule", "lmpc_pack_record",
    "lmpc_synth_cfg_go1", "lmpc_synth_cfg_a1_standing", "lmpc_synth_fill",
    # ABI 2: terrain extension
    "lmpc_terrain_frame", "lmpc_solve_batch_ex", "lmpc_solve_batch_warm", "lmpc_shift_active_set", "lmpc_solve_batch_device_ex", "lmpc_synth_normals",
    # on-device input generation
    "lmpc_command_to_record", "lmpc_build_records_device", "lmpc_solve_commands_device",
    "lmpc_synth_commands", "lmpc_synth_commands_device", "lmpc_synth_normals_device",
    # GRF -> joint torque
    "lmpc_leg_kin_default", "lmpc_foot_jacobian", "lmpc_grf_to_torque", "lmpc_grf_to_torque_device",
    # ABI 3: dense-path selection
    "lmpc_set_dense_path", "lmpc_get_dense_path", "lmpc_set_riccati_path", "lmpc_get_riccati_path",
    # ABI 7: per-leg gait phases, warm-start workspace
    "lmpc_contact_schedule_legs", "lmpc_reserve_warm",
)
ABI_VERSION = 7
# include/lmpc/lmpc_hoqp.h: batched hierarchical QP (whole-body control)
HOQP_SYMBOLS = (
    "lmpc_hoqp_dims_wbc", "lmpc_hoqp_options_default", "lmpc_hoqp_record_len", "lmpc_hoqp_slack_len",
    "lmpc_hoqp_lds_bytes", "lmpc_hoqp_create", "lmpc_hoqp_destroy", "lmpc_hoqp_set_options", "lmpc_hoqp_solve_batch",
    "lmpc_hoqp_solve_device", "lmpc_hoqp_sync", "lmpc_wbc_tasks", "lmpc_wbc_tasks_device",
    "lmpc_hoqp_solve_batch_z", "lmpc_hoqp_solve_device_z",
)
HOQP_MAX_LEVELS = 4
# include/lmpc/lmpc_multi.h: one process, several GPUs (liblmpc_multi.so, RCCL scatter / gather)
MULTI_LIB_PATH = os.path.join(_HERE, "lib", "liblmpc_multi.so")
MULTI_SYMBOLS = (
    "lmpc_multi_abi_version", "lmpc_multi_shard", "lmpc_multi_create", "lmpc_multi_destroy", "lmpc_multi_num_devices",
    "lmpc_multi_set_options", "lmpc_multi_set_dense_path", "lmpc_multi_solve_commands_device",
    "lmpc_multi_solve_synth_device", "lmpc_multi_solve_commands",
)
MULTI_ABI_VERSION = 1
LMPC_ERR_COMM = -6


class LmpcParams(ctypes.Structure):
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


class LmpcOptions(ctypes.Structure):
    _fields_ = [
        ("max_iter", ctypes.c_int),
        ("max_rounds", ctypes.c_int),
        ("max_attempts", ctypes.c_int),
        ("tol_mu", ctypes.c_double),
        ("tol_p", ctypes.c_double),
        ("tol_d", ctypes.c_double),
        # ABI 5: the dense paths' caps and the warm-start budget
        ("gi_max_steps", ctypes.c_int),
        ("dense_iter_cap", ctypes.c_int),
        ("dense_polish_iter", ctypes.c_int),
        ("warm_rounds", ctypes.c_int),
        # ABI 7: the certificate's dynamics check (relative to the state scale)
        ("tol_x", ctypes.c_double),
    ]


class LmpcStateIn(ctypes.Structure):
    _fields_ = [
        ("root_euler", ctypes.c_double * 3),
        ("root_pos", ctypes.c_double * 3),
        ("root_ang_vel", ctypes.c_double * 3),
        ("root_lin_vel", ctypes.c_double * 3),
        ("root_rot_mat", ctypes.c_double * 9),
        ("foot_pos_abs", ctypes.c_double * 12),
        ("root_euler_d", ctypes.c_double * 3),
        ("root_pos_d", ctypes.c_double * 3),
        ("root_lin_vel_d_rel", ctypes.c_double * 3),
        ("root_ang_vel_d_rel", ctypes.c_double * 3),
    ]


class LmpcSynthCfg(ctypes.Structure):
    _fields_ = [
        ("gait", ctypes.c_int),
        ("gait_speed", ctypes.c_double),
        ("default_feet", ctypes.c_double * 12),
        ("standing", ctypes.c_int),
    ]


class LmpcCommand(ctypes.Structure):
    _fields_ = [
        ("state", LmpcStateIn),
        ("gait_phase", ctypes.c_double * 4),  # per leg (ABI 7)
        ("gait_speed", ctypes.c_double),
        ("gait", ctypes.c_int32),
        ("plan_contacts", ctypes.c_uint8 * 4),
    ]


COMMAND_BYTES = ctypes.sizeof(LmpcCommand)  # 408


class LmpcLegKin(ctypes.Structure):
    _fields_ = [
        ("rho_fix", (ctypes.c_double * 5) * 4),
        ("rho_opt", (ctypes.c_double * 3) * 4),
    ]


class LmpcHoqpDims(ctypes.Structure):
    _fields_ = [
        ("num_vars", ctypes.c_int32),
        ("num_levels", ctypes.c_int32),
        ("eq_rows", ctypes.c_int32 * HOQP_MAX_LEVELS),
        ("ineq_rows", ctypes.c_int32 * HOQP_MAX_LEVELS),
    ]


class LmpcHoqpOptions(ctypes.Structure):
    _fields_ = [("max_iter", ctypes.c_int32), ("tol_mu", ctypes.c_double), ("tol_res", ctypes.c_double),
                ("crossover", ctypes.c_int32)]


class LmpcWbcInput(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_double * 324), ("nle", ctypes.c_double * 18), ("J", ctypes.c_double * 216),
        ("dJv", ctypes.c_double * 12), ("base_accel", ctypes.c_double * 6), ("swing_acc", ctypes.c_double * 12),
        ("forces_des", ctypes.c_double * 12), ("torque_limits", ctypes.c_double * 3), ("mu", ctypes.c_double),
        ("contact", ctypes.c_int32 * 4),
    ]


class NativeLibraryError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def lib():
    """Load liblmpc.so (raises NativeLibraryError if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("LMPC_LIB") or LIB_PATH  # LMPC_LIB: diagnostic builds (tools/) only
        if not os.path.exists(path):
            raise NativeLibraryError(
                f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(path)
        vp, dp, i32p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        pp = ctypes.POINTER(LmpcParams)
        L.lmpc_params_go1.argtypes = [pp]
        L.lmpc_params_a1.argtypes = [pp]
        L.lmpc_options_default.argtypes = [ctypes.POINTER(LmpcOptions)]
        L.lmpc_record_len.argtypes = [ctypes.c_int]
        L.lmpc_record_len.restype = ctypes.c_int
        L.lmpc_abi_version.restype = ctypes.c_int
        L.lmpc_strerror.argtypes = [ctypes.c_int]
        L.lmpc_strerror.restype = ctypes.c_char_p
        L.lmpc_create.argtypes = [pp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.lmpc_create.restype = ctypes.c_int
        L.lmpc_destroy.argtypes = [vp]
        L.lmpc_destroy.restype = None
        L.lmpc_set_options.argtypes = [vp, ctypes.POINTER(LmpcOptions)]
        L.lmpc_set_options.restype = ctypes.c_int
        L.lmpc_set_params.argtypes = [vp, pp]
        L.lmpc_set_params.restype = ctypes.c_int
        L.lmpc_set_dense_path.argtypes = [vp, ctypes.c_int]
        L.lmpc_set_dense_path.restype = ctypes.c_int
        L.lmpc_get_dense_path.argtypes = [vp]
        L.lmpc_get_dense_path.restype = ctypes.c_int
        L.lmpc_set_riccati_path.argtypes = [vp, ctypes.c_int]
        L.lmpc_set_riccati_path.restype = ctypes.c_int
        L.lmpc_get_riccati_path.argtypes = [vp]
        L.lmpc_get_riccati_path.restype = ctypes.c_int
        L.lmpc_reserve.argtypes = [vp, ctypes.c_int]
        L.lmpc_reserve.restype = ctypes.c_int
        if hasattr(L, "lmpc_reserve_warm"):  # ABI 7
            L.lmpc_reserve_warm.argtypes = [vp, ctypes.c_int]
            L.lmpc_reserve_warm.restype = ctypes.c_int
        L.lmpc_solve_batch.argtypes = [vp, dp, u8p, ctypes.c_int, dp, i32p, i32p]
        L.lmpc_solve_batch.restype = ctypes.c_int
        L.lmpc_solve_batch_device.argtypes = [vp, vp, vp, ctypes.c_int, vp, vp, vp, vp]
        L.lmpc_solve_batch_device.restype = ctypes.c_int
        L.lmpc_sync.argtypes = [vp]
        L.lmpc_sync.restype = ctypes.c_int
        L.lmpc_predict_contact.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L.lmpc_predict_contact.restype = ctypes.c_int
        L.lmpc_current_contact.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.lmpc_current_contact.restype = ctypes.c_int
        L.lmpc_contact_schedule.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, u8p, u8p]
        L.lmpc_contact_schedule.restype = ctypes.c_int
        if hasattr(L, "lmpc_contact_schedule_legs"):  # ABI 7 (absent from a one-ABI-behind diagnostic build)
            L.lmpc_contact_schedule_legs.argtypes = [ctypes.c_int, dp, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                                     u8p, u8p]
            L.lmpc_contact_schedule_legs.restype = ctypes.c_int
        L.lmpc_pack_record.argtypes = [pp, ctypes.c_int, ctypes.POINTER(LmpcStateIn), dp, dp]
        L.lmpc_pack_record.restype = ctypes.c_int
        L.lmpc_synth_cfg_go1.argtypes = [ctypes.POINTER(LmpcSynthCfg)]
        L.lmpc_synth_cfg_a1_standing.argtypes = [ctypes.POINTER(LmpcSynthCfg)]
        L.lmpc_synth_fill.argtypes = [pp, ctypes.POINTER(LmpcSynthCfg), ctypes.c_int, ctypes.c_uint64,
                                      ctypes.c_int64, ctypes.c_int, dp, u8p]
        L.lmpc_synth_fill.restype = ctypes.c_int
        L.lmpc_terrain_frame.argtypes = [dp, dp]
        L.lmpc_terrain_frame.restype = None
        L.lmpc_solve_batch_ex.argtypes = [vp, dp, u8p, dp, ctypes.c_int, dp, i32p, i32p]
        L.lmpc_solve_batch_ex.restype = ctypes.c_int
        L.lmpc_solve_batch_warm.argtypes = [vp, dp, u8p, dp, ctypes.c_int, u8p, u8p, dp, i32p, i32p]
        L.lmpc_solve_batch_warm.restype = ctypes.c_int
        L.lmpc_shift_active_set.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p]
        L.lmpc_shift_active_set.restype = None
        L.lmpc_solve_batch_device_ex.argtypes = [vp, vp, vp, vp, ctypes.c_int, vp, vp, vp, vp]
        L.lmpc_solve_batch_device_ex.restype = ctypes.c_int
        L.lmpc_synth_normals.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_double, dp]
        L.lmpc_synth_normals.restype = ctypes.c_int
        cp = ctypes.POINTER(LmpcCommand)
        L.lmpc_command_to_record.argtypes = [pp, ctypes.c_int, cp, dp, u8p]
        L.lmpc_command_to_record.restype = ctypes.c_int
        L.lmpc_build_records_device.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp]
        L.lmpc_build_records_device.restype = ctypes.c_int
        L.lmpc_solve_commands_device.argtypes = [vp, vp, vp, ctypes.c_int, vp, vp, vp, vp]
        L.lmpc_solve_commands_device.restype = ctypes.c_int
        L.lmpc_synth_commands.argtypes = [ctypes.POINTER(LmpcSynthCfg), ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, cp]
        L.lmpc_synth_commands.restype = ctypes.c_int
        L.lmpc_synth_commands_device.argtypes = [vp, ctypes.POINTER(LmpcSynthCfg), ctypes.c_uint64, ctypes.c_int64,
                                                 ctypes.c_int, vp, vp]
        L.lmpc_synth_commands_device.restype = ctypes.c_int
        L.lmpc_synth_normals_device.argtypes = [vp, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, ctypes.c_double, vp, vp]
        L.lmpc_synth_normals_device.restype = ctypes.c_int
        kp = ctypes.POINTER(LmpcLegKin)
        L.lmpc_leg_kin_default.argtypes = [kp]
        L.lmpc_leg_kin_default.restype = None
        L.lmpc_foot_jacobian.argtypes = [kp, ctypes.c_int, dp, dp]
        L.lmpc_foot_jacobian.restype = None
        L.lmpc_grf_to_torque.argtypes = [kp, dp, dp, dp, dp]
        L.lmpc_grf_to_torque.restype = ctypes.c_int
        L.lmpc_grf_to_torque_device.argtypes = [vp, kp, vp, vp, vp, ctypes.c_int, vp, vp]
        L.lmpc_grf_to_torque_device.restype = ctypes.c_int
        hdp, hop = ctypes.POINTER(LmpcHoqpDims), ctypes.POINTER(LmpcHoqpOptions)
        L.lmpc_hoqp_dims_wbc.argtypes = [hdp]
        L.lmpc_hoqp_dims_wbc.restype = None
        L.lmpc_hoqp_options_default.argtypes = [hop]
        L.lmpc_hoqp_options_default.restype = None
        L.lmpc_hoqp_record_len.argtypes = [hdp]
        L.lmpc_hoqp_record_len.restype = ctypes.c_int64
        L.lmpc_hoqp_lds_bytes.argtypes = [hdp]
        L.lmpc_hoqp_lds_bytes.restype = ctypes.c_int64
        L.lmpc_hoqp_slack_len.argtypes = [hdp]
        L.lmpc_hoqp_slack_len.restype = ctypes.c_int
        L.lmpc_hoqp_create.argtypes = [hdp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.lmpc_hoqp_create.restype = ctypes.c_int
        L.lmpc_hoqp_destroy.argtypes = [vp]
        L.lmpc_hoqp_destroy.restype = None
        L.lmpc_hoqp_set_options.argtypes = [vp, hop]
        L.lmpc_hoqp_set_options.restype = ctypes.c_int
        L.lmpc_hoqp_solve_batch.argtypes = [vp, dp, ctypes.c_int, dp, dp, i32p, i32p]
        L.lmpc_hoqp_solve_batch.restype = ctypes.c_int
        L.lmpc_hoqp_solve_device.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp, vp, vp]
        L.lmpc_hoqp_solve_device.restype = ctypes.c_int
        L.lmpc_hoqp_solve_batch_z.argtypes = [vp, dp, ctypes.c_int, dp, dp, i32p, i32p, dp, i32p]
        L.lmpc_hoqp_solve_batch_z.restype = ctypes.c_int
        L.lmpc_hoqp_solve_device_z.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp]
        L.lmpc_hoqp_solve_device_z.restype = ctypes.c_int
        L.lmpc_hoqp_sync.argtypes = [vp]
        L.lmpc_hoqp_sync.restype = ctypes.c_int
        L.lmpc_wbc_tasks.argtypes = [ctypes.POINTER(LmpcWbcInput), dp]
        L.lmpc_wbc_tasks.restype = ctypes.c_int
        L.lmpc_wbc_tasks_device.argtypes = [vp, ctypes.c_int, vp, vp]
        L.lmpc_wbc_tasks_device.restype = ctypes.c_int
        # exactly this ABI, diagnostic builds (LMPC_LIB) included: the command and options structs above are ABI-7
        # layouts, and an older library would read their fields at the wrong offsets without an error
        if L.lmpc_abi_version() != ABI_VERSION:
            raise NativeLibraryError(f"{path}: ABI version {L.lmpc_abi_version()}, this binding is ABI {ABI_VERSION}")
        _lib = L
        return L


_mlib = None


def multi_lib():
    """Load liblmpc_multi.so (raises NativeLibraryError if it was not built)."""
    global _mlib
    lib()  # liblmpc.so first: the multi-device library links it
    with _lock:
        if _mlib is not None:
            return _mlib
        if not os.path.exists(MULTI_LIB_PATH):
            raise NativeLibraryError(f"{MULTI_LIB_PATH} not found: build it with __graft_entry__.build()")
        M = ctypes.CDLL(MULTI_LIB_PATH)
        vp, i32p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)
        pp = ctypes.POINTER(LmpcParams)
        M.lmpc_multi_abi_version.restype = ctypes.c_int
        M.lmpc_multi_shard.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p, i32p]
        M.lmpc_multi_shard.restype = None
        M.lmpc_multi_create.argtypes = [pp, ctypes.c_int, i32p, ctypes.c_int, ctypes.POINTER(vp)]
        M.lmpc_multi_create.restype = ctypes.c_int
        M.lmpc_multi_destroy.argtypes = [vp]
        M.lmpc_multi_destroy.restype = None
        M.lmpc_multi_num_devices.argtypes = [vp]
        M.lmpc_multi_num_devices.restype = ctypes.c_int
        M.lmpc_multi_set_options.argtypes = [vp, ctypes.POINTER(LmpcOptions)]
        M.lmpc_multi_set_options.restype = ctypes.c_int
        M.lmpc_multi_set_dense_path.argtypes = [vp, ctypes.c_int]
        M.lmpc_multi_set_dense_path.restype = ctypes.c_int
        M.lmpc_multi_solve_commands_device.argtypes = [vp, vp, vp, ctypes.c_int, vp, vp, vp, vp]
        M.lmpc_multi_solve_commands_device.restype = ctypes.c_int
        M.lmpc_multi_solve_synth_device.argtypes = [vp, ctypes.POINTER(LmpcSynthCfg), ctypes.c_uint64, ctypes.c_int64,
                                                    ctypes.c_int, ctypes.c_double, vp, vp, vp]
        M.lmpc_multi_solve_synth_device.restype = ctypes.c_int
        M.lmpc_multi_solve_commands.argtypes = [vp, vp, vp, ctypes.c_int, vp, vp, vp]
        M.lmpc_multi_solve_commands.restype = ctypes.c_int
        if M.lmpc_multi_abi_version() != MULTI_ABI_VERSION:
            raise NativeLibraryError("liblmpc_multi.so ABI version mismatch")
        _mlib = M
        return M


def check(rc: int, what: str = "lmpc") -> None:
    if rc != LMPC_OK:
        msg = "RCCL communication failed" if rc == LMPC_ERR_COMM else lib().lmpc_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: {msg} ({rc})")

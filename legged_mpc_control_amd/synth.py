"""Robot presets and seeded synthetic problem batches (host side, via the C-ABI).

Instances are keyed by (seed, global_index) with a counter-based Philox4x32-10
generator, so every rank (and the CPU oracle) builds identical inputs without
moving any bytes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N

# BASELINE.json configs -> (robot, gait, H, batch)
CONFIGS = {
    1: dict(name="a1_standing_h10", robot="a1", gait=N.GAIT_TROT, H=10, batch=1, standing=True),
    2: dict(name="go1_trot_h10_b1024", robot="go1", gait=N.GAIT_TROT, H=10, batch=1024, standing=False),
    3: dict(name="go1_trot_h20_b8192", robot="go1", gait=N.GAIT_TROT, H=20, batch=8192, standing=False),
    4: dict(name="go1_mixed_h10_b65536", robot="go1", gait=-1, H=10, batch=65536, standing=False),
    5: dict(name="go1_trot_h30_b4096", robot="go1", gait=N.GAIT_TROT, H=30, batch=4096, standing=False),
}
BASE_SEED = 20261015
TERRAIN_THETA_MAX = 0.3  # config 4 terrain tilt, theta ~ U(0, 0.3) rad


def params(robot: str = "go1") -> N.LmpcParams:
    p = N.LmpcParams()
    if robot == "go1":
        N.lib().lmpc_params_go1(ctypes.byref(p))
    elif robot == "a1":
        N.lib().lmpc_params_a1(ctypes.byref(p))
    else:
        raise ValueError(robot)
    return p


def synth_cfg(robot: str = "go1", gait: int = N.GAIT_TROT, standing: bool = False) -> N.LmpcSynthCfg:
    c = N.LmpcSynthCfg()
    if standing:
        N.lib().lmpc_synth_cfg_a1_standing(ctypes.byref(c))
    else:
        N.lib().lmpc_synth_cfg_go1(ctypes.byref(c))
        if robot == "a1":
            # A1 sim: feet (+-0.17, +-0.17, -0.3), gait speed 3.5 (gazebo_a1_convex.yaml:19-36)
            a1 = N.LmpcSynthCfg()
            N.lib().lmpc_synth_cfg_a1_standing(ctypes.byref(a1))
            c.default_feet[:] = a1.default_feet[:]
            c.gait_speed = a1.gait_speed
        c.gait = gait
    return c


def fill(p: N.LmpcParams, cfg: N.LmpcSynthCfg, H: int, count: int, seed: int, first_index: int = 0):
    """-> (rec [count, 33+12H] f64, contact [count, H, 4] u8)."""
    rl = 33 + 12 * H
    rec = np.zeros((count, rl), dtype=np.float64)
    con = np.zeros((count, H, 4), dtype=np.uint8)
    rc = N.lib().lmpc_synth_fill(ctypes.byref(p), ctypes.byref(cfg), H, seed, first_index, count,
                                 rec.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 con.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    N.check(rc, "lmpc_synth_fill")
    return rec, con


def normals(count: int, seed: int, first_index: int = 0, theta_max: float = TERRAIN_THETA_MAX) -> np.ndarray:
    """Per-leg terrain normals [count, 4, 3] (own Philox stream; records are unaffected)."""
    out = np.zeros((count, 4, 3), dtype=np.float64)
    N.check(N.lib().lmpc_synth_normals(seed, first_index, count, float(theta_max),
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "lmpc_synth_normals")
    return out


def terrain_frame(n) -> np.ndarray:
    """Contact frame R (columns t1, t2, n) of a ground normal (lmpc_terrain_frame)."""
    n = np.ascontiguousarray(n, dtype=np.float64).reshape(3)
    R = np.zeros(9)
    N.lib().lmpc_terrain_frame(n.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                               R.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return R.reshape(3, 3)


def config_normals(config_id: int, count: int | None = None, first_index: int = 0):
    """Terrain normals of a config (config 4 only; None = flat ground for the others)."""
    if config_id != 4:
        return None
    n = CONFIGS[config_id]["batch"] if count is None else count
    return normals(n, BASE_SEED + config_id, first_index)


def commands(cfg: N.LmpcSynthCfg, count: int, seed: int, first_index: int = 0):
    """Host synthetic commands -> ctypes array of LmpcCommand (lmpc_synth_commands)."""
    arr = (N.LmpcCommand * count)()
    N.check(N.lib().lmpc_synth_commands(ctypes.byref(cfg), seed, first_index, count, arr), "lmpc_synth_commands")
    return arr


def command_to_record(p: N.LmpcParams, H: int, cmd: N.LmpcCommand):
    """Host expansion of one command -> (rec [33+12H], contact [H, 4])."""
    rec = np.zeros(33 + 12 * H, dtype=np.float64)
    con = np.zeros((H, 4), dtype=np.uint8)
    N.check(N.lib().lmpc_command_to_record(ctypes.byref(p), H, ctypes.byref(cmd),
                                           rec.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                           con.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "lmpc_command_to_record")
    return rec, con


def config_cfg(config_id: int) -> N.LmpcSynthCfg:
    c = CONFIGS[config_id]
    return synth_cfg(c["robot"], c["gait"], c["standing"])


def config_batch(config_id: int, count: int | None = None, first_index: int = 0, H: int | None = None):
    """Synthetic batch for a BASELINE.json config -> (params, H, rec, contact)."""
    c = CONFIGS[config_id]
    H = c["H"] if H is None else H
    p = params(c["robot"])
    cfg = synth_cfg(c["robot"], c["gait"], c["standing"])
    n = c["batch"] if count is None else count
    rec, con = fill(p, cfg, H, n, BASE_SEED + config_id, first_index)
    return p, H, rec, con

"""Several GPUs from one process (include/lmpc/lmpc_multi.h, liblmpc_multi.so): the batch sharded over the
devices, RCCL only for the scatter of commands and the gather of GRFs.

This is the C++ host's multi-GPU path (no torch in the library); the Python class below binds it for the tests.
bench.py's one-process-per-GPU torch.distributed path shards the same way (lmpc_multi_shard == dist.split_range).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _native as N


def shard(batch: int, n_devices: int, r: int):
    """(first, count) of device r's contiguous shard (lmpc_multi_shard)."""
    f, c = ctypes.c_int32(), ctypes.c_int32()
    N.multi_lib().lmpc_multi_shard(int(batch), int(n_devices), int(r), ctypes.byref(f), ctypes.byref(c))
    return f.value, c.value


class MultiDeviceSolver:
    """lmpc_multi over `devices` (distinct; devices[0] is the root that holds device-pointer batches)."""

    def __init__(self, params: N.LmpcParams, horizon: int, devices: Sequence[int], dense_path: str | None = None,
                 options: N.LmpcOptions | None = None):
        self._M = N.multi_lib()
        self.H = int(horizon)
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int32 * len(self.devices))(*self.devices)
        self._m = ctypes.c_void_p()
        N.check(self._M.lmpc_multi_create(ctypes.byref(params), self.H, arr, len(self.devices), ctypes.byref(self._m)),
                "lmpc_multi_create")
        if options is not None:
            N.check(self._M.lmpc_multi_set_options(self._m, ctypes.byref(options)), "lmpc_multi_set_options")
        if dense_path is not None:
            from .solver import BatchedConvexQPSolver

            N.check(self._M.lmpc_multi_set_dense_path(self._m, BatchedConvexQPSolver.DENSE_PATHS[dense_path]),
                    "lmpc_multi_set_dense_path")

    @property
    def num_devices(self) -> int:
        return self._M.lmpc_multi_num_devices(self._m)

    def _root_check(self, name, t, dtype, shape):
        import torch

        from .hoqp import check_device_tensor

        check_device_tensor(name, t, dtype, shape, torch.device("cuda", self.devices[0]))

    def solve_commands_device(self, d_cmd, d_grf, d_status=None, d_iters=None, d_normals=None, stream=None):
        """Commands uint8 [B, 408] on devices[0] -> GRFs [B, H, 12] (+ status, iters) on devices[0]; synchronous."""
        import torch

        B = int(d_cmd.shape[0])
        self._root_check("d_cmd", d_cmd, torch.uint8, (B, N.COMMAND_BYTES))
        self._root_check("d_grf", d_grf, torch.float64, (B, self.H, 12))
        if d_status is not None:
            self._root_check("d_status", d_status, torch.int32, (B,))
        if d_iters is not None:
            self._root_check("d_iters", d_iters, torch.int32, (B,))
        if d_normals is not None:
            self._root_check("d_normals", d_normals, torch.float64, (B, 4, 3))
        if stream is None:
            stream = torch.cuda.current_stream(self.devices[0])
        sptr = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
        p = lambda t: None if t is None else t.data_ptr()
        N.check(self._M.lmpc_multi_solve_commands_device(self._m, d_cmd.data_ptr(), p(d_normals), B, d_grf.data_ptr(),
                                                         p(d_status), p(d_iters), sptr),
                "lmpc_multi_solve_commands_device")

    def solve_synth_device(self, cfg: N.LmpcSynthCfg, batch: int, seed: int, first_index: int = 0,
                           theta_max: float = -1.0):
        """Every device generates and solves its own shard; results gathered to devices[0] (torch tensors)."""
        import torch

        dev = torch.device("cuda", self.devices[0])
        grf = torch.empty((batch, self.H, 12), dtype=torch.float64, device=dev)
        st = torch.empty(batch, dtype=torch.int32, device=dev)
        it = torch.empty(batch, dtype=torch.int32, device=dev)
        N.check(self._M.lmpc_multi_solve_synth_device(self._m, ctypes.byref(cfg), int(seed), int(first_index), int(batch),
                                                      float(theta_max), grf.data_ptr(), st.data_ptr(), it.data_ptr()),
                "lmpc_multi_solve_synth_device")
        return grf, st, it

    def solve_commands(self, cmd: np.ndarray, normals: np.ndarray | None = None):
        """Host commands uint8 [B, 408] (+ normals [B, 4, 3]) -> host (grf, status, iters)."""
        cmd = np.ascontiguousarray(cmd, dtype=np.uint8)
        B = cmd.shape[0]
        if cmd.shape != (B, N.COMMAND_BYTES):
            raise ValueError("commands must be uint8 [B, COMMAND_BYTES]")
        if normals is not None:
            normals = np.ascontiguousarray(normals, dtype=np.float64)
            if normals.shape != (B, 4, 3):
                raise ValueError("normals must be [B, 4, 3]")
        grf = np.zeros((B, self.H, 12))
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros(B, dtype=np.int32)
        N.check(self._M.lmpc_multi_solve_commands(self._m, cmd.ctypes.data, None if normals is None else normals.ctypes.data,
                                                  B, grf.ctypes.data, st.ctypes.data, it.ctypes.data),
                "lmpc_multi_solve_commands")
        return grf, st, it

    def close(self) -> None:
        if self._m:
            self._M.lmpc_multi_destroy(self._m)
            self._m = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

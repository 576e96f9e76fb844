"""Hierarchical QP of the whole-body controller on the GPU.

Host-side mirror of the reference's interface over the C-ABI of include/lmpc/lmpc_hoqp.h:

  * `Task` -- include/wbc_ctrl/task.h:16-64 (a x = b, d x <= f; `+` stacks self first);
  * `HoQp(task, higher_problem=None)` -- include/wbc_ctrl/HoQp.h:17-50: each object is one priority level,
    solved on construction (HoQp.cpp:19-27); getSolutions(), getStackedSlackSolutions(), getStackedZMatrix(),
    getSlackedNumVars(), getStackedTasks() as in the reference.  The chain is solved on the device in one
    launch (every level's tasks are passed down; the higher levels' results are recomputed identically);
  * `HoqpBatch` -- the batched form: many robots, one launch, host or device (torch) buffers.

The product path is the HIP kernel (lmpc_hoqp.hip); there is no CPU fallback: without the built library or a
GPU these raise.  Numerics and what is comparable across solvers: include/lmpc/lmpc_hoqp.h.
"""
from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N


class Task:
    """a x = b (least squares), d x <= f (slacked).  A 0x0 block (the reference's `matrix_t()`) is absorbed
    by the other operand of `+` (task.h:40-51)."""

    def __init__(self, a=None, b=None, d=None, f=None):
        self.a = np.zeros((0, 0)) if a is None else np.atleast_2d(np.asarray(a, dtype=np.float64))
        self.b = np.zeros(0) if b is None else np.asarray(b, dtype=np.float64).reshape(-1)
        self.d = np.zeros((0, 0)) if d is None else np.atleast_2d(np.asarray(d, dtype=np.float64))
        self.f = np.zeros(0) if f is None else np.asarray(f, dtype=np.float64).reshape(-1)
        if self.a.shape[0] != self.b.size or self.d.shape[0] != self.f.size:
            raise ValueError("Task: row counts of a/b or d/f differ")

    def __add__(self, rhs: "Task") -> "Task":
        def cat(m1, m2):
            if m1.shape[1] <= 0:
                return m2
            if m2.shape[1] <= 0:
                return m1
            if m1.shape[1] != m2.shape[1]:
                raise ValueError("Task +: column counts differ")
            return np.vstack([m1, m2])
        return Task(cat(self.a, rhs.a), np.concatenate([self.b, rhs.b]), cat(self.d, rhs.d),
                    np.concatenate([self.f, rhs.f]))

    def num_vars(self) -> int:
        return max(self.a.shape[1], self.d.shape[1])


def dims_of(levels: Sequence[Task]) -> N.LmpcHoqpDims:
    """Batch dimensions of one chain (level 0 first); num_vars from the first task (HoQp.cpp:49)."""
    if not 1 <= len(levels) <= N.HOQP_MAX_LEVELS:
        raise ValueError(f"1..{N.HOQP_MAX_LEVELS} levels")
    d = N.LmpcHoqpDims()
    d.num_vars = levels[0].num_vars()
    d.num_levels = len(levels)
    for l, t in enumerate(levels):
        for blk in (t.a, t.d):
            if blk.shape[0] and blk.shape[1] != d.num_vars:
                raise ValueError(f"level {l}: {blk.shape[1]} columns, expected {d.num_vars}")
        d.eq_rows[l] = t.a.shape[0]
        d.ineq_rows[l] = t.d.shape[0]
    return d


def record_len(dims: N.LmpcHoqpDims) -> int:
    n = N.lib().lmpc_hoqp_record_len(ctypes.byref(dims))
    if n < 0:
        raise ValueError("hierarchical QP dimensions outside the kernel's limits (include/lmpc/lmpc_hoqp.h)")
    return int(n)


def pack(levels: Sequence[Task], dims: N.LmpcHoqpDims, out: Optional[np.ndarray] = None) -> np.ndarray:
    """One instance record: per level a (row-major), b, d (row-major), f."""
    n = dims.num_vars
    rec = np.zeros(record_len(dims)) if out is None else out
    o = 0
    for l, t in enumerate(levels):
        m, s = dims.eq_rows[l], dims.ineq_rows[l]
        if t.a.shape[0] != m or t.d.shape[0] != s:
            raise ValueError(f"level {l}: rows ({t.a.shape[0]}, {t.d.shape[0]}) != dims ({m}, {s})")
        if m:
            rec[o:o + m * n] = t.a.reshape(-1)
        o += m * n
        rec[o:o + m] = t.b
        o += m
        if s:
            rec[o:o + s * n] = t.d.reshape(-1)
        o += s * n
        rec[o:o + s] = t.f
        o += s
    return rec


class HoqpBatch:
    """A batch of same-shaped hierarchies on one device (lmpc_hoqp_create)."""

    def __init__(self, dims: N.LmpcHoqpDims, max_batch: int, device: int = 0):
        self._L = N.lib()
        self.dims = dims
        self.max_batch = max_batch
        self.device = device
        self.n = dims.num_vars
        self.levels = dims.num_levels
        self.rec_len = record_len(dims)
        self.slack_len = int(self._L.lmpc_hoqp_slack_len(ctypes.byref(dims)))
        self._ctx = ctypes.c_void_p()
        # a context is not thread-safe (lmpc_hoqp.h) and ctypes releases the GIL during a call: every call that
        # uses it (staging buffers, stream, event) holds this lock
        self._lock = threading.Lock()
        N.check(self._L.lmpc_hoqp_create(ctypes.byref(dims), max_batch, device, ctypes.byref(self._ctx)),
                "lmpc_hoqp_create")

    def close(self):
        if self._ctx:
            self._L.lmpc_hoqp_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, max_iter=None, tol_mu=None, tol_res=None, crossover=None):
        o = N.LmpcHoqpOptions()
        self._L.lmpc_hoqp_options_default(ctypes.byref(o))
        if crossover is not None:
            o.crossover = int(crossover)
        if max_iter is not None:
            o.max_iter = max_iter
        if tol_mu is not None:
            o.tol_mu = tol_mu
        if tol_res is not None:
            o.tol_res = tol_res
        with self._lock:
            N.check(self._L.lmpc_hoqp_set_options(self._ctx, ctypes.byref(o)), "lmpc_hoqp_set_options")

    def solve(self, records: np.ndarray, with_z: bool = False):
        """Host path.  records [B][rec_len] -> x [B][levels][n], slack [B][total ineq rows], status [B],
        iters [B][levels]; with_z: also z [B][levels][n][n] and zcols [B][levels], every level's
        getStackedZMatrix() in the first zcols columns (lmpc_hoqp_solve_batch_z)."""
        rec = np.ascontiguousarray(records, dtype=np.float64).reshape(-1, self.rec_len)
        B = rec.shape[0]
        x = np.zeros((B, self.levels, self.n))
        w = np.zeros((B, max(self.slack_len, 1)))
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros((B, self.levels), dtype=np.int32)
        dp, i32p = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
        z = np.zeros((B, self.levels, self.n, self.n)) if with_z else None
        zc = np.zeros((B, self.levels), dtype=np.int32) if with_z else None
        with self._lock:
            N.check(self._L.lmpc_hoqp_solve_batch_z(self._ctx, rec.ctypes.data_as(dp), B, x.ctypes.data_as(dp),
                                                    w.ctypes.data_as(dp), st.ctypes.data_as(i32p),
                                                    it.ctypes.data_as(i32p),
                                                    z.ctypes.data_as(dp) if with_z else None,
                                                    zc.ctypes.data_as(i32p) if with_z else None),
                    "lmpc_hoqp_solve_batch_z")
        if with_z:
            return x, w[:, :self.slack_len], st, it, z, zc
        return x, w[:, :self.slack_len], st, it

    def solve_device(self, d_rec, d_x, d_w, d_status=None, d_iters=None, stream=None, d_z=None, d_zcols=None):
        """Device path on torch tensors (resident in HBM), asynchronous on `stream` (default: torch's current);
        d_z [B][levels][n][n] / d_zcols [B][levels]: every level's getStackedZMatrix() (optional)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        B = int(d_rec.shape[0]) if d_rec.dim() >= 1 else -1
        dev = torch.device("cuda", self.device)
        check_device_tensor("d_rec", d_rec, torch.float64, (B, self.rec_len), dev)
        check_device_tensor("d_x", d_x, torch.float64, (B, self.levels, self.n), dev)
        check_device_tensor("d_w", d_w, torch.float64, (B, max(self.slack_len, 1)), dev, allow_shape=(B, self.slack_len))
        if d_status is not None:
            check_device_tensor("d_status", d_status, torch.int32, (B,), dev)
        if d_iters is not None:
            check_device_tensor("d_iters", d_iters, torch.int32, (B, self.levels), dev)
        if d_z is not None:
            check_device_tensor("d_z", d_z, torch.float64, (B, self.levels, self.n, self.n), dev)
        if d_zcols is not None:
            if d_z is None:
                raise ValueError("d_zcols needs d_z")
            check_device_tensor("d_zcols", d_zcols, torch.int32, (B, self.levels), dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        with self._lock:
            N.check(self._L.lmpc_hoqp_solve_device_z(self._ctx, ptr(d_rec), B, ptr(d_x), ptr(d_w), ptr(d_status),
                                                     ptr(d_iters), ptr(d_z), ptr(d_zcols),
                                                     ctypes.c_void_p(s.cuda_stream)),
                    "lmpc_hoqp_solve_device_z")


def check_device_tensor(name, t, dtype, shape, device, allow_shape=None):
    """A raw pointer handed to the device path must be a contiguous tensor of this dtype and shape on the
    context's device: anything else turns into out-of-bounds device writes or wrong results."""
    if t is None or not hasattr(t, "is_cuda") or not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, the context is on {device}")
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if tuple(t.shape) != tuple(shape) and (allow_shape is None or tuple(t.shape) != tuple(allow_shape)):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")


_batches = {}
_batches_lock = threading.Lock()


def _batch_for(dims: N.LmpcHoqpDims, device: int) -> HoqpBatch:
    key = (dims.num_vars, dims.num_levels, tuple(dims.eq_rows), tuple(dims.ineq_rows), device)
    with _batches_lock:
        if key not in _batches:
            _batches[key] = HoqpBatch(dims, 1, device)
        return _batches[key]


class HoQp:
    """One priority level (HoQp.h:17-50).  HoQp(task) is the highest level; HoQp(task, higher) the next."""

    def __init__(self, task: Task, higher_problem: Optional["HoQp"] = None, device: int = 0):
        self.task_ = task
        self.higher_problem_ = higher_problem
        chain: List[Task] = [task]
        h = higher_problem
        while h is not None:
            chain.insert(0, h.task_)
            h = h.higher_problem_
        self._level = len(chain) - 1
        dims = dims_of(chain)
        batch = _batch_for(dims, device)
        x, w, st, it, z, zc = batch.solve(pack(chain, dims)[None, :], with_z=True)
        self._x = x[0, self._level].copy()
        self._z = z[0, self._level, :, :int(zc[0, self._level])].copy()
        self._slack = w[0, :sum(dims.ineq_rows[:self._level + 1])].copy()
        self.status = int(st[0])
        self.iterations = it[0].copy()
        # stacked tasks, current level first (HoQp.cpp:58)
        prev = higher_problem.getStackedTasks() if higher_problem is not None else Task(
            np.zeros((0, dims.num_vars)), None, np.zeros((0, dims.num_vars)), None)
        self._stacked = task + prev

    def getSolutions(self) -> np.ndarray:  # HoQp.h:41-45
        return self._x.copy()

    def getStackedSlackSolutions(self) -> np.ndarray:  # HoQp.h:36-39
        return self._slack.copy()

    def getStackedTasks(self) -> Task:  # HoQp.h:31-34
        return self._stacked

    def getSlackedNumVars(self) -> int:  # HoQp.h:47-50
        return self._stacked.d.shape[0]

    def getStackedZMatrix(self) -> np.ndarray:  # HoQp.h:26-29: Z after this level (n x nd), Eigen's FullPivLU basis
        return self._z.copy()

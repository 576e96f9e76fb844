"""Restatement of the reference's hierarchical QP (HoQp) -- TEST INFRASTRUCTURE ONLY.

SURVEY.md 8f row 4 (the whole-body-control QP family).  The reference builds one HoQp per priority
level (src/legged_ctrl/src/wbc_ctrl/HoQp.cpp, include/wbc_ctrl/HoQp.h, include/wbc_ctrl/task.h) and
solves each level with qpOASES (`QProblem`, MPC options, nWSR 20; HoQp.cpp:158-174).  qpOASES and
Eigen are not under /root/reference; this module restates

  - the level formulation (HoQp.cpp:74-143): over (z, w) -- z the coordinates in the null space Z of
    every higher level's equalities, w this level's slacks --
        min 1/2 |A Z z + A x_prev - b|^2 + 1/2 |w|^2 + 1/2 1e-12 |z|^2
        s.t. -w <= 0,  D_prev Z z <= f_prev - D_prev x_prev + w_prev,  D Z z - w <= f - D x_prev
    and x = x_prev + Z z (HoQp.h:42-46);
  - Z <- Z ker(A Z) with Eigen's FullPivLU kernel basis (HoQp.cpp:145-153; Eigen 3.3 FullPivLU::compute
    and kernel_retval), which is NOT orthonormal: with the 1e-12 term the optimum depends on the basis
    whenever A Z is rank-deficient, so the basis construction is restated step by step;
  - the stacking order of tasks and slacks, including the reference's quirk: `stacked_tasks_ = task_ +
    stacked_tasks_prev_` puts the current level FIRST (HoQp.cpp:60) while the stacked slack vector puts it
    LAST (HoQp.cpp:176-182), so from the third level on the frozen slacks are paired with the rows of a
    different level (kept, as the reference computes it);
  - the QP solve, by an exact primal active-set method (Nocedal & Wright, Alg. 16.3) from the feasible
    point z = 0, w = max(0, D x_prev - f): qpOASES solves the same strictly convex QP, whose optimum is
    unique, so any exact method returns it up to conditioning (the 1e-12 regularisation makes the KKT
    system ill-conditioned along the null space of A Z: the checker solves it in x87 extended precision,
    where a double solve -- qpOASES's included -- keeps ~4 digits along those directions).

Parity status: the reference's only test (src/test/ho_qp_test.cpp) checks properties on Eigen `Random`
data; `reference_test_tasks()` regenerates that data exactly (glibc rand() after srand(0), Eigen 3.3's
`-1 + 2 rand()/RAND_MAX`, column-major fill) and tests/test_hoqp_oracle.py applies the test's checks.
Every level is also certified by its KKT conditions.  No reference output values exist to pin against.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

EPS = np.finfo(np.float64).eps


# ---------------------------------------------------------------------------------------------
# Eigen FullPivLU (Eigen/src/LU/FullPivLU.h, 3.3): compute(), rank(), kernel()
# ---------------------------------------------------------------------------------------------
def fullpivlu(A):
    """-> dict(lu, p, q, nonzero_pivots, maxpivot).  p, q: permutation index arrays (P = perm of rows)."""
    lu = np.array(A, dtype=np.float64, copy=True)
    rows, cols = lu.shape
    size = min(rows, cols)
    rt = np.arange(size)
    ct = np.arange(size)
    nonzero = size
    maxpivot = 0.0
    for k in range(size):
        corner = np.abs(lu[k:, k:])
        # maxCoeff(&r, &c): column-major visit, first strict maximum wins
        best, br, bc = -1.0, 0, 0
        for c in range(corner.shape[1]):
            col = corner[:, c]
            r = int(np.argmax(col))  # first max within the column
            if col[r] > best:
                best, br, bc = col[r], r, c
        if best == 0.0:
            nonzero = k
            rt[k:] = np.arange(k, size)
            ct[k:] = np.arange(k, size)
            break
        r, c = br + k, bc + k
        maxpivot = max(maxpivot, best)
        rt[k], ct[k] = r, c
        if r != k:
            lu[[k, r], :] = lu[[r, k], :]
        if c != k:
            lu[:, [k, c]] = lu[:, [c, k]]
        if k < rows - 1:
            lu[k + 1:, k] /= lu[k, k]
        if k < size - 1:
            lu[k + 1:, k + 1:] -= np.outer(lu[k + 1:, k], lu[k, k + 1:])
    p = np.arange(rows)
    for k in range(size - 1, -1, -1):  # m_p.applyTranspositionOnTheRight(k, rt[k]), k descending
        p[[k, rt[k]]] = p[[rt[k], k]]
    q = np.arange(cols)
    for k in range(size):  # m_q.applyTranspositionOnTheRight(k, ct[k]), k ascending
        q[[k, ct[k]]] = q[[ct[k], k]]
    return dict(lu=lu, p=p, q=q, nonzero_pivots=nonzero, maxpivot=maxpivot)


def _threshold(dec):
    return EPS * min(dec["lu"].shape)  # NumTraits<double>::epsilon() * diagonalSize()


def fullpivlu_rank(dec):
    thr = abs(dec["maxpivot"]) * _threshold(dec)
    return int(sum(abs(dec["lu"][i, i]) > thr for i in range(dec["nonzero_pivots"])))


def fullpivlu_kernel(A):
    """Eigen's kernel basis (cols x dimker): Ker A = Q Ker U, solved on the trapezoid of U."""
    A = np.asarray(A, dtype=np.float64)
    rows, cols = A.shape
    if rows == 0:
        return np.eye(cols)
    dec = fullpivlu(A)
    lu, q = dec["lu"], dec["q"]
    rank = fullpivlu_rank(dec)
    dimker = cols - rank
    if dimker == 0:  # Eigen returns a single zero column rather than an empty basis
        return np.zeros((cols, 1))
    thr = dec["maxpivot"] * _threshold(dec)
    pivots = [i for i in range(dec["nonzero_pivots"]) if abs(lu[i, i]) > thr]
    m = np.zeros((rank, cols))
    for i in range(rank):
        m[i, i:] = lu[pivots[i], i:]  # row i: head(i) zero, tail from U's pivot row
    m[:, :rank] = np.triu(m[:, :rank])
    for i in range(rank):
        m[:, [i, pivots[i]]] = m[:, [pivots[i], i]]
    # upper-triangular solve in place on the right block
    m[:, rank:] = np.linalg.solve(np.triu(m[:, :rank]), m[:, rank:]) if rank else m[:, rank:]
    for i in range(rank - 1, -1, -1):
        m[:, [i, pivots[i]]] = m[:, [pivots[i], i]]
    K = np.zeros((cols, dimker))
    for i in range(rank):
        K[q[i], :] = -m[i, rank:]
    for k in range(dimker):
        K[q[rank + k], k] = 1.0
    return K


# ---------------------------------------------------------------------------------------------
# Tasks (task.h)
# ---------------------------------------------------------------------------------------------
class Task:
    """a x = b (equalities, least squares), d x <= f (inequalities, slacked)."""

    def __init__(self, a=None, b=None, d=None, f=None, n=None):
        if n is not None:  # Task(num_decision_vars): no rows
            a, b, d, f = np.zeros((0, n)), np.zeros(0), np.zeros((0, n)), np.zeros(0)
        self.a = np.asarray(a, dtype=np.float64)
        self.b = np.asarray(b, dtype=np.float64)
        self.d = np.asarray(d, dtype=np.float64)
        self.f = np.asarray(f, dtype=np.float64)

    def __add__(self, rhs):  # concatenateMatrices / concatenateVectors: self first
        def cm(m1, m2):
            if m1.shape[1] <= 0:
                return m2
            if m2.shape[1] <= 0:
                return m1
            return np.vstack([m1, m2])
        return Task(cm(self.a, rhs.a), np.concatenate([self.b, rhs.b]), cm(self.d, rhs.d),
                    np.concatenate([self.f, rhs.f]))

    def copy(self):
        return Task(self.a.copy(), self.b.copy(), self.d.copy(), self.f.copy())


# ---------------------------------------------------------------------------------------------
# dense QP: min 1/2 x'Hx + c'x  s.t.  D x <= f, H positive definite, from a feasible x0
# ---------------------------------------------------------------------------------------------
def solve_ext(K, rhs):
    """Gaussian elimination with partial pivoting in x87 extended precision (np.longdouble): the 1e-12
    regularisation puts the KKT systems' condition near 1e12, where a double solve keeps ~4 digits."""
    A = np.array(K, dtype=np.longdouble)
    b = np.array(rhs, dtype=np.longdouble)
    n = A.shape[0]
    for k in range(n):
        piv = k + int(np.argmax(np.abs(A[k:, k])))
        if A[piv, k] == 0:
            raise np.linalg.LinAlgError("singular KKT system")
        if piv != k:
            A[[k, piv]] = A[[piv, k]]
            b[[k, piv]] = b[[piv, k]]
        m = A[k + 1:, k] / A[k, k]
        A[k + 1:, k:] -= np.outer(m, A[k, k:])
        b[k + 1:] -= m * b[k]
    x = np.zeros(n, dtype=np.longdouble)
    for k in range(n - 1, -1, -1):
        x[k] = (b[k] - A[k, k + 1:] @ x[k + 1:]) / A[k, k]
    return x

def qp_active_set(H, c, D, f, x0, max_iter=500, tol=1e-12):
    """Primal active-set method (Nocedal & Wright, Alg. 16.3).  Returns (x, mu, info); mu >= 0 are
    the multipliers of D x <= f (H x + c + D'mu = 0 at the optimum).  A degenerate vertex (more rows
    active than it has dimensions, e.g. a friction pyramid at its apex projected on a small null space)
    can make the method cycle; it is then re-run on bounds perturbed by 1e-13 of their scale, row by
    row (Charnes' anti-cycling perturbation), which moves the optimum by that much."""
    try:
        return _qp_active_set(H, c, D, f, x0, max_iter, tol)
    except RuntimeError:
        m = D.shape[0]
        eps = 1e-13 * (1.0 + float(np.max(np.abs(f)))) if m else 0.0
        fp = f + eps * (1.0 + np.arange(m)) / max(m, 1)
        x, mu, info = _qp_active_set(H, c, D, fp, x0, max_iter, tol)
        info["perturbed"] = eps
        return x, mu, info


def _qp_active_set(H, c, D, f, x0, max_iter=500, tol=1e-12):
    n, m = H.shape[0], D.shape[0]
    x = np.array(x0, dtype=np.longdouble)
    scale = 1.0 + np.max(np.abs(f)) if m else 1.0
    # rows that are zero up to rounding (a higher level's row projected on a null space it is orthogonal to)
    # constrain nothing: they never enter the working set
    dscale = float(np.max(np.abs(D))) if m else 0.0
    live = [i for i in range(m) if float(np.max(np.abs(D[i]))) > 1e-12 * dscale]
    W = [i for i in live if abs(float(D[i] @ x) - f[i]) <= tol * scale]
    # keep a linearly independent working set
    Wi = []
    for i in W:
        if np.linalg.matrix_rank(D[Wi + [i]]) == len(Wi) + 1:
            Wi.append(i)
    W = Wi
    at_min = False
    seen, bland = set(), False  # anti-cycling: a working set seen twice at a stationary point -> Bland's rule
    for it in range(max_iter):
        g = np.asarray(H, dtype=np.longdouble) @ x + c
        k = len(W)
        K = np.zeros((n + k, n + k))
        K[:n, :n] = H
        if k:
            K[:n, n:] = D[W].T
            K[n:, :n] = D[W]
        rhs = np.concatenate([-g, np.zeros(k, dtype=np.longdouble)])
        sol = solve_ext(K, rhs)
        p, lam = sol[:n], sol[n:].astype(np.float64)
        # at the working set's minimiser: after a full unblocked step (the next step is rounding noise,
        # which the ill-conditioned KKT systems here make larger than any fixed tolerance), or p ~ 0
        if at_min or float(np.max(np.abs(p))) <= 1e-13 * (1.0 + float(np.max(np.abs(x)))):
            at_min = False
            if k == 0 or np.min(lam) >= -1e-14 * (1.0 + np.max(np.abs(lam))):
                mu = np.zeros(m)
                mu[W] = lam
                return x.astype(np.float64), mu, dict(iters=it, working_set=list(W))
            key = frozenset(W)
            bland = bland or key in seen
            seen.add(key)
            if bland:  # drop the lowest-index row with a negative multiplier (degenerate vertices cycle otherwise)
                neg = [j for j in range(k) if lam[j] < -1e-14 * (1.0 + np.max(np.abs(lam)))]
                W.pop(min(neg, key=lambda j: W[j]))
            else:
                W.pop(int(np.argmin(lam)))
            continue
        alpha, block = 1.0, -1
        pn = float(np.max(np.abs(p)))
        for i in live:
            if i in W:
                continue
            dp = float(D[i] @ p)
            # a row moving at rounding level along p is not blocking: it lies in the span of the working set
            # (e.g. a zero inequality row's slack bound 0 - w <= 0 duplicates -w <= 0)
            if dp > 1e-13 * pn * float(np.max(np.abs(D[i]))):
                a = float((f[i] - D[i] @ x)) / dp
                # a row in the span of the working set cannot block a direction in its null space: it only
                # does so by rounding (degenerate vertices, e.g. a pyramid at its apex)
                if a < alpha and np.linalg.matrix_rank(D[W + [i]]) == k + 1:
                    alpha, block = a, i
        x = x + np.longdouble(max(alpha, 0.0)) * p
        if block >= 0:
            W.append(block)
        else:
            at_min = True
    raise RuntimeError("qp_active_set: iteration cap")


def kkt_residual(H, c, D, f, x, mu):
    """max of stationarity, primal infeasibility, dual infeasibility and complementarity (scaled)."""
    stat = np.max(np.abs(H @ x + c + D.T @ mu)) if len(x) else 0.0
    if D.shape[0]:
        s = f - D @ x
        prim = max(0.0, -np.min(s))
        dual = max(0.0, -np.min(mu))
        comp = np.max(np.abs(mu * s))
    else:
        prim = dual = comp = 0.0
    return max(stat, prim, dual, comp)


# ---------------------------------------------------------------------------------------------
# HoQp (HoQp.cpp / HoQp.h)
# ---------------------------------------------------------------------------------------------
class HoQp:
    def __init__(self, task: Task, higher: "HoQp | None" = None):
        self.task = task
        self.higher = higher
        self._init_vars()       # HoQp.cpp:26-67
        self._formulate()       # :69-143
        self._solve()           # :158-174
        self._build_z()         # :145-153
        self._stack_slacks()    # :176-182

    def _init_vars(self):
        t = self.task
        self.num_slack = t.d.shape[0]
        self.has_eq = t.a.shape[0] > 0
        self.has_ineq = self.num_slack > 0
        if self.higher is not None:
            h = self.higher
            self.z_prev = h.stacked_z
            self.tasks_prev = h.stacked_tasks
            self.slack_prev = h.stacked_slack
            self.x_prev = h.solution()
            self.num_prev_slack = h.stacked_tasks.d.shape[0]
            self.nx = self.z_prev.shape[1]
        else:
            self.nx = max(t.a.shape[1], t.d.shape[1])
            self.tasks_prev = Task(n=self.nx)
            self.z_prev = np.eye(self.nx)
            self.slack_prev = np.zeros(0)
            self.x_prev = np.zeros(self.nx)
            self.num_prev_slack = 0
        self.stacked_tasks = t + self.tasks_prev  # current level first (HoQp.cpp:60)

    def _formulate(self):
        t, nx, nv = self.task, self.nx, self.num_slack
        H = np.zeros((nx + nv, nx + nv))
        if self.has_eq:
            az = t.a @ self.z_prev
            H[:nx, :nx] = az.T @ az + 1e-12 * np.eye(nx)
        H[nx:, nx:] = np.eye(nv)
        c = np.zeros(nx + nv)
        if self.has_eq:
            c[:nx] = (t.a @ self.z_prev).T @ (t.a @ self.x_prev - t.b)
        D = np.zeros((2 * nv + self.num_prev_slack, nx + nv))
        D[:nv, nx:] = -np.eye(nv)
        D[nv:nv + self.num_prev_slack, :nx] = self.tasks_prev.d @ self.z_prev
        if self.has_ineq:
            D[nv + self.num_prev_slack:, :nx] = t.d @ self.z_prev
            D[nv + self.num_prev_slack:, nx:] = -np.eye(nv)
        f = np.zeros(2 * nv + self.num_prev_slack)
        f[nv:nv + self.num_prev_slack] = self.tasks_prev.f - self.tasks_prev.d @ self.x_prev + self.slack_prev
        if self.has_ineq:
            f[nv + self.num_prev_slack:] = t.f - t.d @ self.x_prev
        self.H, self.c, self.D, self.f = H, c, D, f

    def _solve(self):
        nx, nv = self.nx, self.num_slack
        x0 = np.zeros(nx + nv)
        if self.has_ineq:  # z = 0 with the smallest feasible slacks
            x0[nx:] = np.maximum(0.0, self.task.d @ self.x_prev - self.task.f)
        viol = self.D @ x0 - self.f
        if viol.size and np.max(viol) > 1e-9 * (1.0 + np.max(np.abs(self.f))):
            # only the frozen higher-level rows can be violated at z = 0, and only through the slack
            # ordering quirk (level >= 3); qpOASES would report the QP infeasible, which the reference ignores
            raise ValueError("HoQp level infeasible at z = 0 (reference slack-ordering quirk)")
        sol, mu, info = qp_active_set(self.H, self.c, self.D, self.f, x0)
        self.qp_solution, self.qp_mu, self.qp_info = sol, mu, info
        self.z_sol = sol[:nx]
        self.w_sol = sol[nx:]

    def _build_z(self):
        if self.has_eq:
            self.stacked_z = self.z_prev @ fullpivlu_kernel(self.task.a @ self.z_prev)
        else:
            self.stacked_z = self.z_prev

    def _stack_slacks(self):
        if self.higher is not None:
            self.stacked_slack = np.concatenate([self.higher.stacked_slack, self.w_sol])  # current level LAST
        else:
            self.stacked_slack = self.w_sol

    # HoQp.h accessors
    def solution(self):
        return self.x_prev + self.z_prev @ self.z_sol

    def kkt(self):
        return kkt_residual(self.H, self.c, self.D, self.f, self.qp_solution, self.qp_mu)


# ---------------------------------------------------------------------------------------------
# the reference test's data (src/test/ho_qp_test.cpp:10-22)
# ---------------------------------------------------------------------------------------------
def _libc():
    return ctypes.CDLL(ctypes.util.find_library("c"))


def eigen_random(rows, cols, libc):
    """Eigen 3.3 Matrix::Random: -1 + 2 rand()/RAND_MAX per coefficient, column-major order."""
    RAND_MAX = 2147483647  # glibc
    out = np.zeros((rows, cols))
    for c in range(cols):
        for r in range(rows):
            out[r, c] = -1.0 + 2.0 * float(libc.rand()) / float(RAND_MAX)
    return out


def reference_test_tasks():
    """(task_0, task_1) exactly as ho_qp_test.cpp builds them after srand(0)."""
    libc = _libc()
    libc.srand(0)
    a0 = eigen_random(2, 4, libc)
    d0 = eigen_random(2, 4, libc)
    t0 = Task(a0, np.ones(2), d0, np.ones(2))
    t1 = t0.copy()
    t1.a = np.ones((2, 4))
    return t0, t1

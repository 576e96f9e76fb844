"""CPU tests of the hierarchical-QP restatement (oracle/hoqp.py): the reference's own
test (src/test/ho_qp_test.cpp) on its exact data, Eigen's FullPivLU kernel basis, KKT certificates."""
import numpy as np
import pytest

from oracle import hoqp as Q


def is_approx(a, b, prec):
    """Eigen's isApprox: |a - b| <= prec * min(|a|, |b|)."""
    return np.linalg.norm(a - b) <= prec * min(np.linalg.norm(a), np.linalg.norm(b))


def test_reference_test_data_matches_eigen_random():
    """srand(0) + Matrix::Random(2, 4) twice: the first matrix is Eigen's documented Random() example."""
    t0, t1 = Q.reference_test_tasks()
    first = [0.680375, -0.211234, 0.566198, 0.59688, 0.823295, -0.604897, -0.329554, 0.536459]
    assert np.allclose(t0.a.T.reshape(-1), first, atol=5e-7)
    assert np.array_equal(t1.a, np.ones((2, 4))) and np.array_equal(t1.d, t0.d)


def test_reference_two_task_checks():
    """ho_qp_test.cpp:24-45, verbatim checks on the reference's data (prec 1e-6)."""
    t0, t1 = Q.reference_test_tasks()
    h0 = Q.HoQp(t0)
    h1 = Q.HoQp(t1, h0)
    x0, x1 = h0.solution(), h1.solution()
    s0, s1 = h0.stacked_slack, h1.stacked_slack
    prec = 1e-6
    assert s0.shape == (2,) and s1.shape == (4,)
    if np.all(s0 == 0.0):  # isApprox(Zero): exactly zero
        assert is_approx(t0.a @ x0, t0.b, prec)
    if np.all(s1 == 0.0):
        assert is_approx(t1.a @ x1, t1.b, prec)
        assert is_approx(t0.a @ x1, t0.b, prec)
    y = t0.d @ x0
    assert np.all(y <= t0.f + s0[: y.size] + 1e-12)
    y = t1.d @ x1
    assert np.all(y <= t1.f + s1[: y.size] + 1e-12)  # the test indexes the stacked slacks from the front
    assert h0.kkt() <= 1e-10 and h1.kkt() <= 1e-10


def test_level0_without_active_inequalities_is_min_norm():
    """H = A'A + 1e-12 I: with no active inequality the first level returns pinv(A) b -- to ~1e-5 only:
    A'A formed in double carries ~1e-16 errors along the null space of A, where the regulariser is 1e-12
    (the reference forms H the same way, HoQp.cpp:83-85)."""
    t0, _ = Q.reference_test_tasks()
    h0 = Q.HoQp(t0)
    assert np.all(t0.d @ h0.solution() < t0.f)
    assert np.allclose(h0.solution(), np.linalg.pinv(t0.a) @ t0.b, atol=1e-4)
    H = t0.a.T @ t0.a + 1e-12 * np.eye(4)  # the regularised optimum of the double-formed H, solved exactly
    assert np.allclose(h0.solution(), Q.solve_ext(H, t0.a.T @ t0.b).astype(np.float64), atol=1e-9)


@pytest.mark.parametrize("seed", range(40))
def test_fullpivlu_kernel(seed):
    rng = np.random.default_rng(seed)
    r, c = int(rng.integers(1, 7)), int(rng.integers(1, 9))
    A = rng.standard_normal((r, c))
    if r > 1 and seed % 3 == 0:
        A[-1] = 2.0 * A[0] - A[1 % r]  # rank-deficient rows
    K = Q.fullpivlu_kernel(A)
    rank = np.linalg.matrix_rank(A)
    assert K.shape == (c, max(c - rank, 1))
    assert np.max(np.abs(A @ K)) <= 1e-10 * (1 + np.max(np.abs(A)))
    if c > rank:
        # Eigen's basis: an identity block on the non-pivot columns Q[rank:]
        q = Q.fullpivlu(A)["q"]
        assert np.array_equal(K[q[rank:], :], np.eye(c - rank))
        assert np.linalg.matrix_rank(K) == c - rank
    else:
        assert not np.any(K)  # full column rank: one zero column


def test_fullpivlu_matches_permuted_lu():
    rng = np.random.default_rng(7)
    A = rng.standard_normal((4, 6))
    dec = Q.fullpivlu(A)
    lu, p, q = dec["lu"], dec["p"], dec["q"]
    L = np.tril(lu[:, :4], -1) + np.eye(4)
    U = np.triu(lu)
    # Eigen's convention P A Q = L U: P moves row i to p[i] (P A = A[argsort(p)]), A Q = A[:, q]
    assert np.allclose(A[np.argsort(p)][:, q], L @ U, atol=1e-12)
    # full pivoting: every multiplier is at most 1 in magnitude
    assert np.max(np.abs(np.tril(lu[:, :4], -1))) <= 1.0 + 1e-15


def random_task(rng, n, ne, ni, tight):
    a = rng.standard_normal((ne, n))
    d = rng.standard_normal((ni, n))
    f = rng.uniform(-0.5, 0.2, ni) if tight else rng.uniform(0.5, 2.0, ni)
    return Q.Task(a, rng.standard_normal(ne), d, f)


@pytest.mark.parametrize("seed", range(12))
def test_three_levels_kkt_and_priorities(seed):
    """Three levels (the WBC's depth) with active inequalities: every level's QP is certified by KKT, the
    higher levels' equalities hold on the final solution wherever their slacks vanish, and every level's
    inequalities hold within its own slacks."""
    rng = np.random.default_rng(100 + seed)
    n = 8
    tasks = [random_task(rng, n, 2, 3, tight=seed % 2 == 0), random_task(rng, n, 2, 2, tight=False),
             random_task(rng, n, 3, 2, tight=seed % 3 == 0)]
    levels = []
    for t in tasks:
        levels.append(Q.HoQp(t, levels[-1] if levels else None))
    for lv in levels:
        assert lv.kkt() <= 1e-8 * (1 + np.max(np.abs(lv.c)))
    x = levels[-1].solution()
    x0 = levels[0].solution()
    if np.all(levels[0].w_sol == 0.0) and tasks[0].a.shape[0] < n:
        assert np.allclose(tasks[0].a @ x, tasks[0].a @ x0, atol=1e-6)  # lower levels keep A_0 x fixed
    for lv, t in zip(levels, tasks):
        xs = lv.solution()
        assert np.all(t.d @ xs <= t.f + lv.w_sol + 1e-9)
        assert np.all(lv.w_sol >= -1e-12)


def test_qp_active_set_against_enumeration():
    """Small strictly convex QPs: the active-set result equals the best KKT point over all active sets."""
    import itertools

    rng = np.random.default_rng(3)
    for _ in range(30):
        n, m = 3, 4
        M = rng.standard_normal((n, n))
        H = M @ M.T + 0.1 * np.eye(n)
        c = rng.standard_normal(n)
        D = rng.standard_normal((m, n))
        f = rng.uniform(0.1, 1.0, m)  # x = 0 feasible
        x, mu, _ = Q.qp_active_set(H, c, D, f, np.zeros(n))
        best = None
        for k in range(m + 1):
            for S in itertools.combinations(range(m), k):
                S = list(S)
                K = np.block([[H, D[S].T], [D[S], np.zeros((k, k))]]) if k else H
                try:
                    sol = np.linalg.solve(K, np.concatenate([-c, f[S]]))
                except np.linalg.LinAlgError:
                    continue
                xs, lam = sol[:n], sol[n:]
                if np.all(D @ xs <= f + 1e-10) and np.all(lam >= -1e-10):
                    best = xs
        assert best is not None and np.allclose(x, best, atol=1e-9)
        assert Q.kkt_residual(H, c, D, f, x, mu) <= 1e-10


def test_third_level_pairs_slacks_as_the_reference_does():
    """HoQp.cpp:60 stacks tasks current-first, :176-182 stacks slacks current-last: the third level's frozen
    rows are [task_1; task_0] while its frozen slacks are [w_0; w_1] (kept as the reference computes it)."""
    rng = np.random.default_rng(11)
    n = 6
    t0 = random_task(rng, n, 1, 3, tight=False)
    t1 = random_task(rng, n, 1, 1, tight=False)
    t2 = random_task(rng, n, 1, 2, tight=False)
    h0 = Q.HoQp(t0)
    h1 = Q.HoQp(t1, h0)
    h2 = Q.HoQp(t2, h1)
    assert np.array_equal(h2.tasks_prev.d, np.vstack([t1.d, t0.d]))
    assert np.array_equal(h2.slack_prev, np.concatenate([h0.w_sol, h1.w_sol]))
    nv, npv = 2, 4
    xp = h1.solution()
    expect = np.concatenate([t1.f, t0.f]) - np.vstack([t1.d, t0.d]) @ xp + np.concatenate([h0.w_sol, h1.w_sol])
    assert np.allclose(h2.f[nv:nv + npv], expect)
    assert h2.kkt() <= 1e-9


def test_wbc_shaped_hierarchy():
    """The reference WBC's shape (wbc.cpp:93-97): 42 decision variables (18 qdd, 12 forces, 12 torques);
    level 0 = EOM (18 eq) + torque limits (24 ineq) + friction cone (16 ineq, 4 eq) + no-contact motion;
    levels 1-2 equalities only, their inequality blocks 0x0 as `matrix_t()` builds them -- so the slack
    ordering quirk is inert there.  Every level certified by KKT; higher priorities preserved."""
    rng = np.random.default_rng(21)
    n = 42
    a0 = rng.standard_normal((22, n))
    d0 = rng.standard_normal((40, n))
    t0 = Q.Task(a0, rng.standard_normal(22), d0, rng.uniform(0.0, 2.0, 40))
    t1 = Q.Task(rng.standard_normal((12, n)), rng.standard_normal(12), np.zeros((0, 0)), np.zeros(0))
    t2 = Q.Task(rng.standard_normal((12, n)), rng.standard_normal(12), np.zeros((0, 0)), np.zeros(0))
    h0 = Q.HoQp(t0)
    h1 = Q.HoQp(t1, h0)
    h2 = Q.HoQp(t2, h1)
    for h in (h0, h1, h2):
        assert h.kkt() <= 1e-8 * (1 + np.max(np.abs(h.c)))
    assert h1.num_slack == 0 and h2.num_slack == 0
    assert np.array_equal(h2.slack_prev, h0.w_sol)  # only level 0 has slacks: aligned with its rows
    x = h2.solution()
    assert np.all(t0.d @ x <= t0.f + h0.w_sol + 1e-8)
    if np.all(h0.w_sol == 0.0):
        assert np.allclose(t0.a @ x, t0.a @ h0.solution(), atol=1e-6)

"""Host-side check of the dataflow Cholesky's task list (ba_plan.cpp
build_chol_tasks): executed sequentially in ticket order by a numpy model of
each task (the kernel's tile algebra, chol_dataflow_kernel; potrf(k) also
applies its tile's last update and solves trsm(k+1,k); bsolve(c) also applies
bupd(c,c-1)), every dependency
the kernel polls for must already hold, every task must run exactly once, and
the result must be the damped SPD solution.  No GPU needed."""
import ctypes

import numpy as np
import pytest

POTRF, TRSM, UPD, BSOLVE, BUPD = range(5)


def tasks_for(n):
    from droid_backends._lib import check, lib
    h = ctypes.c_void_p()
    check(lib.droid_chol_plan_create(n, ctypes.byref(h)), "chol plan")
    try:
        ld, nt, fo = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.droid_chol_plan_info(h, ctypes.byref(ld), ctypes.byref(nt), ctypes.byref(fo)), "info")
        out = np.zeros(max(4 * nt.value, 1), np.int32)
        check(lib.droid_chol_plan_tasks(h, out.ctypes.data_as(ctypes.c_void_p)), "tasks")
        return out[:4 * nt.value].reshape(-1, 4), ld.value
    finally:
        lib.droid_ba_plan_destroy(h)


def emulate(M, n, tasks):
    """M: (n+1, n) augmented (rows 0..n-1 lower A, row n = b). Returns x."""
    nbc, nbr = (n + 63) // 64, (n + 64) // 64
    ver = np.zeros((nbr, nbc), int)
    yver = np.zeros(nbc, int)
    xdone = np.zeros(nbc, int)
    linv = {}
    y = np.zeros(nbc * 64)
    x = np.zeros(n)
    blk = lambda i: slice(64 * i, min(64 * i + 64, n + 1))
    col = lambda k: slice(64 * k, min(64 * k + 64, n))
    seen = set()
    for t, i, j, k in tasks:
        key = (t, i, j, k)
        assert key not in seen
        seen.add(key)
        if t == POTRF:                       # + the tile's last update (k,k,k-1) and trsm(k+1,k)
            assert ver[k, k] >= max(k - 1, 0)
            R = blk(k)
            Bp = col(k).stop - col(k).start
            T = M[R, col(k)].copy()
            if k > 0:
                assert ver[k, k - 1] >= k
                T -= M[R, col(k - 1)] @ M[col(k), col(k - 1)].T
            L = np.linalg.cholesky(np.tril(T[:Bp]) + np.tril(T[:Bp], -1).T)
            T[:Bp] = L
            if T.shape[0] > Bp:                                      # rhs row inside the diagonal tile
                T[Bp:] = np.linalg.solve(L, T[Bp:].T).T
                y[64 * k:64 * k + Bp] = T[Bp]
                yver[k] = 1
            M[R, col(k)] = T
            linv[k] = np.linalg.inv(L)
            ver[k, k] = k + 1
            if k + 1 < nbr:
                assert ver[k + 1, k] >= k
                M[blk(k + 1), col(k)] = M[blk(k + 1), col(k)] @ linv[k].T
                if k + 1 == nbr - 1:
                    y[64 * k:64 * k + Bp] = M[n, col(k)]
                    yver[k] = 1
                ver[k + 1, k] = k + 1
        elif t == TRSM:
            assert ver[i, k] >= k and ver[k, k] >= k + 1
            M[blk(i), col(k)] = M[blk(i), col(k)] @ linv[k].T
            if i == nbr - 1:
                y[64 * k:64 * k + (col(k).stop - col(k).start)] = M[n, col(k)]
                yver[k] = 1
            ver[i, k] = k + 1
        elif t == UPD:
            assert ver[i, j] >= k and ver[i, k] >= k + 1 and ver[j, k] >= k + 1
            M[blk(i), col(j)] -= M[blk(i), col(k)] @ M[col(j), col(k)].T
            ver[i, j] = k + 1
        elif t == BSOLVE:                    # + bupd(c, c-1)
            c = i
            assert ver[c, c] >= c + 1 and yver[c] >= 1 + (nbc - 1 - c)
            Bp = col(c).stop - col(c).start
            x[col(c)] = linv[c].T @ y[64 * c:64 * c + Bp]
            xdone[c] = 1
            if c > 0:
                assert ver[c, c - 1] >= c and yver[c - 1] >= 1 + (nbc - 1 - c)
                y[64 * (c - 1):64 * c] -= M[col(c), col(c - 1)].T @ x[col(c)]
                yver[c - 1] = 1 + (nbc - c)
        else:
            r, c = i, j
            assert xdone[r] and ver[r, c] >= c + 1 and yver[c] >= 1 + (nbc - 1 - r)
            y[64 * c:64 * c + 64] -= M[col(r), col(c)].T @ x[col(r)]
            yver[c] = 1 + (nbc - r)
    return x, len(seen)


@pytest.mark.parametrize("n", [6, 63, 64, 65, 128, 130, 300, 1530])
def test_task_list_solves_spd(n):
    rng = np.random.default_rng(n)
    tasks, ld = tasks_for(n)
    assert ld % 8 == 0 and ld >= n + 1
    nbc, nbr = (n + 63) // 64, (n + 64) // 64
    expect = nbc + sum(max(0, nbr - k - 2) for k in range(nbc)) \
        + sum((nbr - jb) * jb for jb in range(1, nbc)) - (nbc - 1) + nbc + nbc * (nbc - 1) // 2 - (nbc - 1)
    assert len(tasks) == expect
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    A = (Q * np.geomspace(1, 1e3, n)) @ Q.T
    b = rng.normal(size=n)
    M = np.zeros((n + 1, n))
    M[:n] = np.tril(A)
    M[n] = b
    x, ran = emulate(M, n, tasks)
    assert ran == len(tasks)
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-8, atol=1e-10)

"""Host-side check of the dataflow Cholesky's plan (ba_plan.cpp
build_chol_structure): the task list is executed sequentially in ticket order
by a numpy model of each task (the kernel's tile algebra, chol_dataflow_kernel;
potrf(k) also applies its tile's last update and solves tile (k+1,k) when it
exists, and may run potrf(k+1) next (a chain); trsm(i,k) may also apply the
update (i,k+1,k); bcol(c) is the whole back solve of block column c);
every version the kernel polls for must already hold, every tile's updates must
arrive in sequence, every task must run exactly once, and the result must be
the damped SPD solution.  Dense systems (the chol-only plan) and the
tile-sparse, pose-permuted reduced systems of BA plans (C2, C3 and a C5-shaped
2048-keyframe graph) are covered.  No GPU needed."""
import ctypes
import time

import numpy as np
import pytest

POTRF, TRSM, UPD, BCOL = range(4)


def _lib():
    from droid_backends._lib import check, lib
    return check, lib


def structure(h, n):
    check, lib = _lib()
    nt, fo, ns, nsa = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib.droid_chol_plan_info(h, ctypes.byref(nt), ctypes.byref(fo), ctypes.byref(ns), ctypes.byref(nsa)),
          "info")
    nbc, nbr = (n + 63) // 64, (n + 64) // 64
    tasks = np.zeros(max(8 * nt.value, 1), np.int32)
    check(lib.droid_chol_plan_tasks(h, tasks.ctypes.data_as(ctypes.c_void_p)), "tasks")
    slot = np.zeros(max(nbr * nbc, 1), np.int32)
    fin = np.zeros(max(ns.value, 1), np.int32)
    ycnt = np.zeros(max(nbc, 1), np.int32)
    outmap = np.zeros(max(n, 1), np.int32)
    check(lib.droid_chol_plan_structure(h, slot.ctypes.data_as(ctypes.c_void_p), fin.ctypes.data_as(ctypes.c_void_p),
                                        ycnt.ctypes.data_as(ctypes.c_void_p), outmap.ctypes.data_as(ctypes.c_void_p)),
          "structure")
    return dict(tasks=tasks[:8 * nt.value].reshape(-1, 8), slot=slot[:nbr * nbc].reshape(nbr, nbc),
                fin=fin[:ns.value], ycnt=ycnt[:nbc], outmap=outmap[:n], nslots=ns.value, nslots_input=nsa.value,
                nbc=nbc, nbr=nbr)


def chol_plan(n):
    check, lib = _lib()
    h = ctypes.c_void_p()
    check(lib.droid_chol_plan_create(n, ctypes.byref(h)), "chol plan")
    try:
        return structure(h, n)
    finally:
        lib.droid_ba_plan_destroy(h)


def ba_plan(ii, jj, N, t0, t1, H=4, W=8):
    check, lib = _lib()
    ii = np.ascontiguousarray(ii, np.int64)
    jj = np.ascontiguousarray(jj, np.int64)
    h = ctypes.c_void_p()
    kx = np.unique(np.concatenate([np.arange(t0, t1), ii]))
    t = time.perf_counter()
    check(lib.droid_ba_plan_create(ii.ctypes.data_as(ctypes.c_void_p), jj.ctypes.data_as(ctypes.c_void_p), len(ii),
                                   N, H, W, t0, t1, len(kx), 0, 0, 2 ** 31 - 1, ctypes.byref(h)), "ba plan")
    secs = time.perf_counter() - t
    try:
        P = t1 - t0
        kind, nwide, ntasks = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        perm = np.zeros(max(P, 1), np.int32)
        check(lib.droid_ba_plan_order(h, ctypes.byref(kind), perm.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(nwide), ctypes.byref(ntasks)), "order")
        s = structure(h, 6 * P)
        s.update(perm=perm[:P], kind=kind.value, nwide=nwide.value, plan_seconds=secs)
        return s
    finally:
        lib.droid_ba_plan_destroy(h)


def emulate(M, n, st):
    """M: (n+1, n) augmented (rows 0..n-1 lower A, row n = b), modified in
    place on the plan's tiles only.  Returns x (permuted order)."""
    nbc, nbr, slot, fin, ycnt = st["nbc"], st["nbr"], st["slot"], st["fin"], st["ycnt"]
    ver = np.zeros(st["nslots"], int)
    yver = np.zeros(nbc, int)
    xdone = np.zeros(nbc, int)
    lver = np.zeros(nbc, int)     # L_kk^-1 stored: published by potrf(k) after its pivot tiles
    linv = {}
    y = np.zeros(nbc * 64)
    x = np.zeros(n)
    blk = lambda i: slice(64 * i, min(64 * i + 64, n + 1))
    col = lambda k: slice(64 * k, min(64 * k + 64, n))
    S = lambda i, j: slot[i, j]
    seen = set()
    tasks = st["tasks"]
    for q, (t, i, j, k, a, b, c, ch) in enumerate(tasks):
        if t == POTRF and c:                                         # chained: potrf(k) runs potrf(k+1) next
            nx = tasks[c - 1]
            assert c - 1 > q and nx[0] == POTRF and nx[3] == k + 1 and nx[4] == k and nx[7] == 1 and b
        if t == POTRF and ch:                                        # the placeholder of a chained potrf
            assert any(tt[0] == POTRF and tt[6] == q + 1 for tt in tasks[:q])
    for t, i, j, k, a, b, c, _ in tasks:
        key = (t, i, j, k)
        assert key not in seen
        seen.add(key)
        if t == POTRF:
            s = S(k, k)
            assert s >= 0 and ver[s] >= (fin[s] - 2 if a >= 0 else 0)
            R = blk(k)
            Bp = col(k).stop - col(k).start
            T = M[R, col(k)].copy()
            if a >= 0:                                               # the tile's last update (k,k,a)
                assert ver[s] == fin[s] - 2 and ver[S(k, a)] >= fin[S(k, a)]
                T -= M[R, col(a)] @ M[col(k), col(a)].T
            L = np.linalg.cholesky(np.tril(T[:Bp]) + np.tril(T[:Bp], -1).T)
            T[:Bp] = L
            if T.shape[0] > Bp:                                      # rhs row inside the diagonal tile
                T[Bp:] = np.linalg.solve(L, T[Bp:].T).T
                y[64 * k:64 * k + Bp] = T[Bp]
                yver[k] = 1
            M[R, col(k)] = T
            linv[k] = np.linalg.inv(L)
            ver[s] = fin[s]
            for d, fused in ((1, b),):                               # the tile (k+1,k)
                if fused:
                    sb = S(k + d, k)
                    assert sb >= 0 and ver[sb] >= fin[sb] - 1
                    # forward substitution against L_kk itself (not via L_kk^-1)
                    M[blk(k + d), col(k)] = np.linalg.solve(L, M[blk(k + d), col(k)].T).T
                    if k + d == nbr - 1:
                        y[64 * k:64 * k + Bp] = M[n, col(k)]
                        yver[k] = 1
                    ver[sb] = fin[sb]
                else:                                                # the plan fuses (k+1,k) whenever it exists
                    assert k + d >= nbr or S(k + d, k) < 0
            lver[k] = 1
        elif t == TRSM:
            s = S(i, k)
            assert s >= 0 and ver[s] >= fin[s] - 1 and lver[k]
            M[blk(i), col(k)] = M[blk(i), col(k)] @ linv[k].T
            if i == nbr - 1:
                y[64 * k:64 * k + (col(k).stop - col(k).start)] = M[n, col(k)]
                yver[k] = 1
            ver[s] = fin[s]
            if b:                                                    # + the update (i,k+1,k), the tile's last
                su = S(i, k + 1)
                assert su >= 0 and ver[su] == a and ver[S(k + 1, k)] >= fin[S(k + 1, k)] and a == fin[su] - 2
                M[blk(i), col(k + 1)] -= M[blk(i), col(k)] @ M[col(k + 1), col(k)].T
                ver[su] = a + 1
        elif t == UPD:
            s = S(i, j)
            assert s >= 0 and ver[s] == a                           # updates arrive in sequence
            assert ver[S(i, k)] >= fin[S(i, k)] and ver[S(j, k)] >= fin[S(j, k)]
            M[blk(i), col(j)] -= M[blk(i), col(k)] @ M[col(j), col(k)].T
            ver[s] = a + 1
        else:                                                        # bcol(c): the whole back solve of x_c
            c = i
            assert lver[c] and yver[c] >= 1
            Bp = col(c).stop - col(c).start
            yc = y[64 * c:64 * c + Bp].copy()
            rows = [r for r in range(nbc - 1, c, -1) if S(r, c) >= 0]
            for r in rows:                                           # x_r published, L_rc final
                assert xdone[r] and ver[S(r, c)] >= fin[S(r, c)]
                yc -= M[col(r), col(c)].T @ x[col(r)]
            x[col(c)] = linv[c].T @ yc
            xdone[c] = 1
    assert np.all(ver == fin) and np.all(yver == ycnt) and np.all(xdone == 1) and np.all(lver == 1)
    return x, len(seen)


def _spd_with_blocks(P, pairs, rng):
    """random SPD 6P x 6P matrix with nonzero 6x6 blocks only on the diagonal and `pairs`."""
    A = np.zeros((6 * P, 6 * P))
    for a, b in pairs:
        B = rng.normal(size=(6, 6))
        A[6 * a:6 * a + 6, 6 * b:6 * b + 6] = B
        A[6 * b:6 * b + 6, 6 * a:6 * a + 6] = B.T
    A += np.diag(np.abs(A).sum(1) + 1.0 + rng.uniform(0, 1, 6 * P))
    return A


def _pose_pairs(ii, jj, t0, t1):
    """blocks of the reduced system: edge (i,j) plus every pair of optimised
    rows sharing a depth frame (droid_kernels.cu:1241-1272)."""
    P = t1 - t0
    pairs = set()
    rows = {}
    for i, j in zip(ii.tolist(), jj.tolist()):
        if t0 <= i < t1 and t0 <= j < t1 and i != j:
            pairs.add((max(i, j) - t0, min(i, j) - t0))
        r = rows.setdefault(i, {i - t0} if t0 <= i < t1 else set())
        if t0 <= j < t1:
            r.add(j - t0)
    for r in rows.values():
        r = sorted(r)
        for x in range(len(r)):
            for y in range(x):
                pairs.add((r[x], r[y]))
    return sorted(pairs), P


def _check_solves(st, A, perm, rng):
    n = A.shape[0]
    b = rng.normal(size=n)
    pos = (6 * np.repeat(perm, 6) + np.tile(np.arange(6), len(perm)))   # var v -> permuted index
    Ap = np.zeros_like(A)
    Ap[np.ix_(pos, pos)] = A
    bp = np.zeros(n)
    bp[pos] = b
    # every nonzero of the permuted lower triangle lies in a tile of the plan
    tiles = {(r // 64, c // 64) for r, c in zip(*np.nonzero(np.tril(Ap)))}
    assert all(st["slot"][i, j] >= 0 for i, j in tiles)
    M = np.zeros((n + 1, n))
    M[:n] = np.tril(Ap)
    M[n] = bp
    x, ran = emulate(M, n, st)
    assert ran == len(st["tasks"])
    dx = np.zeros(n)
    dx[st["outmap"]] = x
    np.testing.assert_allclose(dx, np.linalg.solve(A, b), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("n", [6, 63, 64, 65, 128, 130, 300, 1530])
def test_dense_task_list_solves_spd(n):
    rng = np.random.default_rng(n)
    st = chol_plan(n)
    nbc, nbr = (n + 63) // 64, (n + 64) // 64
    # the dense DAG: potrf + trsm below the fused tile + updates but the ones
    # fused into potrf (the diagonal's last) and into trsm (each (i,k+1,k)) +
    # one back-solve task per block column
    ntrsm = sum(max(0, nbr - k - 2) for k in range(nbc))
    expect = nbc + ntrsm + sum((nbr - jb) * jb for jb in range(1, nbc)) - (nbc - 1) \
        - sum(max(0, nbr - k - 2) for k in range(nbc - 1)) + nbc
    assert len(st["tasks"]) == expect
    assert st["nslots"] == st["nslots_input"] == sum(min(i + 1, nbc) for i in range(nbr))
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    A = (Q * np.geomspace(1, 1e3, n)) @ Q.T
    b = rng.normal(size=n)
    M = np.zeros((n + 1, n))
    M[:n] = np.tril(A)
    M[n] = b
    x, ran = emulate(M, n, st)
    assert ran == len(st["tasks"])
    np.testing.assert_allclose(x[st["outmap"]], np.linalg.solve(A, b), rtol=1e-8, atol=1e-10)


def _graph(name):
    from droid_mi355x import synthetic
    if name == "C2":
        ii, jj = synthetic.c2_edges()
        return ii, jj, 16, 8, 16
    if name == "C3":
        ii, jj = synthetic.c3_edges()
        return ii, jj, 256, 1, 256
    if name == "C5":
        ii, jj = synthetic.c5_edges()
        return ii, jj, 2048, 1, 2048
    if name == "laps":   # C5's lapping trajectory at 512 KF: the plan picks nested dissection
        ii, jj = synthetic.c5_edges(num_kf=512, lap=64)
        return ii, jj, 512, 1, 512
    if name == "band":   # +-1..+-3 only: block-tridiagonal in tiles after any sane order
        ii, jj = synthetic.c5_edges(num_kf=600, loop_pairs=0)
        return ii, jj, 600, 1, 600
    raise ValueError(name)


@pytest.mark.parametrize("name", ["C2", "C3", "band"])
def test_ba_plan_task_list_solves_reduced_system(name):
    ii, jj, N, t0, t1 = _graph(name)
    st = ba_plan(ii, jj, N, t0, t1)
    pairs, P = _pose_pairs(ii, jj, t0, t1)
    rng = np.random.default_rng(7)
    _check_solves(st, _spd_with_blocks(P, pairs, rng), st["perm"], rng)


def test_nested_dissection_order_solves():
    """A lapping trajectory's reduced system is a banded cylinder: the plan
    picks the tile-aligned nested dissection (kind 3) for its shorter Cholesky
    critical path, and that task list solves the system."""
    ii, jj, N, t0, t1 = _graph("laps")
    st = ba_plan(ii, jj, N, t0, t1)
    assert st["kind"] == 3
    assert sorted(st["perm"].tolist()) == list(range(t1 - t0))
    pairs, P = _pose_pairs(ii, jj, t0, t1)
    rng = np.random.default_rng(9)
    _check_solves(st, _spd_with_blocks(P, pairs, rng), st["perm"], rng)


def test_nested_dissection_disconnected_graph_solves(ba_order):
    """Forced nested dissection on a pose graph in three pieces (two lapping
    trajectories and a run of poses without edges): every pose is ordered once
    and the task list still solves the reduced system."""
    from droid_mi355x import synthetic
    ba_order("nd")
    a_i, a_j = synthetic.c5_edges(num_kf=160, lap=40)
    b_i, b_j = synthetic.c5_edges(num_kf=120, lap=30)
    ii = np.concatenate([a_i, b_i + 200])
    jj = np.concatenate([a_j, b_j + 200])
    N, t0, t1 = 320, 1, 320   # poses 160..199 and 320.. have no edges
    st = ba_plan(ii, jj, N, t0, t1)
    assert st["kind"] == 3
    assert sorted(st["perm"].tolist()) == list(range(t1 - t0))
    pairs, P = _pose_pairs(ii, jj, t0, t1)
    rng = np.random.default_rng(10)
    _check_solves(st, _spd_with_blocks(P, pairs, rng), st["perm"], rng)


def test_c5_plan_is_tile_sparse():
    """2048 KF / ~16k edges with revisit loops: the chosen
    pose order keeps the factor far from dense, and the plan builds in well
    under a second."""
    ii, jj, N, t0, t1 = _graph("C5")
    assert 15000 <= len(ii) <= 17500
    st = ba_plan(ii, jj, N, t0, t1)
    nbc = st["nbc"]
    dense = sum(min(i + 1, nbc) for i in range(st["nbr"]))
    assert st["kind"] != 0 and st["nslots"] < 0.2 * dense
    assert st["plan_seconds"] < 5.0
    # the all-reduced region (input tiles) of a sharded C5 BA
    assert st["nslots_input"] * 64 * 64 * 8 < 150e6


@pytest.mark.parametrize("order", ["rcm", "mindeg", "nd"])
def test_forced_orders_solve(order, ba_order):
    ba_order(order)
    ii, jj, N, t0, t1 = _graph("C2")
    st = ba_plan(ii, jj, N, t0, t1)
    assert st["kind"] == {"rcm": 1, "mindeg": 2, "nd": 3}[order]
    assert sorted(st["perm"].tolist()) == list(range(t1 - t0))
    pairs, P = _pose_pairs(ii, jj, t0, t1)
    rng = np.random.default_rng(8)
    _check_solves(st, _spd_with_blocks(P, pairs, rng), st["perm"], rng)


def test_high_degree_frames_plan():
    """frames with 40+ outgoing edges (the backend's max_factors = 16 t regime,
    droid_backend.py:31) are planned on the wide Schur path, no error."""
    from droid_mi355x import synthetic
    ii, jj = synthetic.dense_edges(num_kf=48, out_degree=42, rng=np.random.default_rng(3))
    st = ba_plan(ii, jj, 48, 1, 48)
    assert st["nwide"] > 0
    pairs, P = _pose_pairs(ii, jj, 1, 48)
    rng = np.random.default_rng(9)
    _check_solves(st, _spd_with_blocks(P, pairs, rng), st["perm"], rng)

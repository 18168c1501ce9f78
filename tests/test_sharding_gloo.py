"""Multi-rank (world_size 2, gloo on CPU) coverage of the edge-sharded BA
(SURVEY.md §8e).

The GPU path (DepthVideo.ba_sharded) relies on one algebraic fact: with edges
sharded by source frame ii, every depth frame's Schur terms live on one rank,
so the SUM over ranks of the per-rank reduced systems (A_r - S_r, b_r - bS_r)
equals the unsharded reduced system.  These tests check that fact with the
oracle on each rank and a real gloo all_reduce, plus the partition itself.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from droid_mi355x import sharding, synthetic
from oracle import ba as oba

H, W = 6, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    return synthetic.ba_problem("C2", H=H, W=W, sens_fraction=0.3)


def _local_system(prob, rank, world):
    ii, jj = prob["ii"], prob["jj"]
    N = prob["disps"].shape[0]
    ii_l, jj_l, (lo, hi) = sharding.shard_edges(ii, jj, N, rank, world)
    t0, t1 = prob["t0"], prob["t1"]
    kx_full = np.unique(np.concatenate([np.arange(t0, t1), ii]))
    kx_l = np.unique(np.concatenate([np.arange(t0, t1), ii_l]))
    eta_l = prob["eta"][np.searchsorted(kx_full, kx_l)]
    sel = np.isin(np.arange(len(ii)), np.nonzero((ii >= lo) & (ii < hi))[0])
    out = oba.ba(prob["poses"], prob["disps"], prob["intrinsics"], prob["disps_sens"], prob["targets"][sel],
                 prob["weights"][sel], eta_l, ii_l, jj_l, t0, t1, 1, 1e-4, 0.1, False, return_system=True)
    A, b = out["system"]
    return A, b, len(ii_l)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prob = _problem()
        A, b, ne = _local_system(prob, rank, world)
        t = torch.from_numpy(np.concatenate([A.ravel(), b]))
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        n_edges = torch.tensor([ne], dtype=torch.int64)
        dist.all_reduce(n_edges)
        if rank == 0:
            q.put((t.numpy().copy(), int(n_edges.item())))
    finally:
        dist.destroy_process_group()


def test_shard_edges_partition():
    ii, jj = synthetic.c3_edges(rng=np.random.default_rng(1003))
    N = int(max(ii.max(), jj.max())) + 1
    for world in (2, 4, 8):
        blocks = sharding.frame_blocks(ii, N, world)
        assert blocks[0][0] == 0 and blocks[-1][1] == N
        assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
        seen = np.zeros(len(ii), int)
        counts = []
        for r in range(world):
            ii_l, jj_l, (lo, hi) = sharding.shard_edges(ii, jj, N, r, world)
            assert np.all((ii_l >= lo) & (ii_l < hi))
            m = (ii >= lo) & (ii < hi)
            seen[m] += 1
            assert np.array_equal(ii[m], ii_l) and np.array_equal(jj[m], jj_l)
            counts.append(len(ii_l))
        assert np.all(seen == 1)                              # every edge on exactly one rank
        assert max(counts) <= 1.15 * len(ii) / world + 16     # out-degree balanced


@pytest.mark.timeout(300)
def test_allreduced_shard_systems_equal_full_system():
    prob = _problem()
    ref = oba.ba(prob["poses"], prob["disps"], prob["intrinsics"], prob["disps_sens"], prob["targets"],
                 prob["weights"], prob["eta"], prob["ii"], prob["jj"], prob["t0"], prob["t1"], 1, 1e-4, 0.1,
                 False, return_system=True)
    A, b = ref["system"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, n_edges = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = A.shape[0]
    assert n_edges == len(prob["ii"])
    np.testing.assert_allclose(got[:n * n].reshape(n, n), A, rtol=1e-9, atol=1e-9 * np.abs(A).max())
    np.testing.assert_allclose(got[n * n:], b, rtol=1e-9, atol=1e-9 * np.abs(b).max())
    # and the solve of the summed system is the unsharded dx
    dx_sum, ok1 = oba.solve(got[:n * n].reshape(n, n), got[n * n:], 1e-4, 0.1)
    dx_ref, ok2 = oba.solve(A, b, 1e-4, 0.1)
    assert ok1 and ok2
    np.testing.assert_allclose(dx_sum, dx_ref, atol=1e-9)


def _plan_structure(ii, jj, gii, gjj, N, t0, t1, own):
    """pose order + factor tile map of a (sharded) BA plan, via the C ABI (no GPU)."""
    import ctypes
    from droid_backends._lib import check, lib
    ii, jj, gii, gjj = (np.ascontiguousarray(a, np.int64) for a in (ii, jj, gii, gjj))
    kx = np.unique(np.concatenate([np.arange(max(t0, own[0]), min(t1, own[1])), ii]))
    h = ctypes.c_void_p()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    check(lib.droid_ba_plan_create_sharded(vp(ii), vp(jj), len(ii), vp(gii), vp(gjj), len(gii), N, H, W, t0, t1,
                                           len(kx), 0, own[0], own[1], ctypes.byref(h)), "plan")
    try:
        P = t1 - t0
        n = 6 * P
        nbc, nbr = (n + 63) // 64, (n + 64) // 64
        perm = np.zeros(P, np.int32)
        slot = np.zeros(nbr * nbc, np.int32)
        kind, nw, nt = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.droid_ba_plan_order(h, ctypes.byref(kind), vp(perm), ctypes.byref(nw), ctypes.byref(nt)), "order")
        check(lib.droid_chol_plan_structure(h, vp(slot), None, None, None), "structure")
        return perm, slot
    finally:
        lib.droid_ba_plan_destroy(h)


def _gather_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from droid_mi355x.depth_video import global_edges
        ii, jj = synthetic.c5_edges(num_kf=512, lap=128)
        N = 512
        ii_l, jj_l, own = sharding.shard_edges(ii, jj, N, rank, world)
        comm = dict(group=None, own=own, version=0)
        key = (1, N, False, "update")
        gii, gjj = global_edges(ii_l, jj_l, comm, key)
        assert global_edges(ii_l, jj_l, comm, key)[0] is gii     # cached per (version, call)
        perm, slot = _plan_structure(ii_l, jj_l, gii, gjj, N, 1, N, own)
        parts = [None] * world
        dist.all_gather_object(parts, (np.sort(gii * N + gjj), perm, slot))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_plans_share_one_factor_structure():
    """Every rank gathers the same global edge list and derives the same pose
    order and tile map from it, so the per-rank reduced systems add up tile by
    tile in ba_sharded's all-reduce."""
    ii, jj = synthetic.c5_edges(num_kf=512, lap=128)
    ref_perm, ref_slot = _plan_structure(ii, jj, ii, jj, 512, 1, 512, (0, 2 ** 31 - 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for edges, perm, slot in parts:
        np.testing.assert_array_equal(edges, np.sort(ii * 512 + jj))
        np.testing.assert_array_equal(perm, ref_perm)
        np.testing.assert_array_equal(slot, ref_slot)


def _version_worker(rank, world, port, q):
    """an edit that changes ONE rank's shard must make every rank
    re-gather (version bump in lockstep), and a rank that changed its edges
    without a version bump must fail loudly instead of using a stale list."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from droid_mi355x.depth_video import global_edges
        ii, jj = synthetic.c3_edges(num_kf=32, num_edges=160, rng=np.random.default_rng(3))
        ii_l, jj_l, own = sharding.shard_edges(ii, jj, 32, rank, world)
        comm = dict(group=None, own=own, version=0)
        key = (1, 32, False, "update")
        g0 = global_edges(ii_l, jj_l, comm, key)
        # the edit adds an edge only on the last rank's shard; every rank bumps the version
        if rank == world - 1:
            ii_l, jj_l = np.append(ii_l, own[1] - 1), np.append(jj_l, 0)
        comm["version"] += 1
        g1 = global_edges(ii_l, jj_l, comm, key)            # both ranks gather again (no hang)
        grew = len(g1[0]) == len(g0[0]) + 1
        # a shard change without the version bump: that rank raises
        stale_error = None
        if rank == 0:
            try:
                global_edges(np.append(ii_l, own[0]), np.append(jj_l, 31), comm, key)
            except RuntimeError as ex:
                stale_error = str(ex)
        dist.barrier()
        q.put((rank, grew, stale_error))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_global_edges_regather_agreed_across_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_version_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, e)) for r, g, e in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] and res[1][0]
    assert res[0][1] is not None and "not in the global edge list" in res[0][1]


def _status_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from droid_mi355x.depth_video import or_reduce_status
        # [this solve, sticky]: rank 0 non-SPD (bit 0) then a timeout (bit 1);
        # rank 1 corrupt state (bits 1 and 2) - MAX of the packed words would give 6 / 6
        words = {0: [1, 3], 1: [6, 6]}[rank]
        status = torch.tensor(words, dtype=torch.int32)
        or_reduce_status(status)
        q.put((rank, status.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_status_words_or_reduced_per_bit():
    """the sharded BA agrees on the status words per bit (OR), so a
    rank's non-SPD bit survives another rank's higher timeout / corrupt word."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_status_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] == [7, 7]


def test_plan_rejects_local_edges_missing_from_global_list():
    """ADVICE r2 (ba_plan.cpp): a local edge whose blocks have no input tile in
    the factor structure built from the global list is an error, not a write
    through slot -1."""
    ii, jj = synthetic.c5_edges(num_kf=512, lap=128)
    with pytest.raises(RuntimeError, match="not covered by the global edge list"):
        # local edge (300, 40) pairs poses far apart; the global list is only the temporal chain
        m = np.abs(ii - jj) <= 1
        _plan_structure(np.array([300]), np.array([40]), ii[m], jj[m], 512, 1, 512, (256, 512))

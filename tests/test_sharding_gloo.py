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


def test_reduced_system_index_covers_lower_triangle_and_rhs():
    """ba_sharded all-reduces only what the Cholesky reads: the packed index
    holds every (row, col <= row) of A - S and the rhs row, nothing else."""
    from types import SimpleNamespace
    from droid_mi355x.depth_video import reduced_system_index
    n, ld = 12, 16
    plan = SimpleNamespace(n=n, ld=ld, system=torch.zeros((n + 1, ld), dtype=torch.float64))
    idx = reduced_system_index(plan).numpy()
    assert len(idx) == n * (n + 1) // 2 + n == len(np.unique(idx))
    r, c = idx // ld, idx % ld
    assert ((r < n) & (c <= r) | (r == n) & (c < n)).all()
    # a packed sum over two "ranks" equals the full sum on those positions
    a, b = torch.randn(n + 1, ld, dtype=torch.float64), torch.randn(n + 1, ld, dtype=torch.float64)
    out = a.clone().view(-1)
    out.index_copy_(0, torch.as_tensor(idx), a.view(-1)[idx] + b.view(-1)[idx])
    full = (a + b).view(-1)
    assert torch.equal(out[idx], full[idx])
    assert reduced_system_index(plan) is plan._tri_index   # cached on the plan

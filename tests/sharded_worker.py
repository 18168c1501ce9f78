"""Worker for tests/test_gpu_sharded.py (not a test module): runs FactorGraph.update()
on a small deterministic graph, either unsharded (WORLD_SIZE unset / 1) or as one
rank of the edge-sharded path (edges split by source frame, one
all-reduce of the reduced camera system per Gauss-Newton iteration)
with every rank on cuda:0 and gloo collectives - the layout bench.py uses on
one GPU (DROID_BENCH_ONE_DEVICE=1).  Writes <out>.rank<R>.npz: poses, disps and
the [lo, hi) frames whose depths this rank owns.

usage: python tests/sharded_worker.py <out prefix>  (under torch.distributed.run for N ranks)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "droid-slam_amd"), os.path.join(HERE, "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    out = sys.argv[1]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")

    from fill import det_fill
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, sharding, synthetic
    from droid_mi355x.fused import FusedUpdateModule

    n, H, W = 16, 16, 32
    rng = np.random.default_rng(41)
    ii, jj = synthetic.c3_edges(n, 72, rng=np.random.default_rng(42), max_out=8)
    comm = None
    own = (0, n)
    if world > 1:
        ii_l, jj_l, own = sharding.shard_edges(ii, jj, n, rank, world)
        comm = dict(group=None, own=own, t0=max(1, int(ii.min()) + 1), t1=int(max(ii.max(), jj.max())) + 1)
    else:
        ii_l, jj_l = ii, jj
    gt = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, device=dev)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).to(dev)
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).to(dev)
    video.intrinsics[:n] = torch.tensor([[H / 1.5, H / 1.5, W / 2, H / 2]] * n, device=dev)
    video.fmaps[:n] = torch.from_numpy(rng.normal(size=(n, 1, 128, H, W)).astype(np.float16)).to(dev)
    video.nets[:n] = torch.from_numpy(np.tanh(rng.normal(size=(n, 128, H, W))).astype(np.float16)).to(dev)
    video.inps[:n] = torch.from_numpy(np.maximum(rng.normal(size=(n, 128, H, W)), 0).astype(np.float16)).to(dev)
    video.counter.value = n
    m = UpdateModule().to(dev).eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device=dev)
    g.comm = comm
    disps0 = video.disps[:n].cpu().numpy()
    with torch.no_grad():
        g.add_factors(ii_l, jj_l)
        for _ in range(2):
            g.update()
    torch.cuda.synchronize()
    np.savez("%s.rank%d.npz" % (out, rank), poses=video.poses[:n].cpu().numpy(),
             disps=video.disps[:n].cpu().numpy(), disps0=disps0, own=np.asarray(own), edges=len(ii_l))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

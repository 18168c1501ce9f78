"""Worker for tests/test_gpu_ba_scale.py (not a test module): one rank of the
edge-sharded BA (DepthVideo.ba_sharded: local linearisation and Schur terms,
gloo all-reduce of the reduced system's input tiles, identical Cholesky on
every rank) on a C5-shaped problem (2048 KF / ~16k edges), every
rank on cuda:0.  Writes <out>.rank<R>.npz: poses, disps, dx and the [lo, hi)
frames whose depths this rank owns.

With a 4th argument "inject", rank 0 alone makes its dataflow solves abort
(droid_chol_set_fault_inject, so the worker binds the A/B library, which
exports it): first in every GN iteration of one call, then
in the first iteration of a second call.  The status words are all-reduced
before each step is applied, so every rank must skip the same steps and raise;
the npz then also holds each call's poses / disps and whether it raised.

usage: python -m torch.distributed.run --nproc-per-node 2 tests/sharded_ba_worker.py <out prefix> <H> <W> [inject]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "droid-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    out, H, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    inject = len(sys.argv) > 4 and sys.argv[4] == "inject"
    if inject:   # the fault-injection hook ships in the testing builds only (include/droid_backends_testing.h)
        os.environ["DROID_HIP_LIB"] = os.path.join(ROOT, "droid-slam_amd", "lib", "ab", "libdroid_hip.so")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from droid_mi355x import sharding, synthetic
    from droid_mi355x.depth_video import ba_sharded

    prob = synthetic.ba_problem("C5", H=H, W=W)
    ii, jj, t0, t1 = prob["ii"], prob["jj"], prob["t0"], prob["t1"]
    N = prob["disps"].shape[0]
    ii_l, jj_l, own = sharding.shard_edges(ii, jj, N, rank, world)
    sel = (ii >= own[0]) & (ii < own[1])
    kx = np.unique(np.concatenate([np.arange(t0, t1), ii]))
    kx_l = np.unique(np.concatenate([np.arange(max(t0, own[0]), min(t1, own[1])), ii_l]))
    eta_l = prob["eta"][np.searchsorted(kx, kx_l)]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    poses, disps = d(prob["poses"]), d(prob["disps"])
    comm = dict(group=None, own=own)
    if inject:
        import droid_backends
        rec = {}
        for call, mode in (("all", droid_backends.CHOL_INJECT_ALL), ("once", droid_backends.CHOL_INJECT_ONCE)):
            droid_backends.chol_set_fault_inject(mode if rank == 0 else droid_backends.CHOL_INJECT_OFF)
            ba_sharded(poses, disps, d(prob["intrinsics"]), d(prob["disps_sens"]), d(prob["targets"][sel]),
                       d(prob["weights"][sel]), d(eta_l), ii_l, jj_l, t0, t1, 2, 1e-5, 1e-2, False, comm)
            droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_OFF)
            try:
                comm["_last_plan"].check_status()
                raised = False
            except RuntimeError as e:
                raised = "timed out" in str(e)
            rec[call + "_poses"] = poses.cpu().numpy()
            rec[call + "_disps"] = disps.cpu().numpy()
            rec[call + "_raised"] = np.asarray(raised)
        np.savez("%s.rank%d.npz" % (out, rank), own=np.asarray(own), **rec)
        dist.barrier()
        dist.destroy_process_group()
        return
    dx, dz = ba_sharded(poses, disps, d(prob["intrinsics"]), d(prob["disps_sens"]), d(prob["targets"][sel]),
                        d(prob["weights"][sel]), d(eta_l), ii_l, jj_l, t0, t1, 2, 1e-5, 1e-2, False, comm)
    torch.cuda.synchronize()
    np.savez("%s.rank%d.npz" % (out, rank), poses=poses.cpu().numpy(), disps=disps.cpu().numpy(),
             dx=dx.cpu().numpy(), own=np.asarray(own), edges=len(ii_l))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

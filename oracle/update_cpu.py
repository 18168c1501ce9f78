"""CPU baseline of FactorGraph.update() (factor_graph.py:196-242), built from
the oracle restatements - the "reference's pure-PyTorch CPU path" BASELINE.md
asks for does not exist in the reference (droid_backends is CUDA-only,
geom/ba.py needs lietorch), so this restatement stands in for it.

TEST INFRASTRUCTURE ONLY (oracle/__init__.py): used by bench.py's
cpu_baseline leg, never by the product.

Full runs, no extrapolation (BASELINE.md "CPU baseline"):
  C1  CorrBlock on 2 frames / 1 edge at 48x64, r=3: volume + pyramid + 4-level
      lookup (median of `repeats`);
  C2 / C3  one complete update(): reprojection + motion features, the 4-level
      lookup of every edge, UpdateModule (fp32 torch convs) with GraphAgg, and
      ba_cuda's semantics (fp64) for `itrs` Gauss-Newton iterations - over ALL
      edges.  The correlation volumes belong to add_factors in the reference
      (factor_graph.py:112-116), not to update(); they are built here chunk by
      chunk of source frames (memory) and their time is reported separately,
      outside the update rate.
The correlation runs as torch fp32 on the CPU (matmul + avg_pool2d volume,
grid_sample lookup: oracle/corr.py *_torch, equal to the loop restatement of
correlation_kernels.cu, tests/test_oracle_golden.py), as a pure-PyTorch port
of CorrBlock would.
"""
import os
import time

import numpy as np
import torch

from . import ba as oba
from . import corr as oc
from . import geometry as og
from . import update_module as oum


def cpu_info():
    """lscpu-equivalent facts from /proc/cpuinfo: model, sockets, physical cores, logical CPUs."""
    model, sockets, cores = None, set(), set()
    logical = 0
    try:
        phys = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    logical += 1
                elif k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    phys = v
                    sockets.add(v)
                elif k == "core id":
                    cores.add((phys, v))
    except OSError:
        pass
    return dict(model=model, sockets=len(sockets) or None, physical_cores=len(cores) or None,
                logical_cpus=logical or os.cpu_count(), os_cpu_count=os.cpu_count(),
                affinity_cpus=len(os.sched_getaffinity(0)), cgroup_cpu_quota=cgroup_cpu_quota())


def cgroup_cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None
    when unlimited / unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def baseline_threads():
    """Threads for the CPU baseline: torch.set_num_threads(os.cpu_count()) as
    BASELINE.md asks (not OMP_NUM_THREADS), bounded by the CPUs this process
    may actually run on - its affinity mask and, when set, its cgroup CPU
    quota (a shared GPU box shows the whole host in os.cpu_count())."""
    n = os.cpu_count() or 1
    n = min(n, len(os.sched_getaffinity(0)))
    q = cgroup_cpu_quota()
    if q is not None:
        n = min(n, max(1, int(q)))
    return max(1, n)


def time_c1(threads, H=48, W=64, repeats=3, seed=1001):
    """C1: 2-frame / 1-edge CorrBlock (corr.py:24-50), fp32 on the CPU."""
    torch.set_num_threads(threads)
    rng = np.random.default_rng(seed)
    f1 = rng.normal(size=(1, 1, 128, H, W)).astype(np.float32)
    f2 = rng.normal(size=(1, 1, 128, H, W)).astype(np.float32)
    coords = (og.coords_grid(H, W, np.float32)[None, None] + rng.normal(0, 2, (1, 1, H, W, 2))).astype(np.float32)
    f1, f2, c = torch.from_numpy(f1), torch.from_numpy(f2), torch.from_numpy(coords[0])
    ts = []
    for _ in range(repeats):
        t = time.perf_counter()
        pyr = oc.corr_pyramid_torch(f1, f2)
        oc.lookup_pyramid_torch(pyr, c, 3)
        ts.append(time.perf_counter() - t)
    return dict(ms=1000 * float(np.median(ts)), repeats=repeats)


def time_update(prob, fmaps, nets, inps, params, threads, itrs=2, chunk_frames=4, lm=1e-4, ep=0.1):
    """One complete update() of the graph in `prob` (synthetic.ba_problem)
    with per-edge features gathered from per-frame fmaps / nets / inps (N,...),
    as add_factors does (factor_graph.py:108-118).  Returns ms per stage."""
    torch.set_num_threads(threads)
    p = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in params.items()}
    ii, jj = prob["ii"], prob["jj"]
    N, H, W = prob["disps"].shape
    intr = np.tile(prob["intrinsics"][None], (N, 1))
    st = {"reproject": 0.0, "corr volumes (add_factors, excluded)": 0.0, "lookup": 0.0, "update_op": 0.0, "ba": 0.0}

    t = time.perf_counter()
    coords1, _ = og.projective_transform(prob["poses"], prob["disps"], intr, ii, jj, dtype=np.float32)
    target0 = prob["targets"].transpose(0, 2, 3, 1)
    motn = np.concatenate([coords1 - og.coords_grid(H, W, np.float32), target0 - coords1], -1)
    motn = motn.transpose(0, 3, 1, 2).clip(-64, 64).astype(np.float32)
    st["reproject"] += time.perf_counter() - t

    delta = np.zeros((len(ii), H, W, 2), np.float32)
    weight = np.zeros((len(ii), H, W, 2), np.float32)
    frames = np.unique(ii)
    for c in range(0, len(frames), chunk_frames):        # GraphAgg is per source frame: chunking is exact
        sel = np.nonzero(np.isin(ii, frames[c:c + chunk_frames]))[0]
        si, sj = ii[sel], jj[sel]
        t = time.perf_counter()
        pyr = oc.corr_pyramid_torch(torch.from_numpy(fmaps[si][None].astype(np.float32)),
                                    torch.from_numpy(fmaps[sj][None].astype(np.float32)))
        st["corr volumes (add_factors, excluded)"] += time.perf_counter() - t
        t = time.perf_counter()
        corr = oc.lookup_pyramid_torch(pyr, torch.from_numpy(coords1[sel]), 3)[None]
        st["lookup"] += time.perf_counter() - t
        del pyr
        t = time.perf_counter()
        with torch.no_grad():
            _, d, w, _, _ = oum.update_module(p, torch.from_numpy(nets[si][None].astype(np.float32)),
                                              torch.from_numpy(inps[si][None].astype(np.float32)),
                                              corr, torch.from_numpy(motn[sel][None]),
                                              torch.from_numpy(si), torch.from_numpy(sj))
        delta[sel], weight[sel] = d[0].numpy(), w[0].numpy()
        st["update_op"] += time.perf_counter() - t

    t = time.perf_counter()
    target = (coords1 + delta).transpose(0, 3, 1, 2)
    oba.ba(prob["poses"], prob["disps"], prob["intrinsics"], prob["disps_sens"], target,
           weight.transpose(0, 3, 1, 2), prob["eta"], ii, jj, prob["t0"], prob["t1"], itrs, lm, ep, False)
    st["ba"] += time.perf_counter() - t
    total = sum(v for k, v in st.items() if "excluded" not in k)
    return dict(seconds_per_update=total, ms={k: 1000 * v for k, v in st.items()}, edges=len(ii),
                threads=torch.get_num_threads())

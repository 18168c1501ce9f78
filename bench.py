#!/usr/bin/env python
"""Benchmark: FactorGraph.update() iterations/s on the C3 global-BA graph
(256 keyframes, 2048 edges, 384x512 images -> 48x64 at 1/8 resolution).

One step = one full update(): fused reprojection + motion features, 4-level
correlation lookup, update operator (ConvGRU etc., fp16), GraphAgg, and the
dense BA with itrs=2 Gauss-Newton iterations - all on the GPU, inputs resident
in HBM.  N>1 GPUs (torch.distributed.run, RCCL): the SAME graph is split by
source frame (strong scaling); each rank runs its edges and its depth frames,
and the reduced camera system is all-reduced once per GN iteration.

Prints ONE JSON line (rank 0) with the roofline of the dominant hand-written
kernel (the ConvGRU z|r gate conv, MFMA-bound) measured live with
HIP events on its launch stream, a secondary HBM roofline for the correlation
lookup, and the CPU baseline (oracle restatement, bounded sample) on rank 0 at
N=1.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "droid-slam_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PEAK_F16_TFLOPS = 2500.0        # MI355X_MICROARCH.md: dense fp16/bf16 MFMA peak (no sparsity)
LOOKUP_BYTES_PER_EDGE = 2801664  # volume-API lookup, 4 lvl x 64 taps x 2 B x HW + coords + out
# fused lookup + corr_encoder[0] (corr_ce0_kernel): the same window reads + coords, 128-ch fp16 output
LOOKUP_CE0_BYTES_PER_EDGE = 4 * 64 * 2 * 3072 + 2 * 4 * 3072 + 128 * 2 * 3072
# on-demand lookup (corr_alt_ce0): SURVEY.md §8d fused feature-pyramid row (fmap1 + fmap2 pyramid + coords)
# with the 128-channel corr_encoder[0] output instead of the 196-channel lookup
ALT_BYTES_PER_EDGE = 786432 + 1044480 + 24576 + 128 * 2 * 3072
# ConvGRU z|r conv (modules/gru.py:19-32, convz+convr fused): 3x3, 448 -> 256 channels
ZR_FLOPS_PER_PIXEL = 2 * 256 * 448 * 9
# ... with the context features factored out per source frame (droid_conv_gru_pre_f16):
# the per-edge z|r conv runs over net | corr | flow = 320 channels
ZR_PRE_FLOPS_PER_PIXEL = 2 * 256 * 320 * 9
ZR_KERNEL = "conv_band_kernel<256,256>"   # csrc/conv_kernels.hip, chosen for 48x64 maps
ZR_KERNEL_MATCH = "conv_band_kernel<256, 256, false, false, 1"   # its symbol in rocprof / PMC summaries
ZRP_KERNEL_MATCH = "conv_band_kernel<256, 256, false, false, 6"  # ... the factored-gate instantiation
LOOKUP_KERNEL = "corr_pyramid_f16_r3_kernel"
# SURVEY.md §8d whole-iteration floors.  Update-operator convs per edge-pixel:
# corr_encoder 1x1 196->128 + 3x3 128->128, flow_encoder 7x7 4->128 + 3x3 128->64,
# ConvGRU convz|convr|convq 3x3 448->128 + w 1x1 128->128, delta/weight 3x3
# 128->128 + 3x3 128->2 each, GraphAgg conv1 3x3 128->128 (droid_net.py:59-143,
# gru.py:19-32); per unique source frame-pixel: GraphAgg conv2 3x3 128->128,
# eta 3x3 128->1.
CONV_FLOPS_PER_EDGE_PIXEL = 2 * (196 * 128 + 128 * 128 * 9 + 4 * 128 * 49 + 128 * 64 * 9 + 3 * 448 * 128 * 9
                                 + 128 * 128 + 2 * (128 * 128 * 9 + 128 * 2 * 9) + 128 * 128 * 9)
# (GraphAgg's upmask, 1x1 128->576, is not counted: the reference's update()
# discards it, factor_graph.py:209, and the fused operator never computes it)
CONV_FLOPS_PER_FRAME_PIXEL = 2 * (128 * 128 * 9 + 128 * 9)
# factored gates: 3 x 128 inp channels move from per-edge to per-source-frame pixels
GATE_INP_FLOPS_PER_PIXEL = 2 * 3 * 128 * 128 * 9
# HBM-bound stages per update (fused lookup path): lookup 3,059,712 B/edge (§8d fused row),
# BA 2 GN x (49,152 B/edge + 49,152 B/frame), reproject + motn 110,592 B/edge
HBM_BYTES_PER_EDGE = 3059712 + 2 * 49152 + 110592
HBM_BYTES_PER_FRAME = 2 * 49152


LOOKUP_FN = ["corr_lookup_ce0"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_state(args, rank, world, device):
    import droid_backends  # noqa: F401
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, sharding, synthetic

    H, W = args.ht // 8, args.wd // 8
    rng = np.random.default_rng(1003)
    stereo = args.config == "C4"
    if stereo:   # C4: 128 KF, one stereo (i, i) edge per frame + temporal + loops
        ii, jj = synthetic.c4_edges(args.frames, rng=np.random.default_rng(1004))
    elif args.config == "C2":   # frontend window: 16-KF buffer, 96 edges
        ii, jj = synthetic.c2_edges()
    elif args.config == "C5":   # 2048 KF, 8 laps of a circuit, temporal + revisit loops (~16k edges)
        ii, jj = synthetic.c5_edges(args.frames, rng=np.random.default_rng(1005))
    else:
        ii, jj = synthetic.c3_edges(args.frames, args.edges, rng=np.random.default_rng(1003))
    comm = None
    if world > 1 or args.force_dist:
        ii_l, jj_l, own = sharding.shard_edges(ii, jj, args.frames, rank, world)
        # the BA gathers the global edge list once per edge-set version (every rank
        # derives the same reduced-system tile structure from it)
        comm = dict(group=None, own=own, t0=max(1, int(ii.min()) + 1), t1=int(max(ii.max(), jj.max())) + 1,
                    version=0)
    else:
        ii_l, jj_l = ii, jj
    n = args.frames
    gt = synthetic.trajectory_laps(n, 256, rng) if args.config == "C5" else synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
    video = DepthVideo(image_size=(args.ht, args.wd), buffer=n, stereo=stereo, device=device)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).to(device)
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).to(device)
    video.intrinsics[:n] = torch.from_numpy(np.tile(synthetic.INTRINSICS, (n, 1))).to(device)
    g = torch.Generator(device=device).manual_seed(1003)
    video.fmaps[:n] = torch.randn((n, 2 if stereo else 1, 128, H, W), generator=g, device=device).half()
    video.nets[:n] = torch.tanh(torch.randn((n, 128, H, W), generator=g, device=device)).half()
    video.inps[:n] = torch.relu(torch.randn((n, 128, H, W), generator=g, device=device)).half()
    video.counter.value = n
    torch.manual_seed(1003)
    net = UpdateModule().to(device).eval()
    if args.reference_layout:
        from droid_mi355x.fused import ReferenceLayoutUpdateModule
        net = ReferenceLayoutUpdateModule(net)
    elif not args.reference_op:
        from droid_mi355x.fused import FusedUpdateModule
        net = FusedUpdateModule(net)
    corr_impl = "alt" if args.lowmem else args.corr if not args.reference_op else "volume"
    graph = FactorGraph(video, net, device=device, corr_impl=corr_impl)
    graph.comm = comm
    if args.reference_api:
        graph.tiled_volume = False   # the reference's own row-major volume layout
    with torch.no_grad():
        graph.add_factors(ii_l, jj_l)
        if args.reference_api:
            graph.corr = ReferenceApiCorr(graph.corr)
        if args.config == "C2":
            # the frontend's state: edges older than the window stored inactive
            # (droid_frontend.py:42,106) - update(use_inactive=True) then optimises
            # [8, 16) with the stored edges into [5, 8) joining the BA
            graph.update(use_inactive=False)
            graph.rm_factors(graph.ii < 7, store=True)
    torch.cuda.synchronize(device)
    return video, graph, (ii, jj), len(graph._ii)


class ReferenceApiCorr:
    """The reference's CorrBlock.__call__ verbatim in structure
    (/root/reference/droid_slam/modules/corr.py:40-50, restated): coords
    permuted to (B*N, 2, H, W), then per level one
    droid_backends.corr_index_forward on the reference-layout volume
    (E, H, W, H2/2^i, W2/2^i) at coords / 2^i, and a torch.cat of the four
    49-channel results - what a maintainer gets by swapping only the
    droid_backends extension under the reference's own modules/corr.py.
    HIP events bracket each whole call (4 launches + the cat) on torch's
    current stream, the stream the C ABI launches on."""

    def __init__(self, block):
        self.block = block
        self.corr_pyramid = block.reference_pyramid()   # row-major (untiled) levels
        self.num_levels, self.radius = block.num_levels, block.radius
        self.events, self.active = [], False

    def __call__(self, coords):
        import droid_backends
        if self.active:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
        out_pyramid = []
        batch, num, ht, wd, _ = coords.shape
        coords = coords.permute(0, 1, 4, 2, 3)
        coords = coords.contiguous().view(batch * num, 2, ht, wd)
        for i in range(self.num_levels):
            corr, = droid_backends.corr_index_forward(self.corr_pyramid[i], coords / 2 ** i, self.radius)
            out_pyramid.append(corr.view(batch, num, -1, ht, wd))
        out = torch.cat(out_pyramid, dim=2)
        if self.active:
            e.record()
            self.events.append((s, e))
        return out

    def mean_ms(self):
        torch.cuda.synchronize()
        return float(np.mean([s.elapsed_time(e) for s, e in self.events])) if self.events else None


class KernelTimer:
    """HIP events around every call of a droid_backends entry point, on the
    stream it launches on (torch's current stream)."""

    def __init__(self, module, name, when=None):
        self.module, self.name = module, name
        self.orig = getattr(module, name)
        self.events = []
        self.active = False

        def wrapped(*a, **k):
            if not self.active or (when is not None and not when(*a, **k)):
                return self.orig(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = self.orig(*a, **k)
            e.record()
            self.events.append((s, e))
            return out

        setattr(module, name, wrapped)

    def mean_ms(self):
        torch.cuda.synchronize()
        if not self.events:
            return None
        return float(np.mean([s.elapsed_time(e) for s, e in self.events]))


def stage_breakdown(graph, video, steps=3):
    """ms per stage of update() (separate, untimed pass)."""
    import droid_backends
    names = {"reproject+motn": (droid_backends, "projective_transform"),
             "corr lookup": (droid_backends, LOOKUP_FN[0])}
    timers = {k: KernelTimer(m, n) for k, (m, n) in names.items()}
    # update operator and BA: wrap bound callables
    op_t, ba_t = [], []
    orig_op, orig_ba = graph.update_op, video.ba

    def op(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_op(*a, **k)
        e.record()
        op_t.append((s, e))
        return out

    def ba(*a, **k):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_ba(*a, **k)
        e.record()
        ba_t.append((s, e))
        return out

    graph.update_op, video.ba = op, ba
    for t in timers.values():
        t.active = True
    with torch.no_grad():
        for _ in range(steps):
            graph.update()
    torch.cuda.synchronize()
    graph.update_op, video.ba = orig_op, orig_ba
    out = {k: t.mean_ms() for k, t in timers.items()}
    for t in timers.values():
        setattr(t.module, t.name, t.orig)
    out["update_op (convs)"] = float(np.mean([s.elapsed_time(e) for s, e in op_t]))
    out["ba (2 GN iters)"] = float(np.mean([s.elapsed_time(e) for s, e in ba_t]))
    return out


def frontend_edge_change(graph, video, changes=5):
    """The frontend changes its edge set once per keyframe (droid_frontend.py:
    __update: rm_factors + add_proximity_factors, then 4-6 update() calls on the
    new set).  Host cost of the BA plan rebuild (kx, Schur rows, assembly lists,
    pose order, tile tasks) and the wall time of the first update() after an
    edge change (new plan + edge-list uploads + the new edges' corr volumes)."""
    import droid_backends
    ii_h, jj_h = graph._ii.copy(), graph._jj.copy()
    N, H, W = video.disps.shape
    t0 = max(1, int(ii_h.min()) + 1)
    m = (graph._ii_inac >= t0 - 3) & (graph._jj_inac >= t0 - 3)
    ii_ba, jj_ba = np.concatenate([graph._ii_inac[m], ii_h]), np.concatenate([graph._jj_inac[m], jj_h])
    t1 = int(max(ii_ba.max(), jj_ba.max())) + 1
    plan_ms, step_ms = [], []
    with torch.no_grad():
        for c in range(changes):
            h0 = time.perf_counter()
            droid_backends.BaPlan(ii_ba, jj_ba, N, H, W, t0, t1, len(np.unique(ii_ba)), False, video.disps.device)
            plan_ms.append(1000 * (time.perf_counter() - h0))
            # drop one edge pair and add it back: a new edge set each time (plan cache cleared)
            torch.cuda.synchronize()
            h0 = time.perf_counter()
            sel = (graph._ii == 15) & (graph._jj == 12) | (graph._ii == 12) & (graph._jj == 15)
            graph.rm_factors(sel, store=False)
            graph.add_factors(np.array([15, 12]), np.array([12, 15]))
            droid_backends._PLAN_CACHE.clear()
            graph.update(use_inactive=True)
            torch.cuda.synchronize()
            step_ms.append(1000 * (time.perf_counter() - h0))
    return {"plan_build_ms_host": float(np.median(plan_ms)), "edge_change_plus_update_ms": float(np.median(step_ms)),
            "ba_edges": int(len(ii_ba)), "note": "median of %d edge-set changes (rm + add one edge pair, "
                                                 "its corr volume, plan rebuild, one update)" % changes}


def cpu_baseline(graph, video, args):
    """BASELINE.md's CPU baseline, full runs (no extrapolation): C1 (2-frame
    CorrBlock, median of 3), C2 (one full update() of the frontend graph,
    median of 3) and C3 (ONE full update() of this run's 256-KF / 2048-edge
    graph, with this run's features and weights) through the oracle
    restatement (oracle/update_cpu.py) on the host cores, ms per stage."""
    from droid_mi355x import synthetic
    from oracle import update_cpu
    threads = update_cpu.baseline_threads()
    params = {k: v.detach().float().cpu().numpy() for k, v in graph.update_op.state_dict().items()}
    H, W = args.ht // 8, args.wd // 8
    t_all = time.time()
    c1 = update_cpu.time_c1(threads, H, W)
    rng = np.random.default_rng(1002)
    p2 = synthetic.ba_problem("C2", H=H, W=W)
    n2 = p2["disps"].shape[0]
    f2 = (rng.normal(size=(n2, 128, H, W)).astype(np.float16), np.tanh(rng.normal(size=(n2, 128, H, W))).astype(np.float16),
          np.maximum(rng.normal(size=(n2, 128, H, W)), 0).astype(np.float16))
    c2 = [update_cpu.time_update(p2, *f2, params, threads) for _ in range(3)]
    c2 = sorted(c2, key=lambda r: r["seconds_per_update"])[1]
    p3 = synthetic.ba_problem("C3", H=H, W=W)
    n = args.frames
    f3 = (video.fmaps[:n, 0].cpu().numpy(), video.nets[:n].cpu().numpy(), video.inps[:n].cpu().numpy())
    c3 = update_cpu.time_update(p3, *f3, params, threads)
    info = update_cpu.cpu_info()
    r = lambda d: {k: round(v, 1) for k, v in d.items()}
    return {"value": 1.0 / c3["seconds_per_update"], "unit": "iters/s", "cores": c3["threads"], "kind": "port",
            "sample": ("full runs, no extrapolation: ONE complete C3 update() (2048 edges, 256 KF, 48x64: "
                       "reprojection, 4-level lookup, UpdateModule fp32, BA itrs=2 fp64) through the oracle "
                       "restatement on %d host threads; corr volumes built per chunk and timed apart (they belong "
                       "to add_factors)" % c3["threads"]),
            "cpu": info, "threads": c3["threads"], "physical_cores": info.get("physical_cores"),
            "sockets": info.get("sockets"), "cpu_model": info.get("model"),
            "C1": {"ms": round(c1["ms"], 2), "median_of": c1["repeats"],
                   "what": "2 frames / 1 edge CorrBlock 48x64 r=3 (volume + pyramid + lookup)"},
            "C2": {"iters_per_s": 1.0 / c2["seconds_per_update"], "ms_per_stage": r(c2["ms"]), "median_of": 3,
                   "edges": c2["edges"]},
            "C3": {"iters_per_s": 1.0 / c3["seconds_per_update"], "ms_per_stage": r(c3["ms"]), "runs": 1,
                   "edges": c3["edges"]},
            "wall_s": round(time.time() - t_all, 1)}


def lib_sha16():
    """sha256 (16 hex digits) of the libdroid_hip.so this process loaded."""
    import hashlib
    from droid_backends import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(name, e_local, kernel):
    """HBM bytes per launch from a committed PMC pass (profiles/pmc_<name>.json,
    FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) of this
    launch's edge count and of the kernel named, measured on the very library
    this process loaded (the record's lib_sha16); None when no such measurement
    exists (a pass on an older build says nothing about the current kernel)."""
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % name)
    if os.path.exists(p):
        try:
            with open(p) as f:
                d = json.load(f)
            if (d.get("edges") == e_local and kernel in (d.get("kernel") or "")
                    and d.get("lib_sha16") == lib_sha16()):
                return d.get("traffic_bytes_per_launch")
        except Exception:
            return None
    return None


def launcher_command(n, port, argv):
    """The child command `bench.py --gpus N` runs when started without
    torch.distributed.run: N local ranks over 127.0.0.1, same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, one_dev):
    """Run N ranks as a child process (never an exec: nothing here has touched
    the GPU, and the child is a separate program), relay their output, return
    the child's exit code."""
    import socket
    import subprocess
    if not one_dev:
        have = torch.cuda.device_count()   # does not initialise the GPU on this image
        if have < n:
            log("error: --gpus %d but only %d visible GPU(s)" % (n, have))
            return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    cmd = launcher_command(n, port, sys.argv[1:])
    log("launching %d ranks: %s" % (n, " ".join(cmd)))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=["C2", "C3", "C4", "C5"], default="C3",
                    help="C3 (default, the metric's config): 256 KF / 2048 edges mono; "
                         "C4: stereo, 128 KF, (i, i) stereo edges + temporal + loops (~1k edges); "
                         "C2: frontend window, 16-KF buffer, 96 edges, update(use_inactive=True); "
                         "C5: 2048 KF / ~16k edges (the edge-sharded global BA), on-demand (pyramid) "
                         "correlation - its volumes would need ~300 GB")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--edges", type=int, default=2048)
    ap.add_argument("--ht", type=int, default=384)
    ap.add_argument("--wd", type=int, default=512)
    ap.add_argument("--corr", choices=["pyramid", "volume"], default="volume",
                    help="correlation: 'volume' = CorrBlock's all-pairs volume (built in add_factors), "
                         "'pyramid' = windows computed on demand on MFMA from the feature pyramid")
    ap.add_argument("--lowmem", action="store_true",
                    help="time update_lowmem(steps=1) (the global-BA backend's step, factor_graph.py:245-290: "
                         "on-demand correlation, BA over [1, t) with lm=1e-5, ep=1e-2) instead of update()")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--breakdown", action="store_true")
    ap.add_argument("--reference-op", action="store_true",
                    help="run the reference-structured UpdateModule (torch/MIOpen convs, NCHW) instead of the fused MFMA operator")
    ap.add_argument("--reference-layout", action="store_true",
                    help="the reference's update() structure (NCHW state, materialised lookup) with the MI355X "
                         "UpdateModule drop-in (ReferenceLayoutUpdateModule): what the reference's own "
                         "factor_graph.py gets from swapping the module only")
    ap.add_argument("--reference-api", action="store_true",
                    help="the literal drop-in: --reference-layout with the reference's own CorrBlock.__call__ "
                         "(modules/corr.py:40-50: 4 x droid_backends.corr_index_forward on the row-major volume "
                         "+ torch.cat) instead of the one-launch tiled lookup")
    args = ap.parse_args()
    if args.reference_api:
        args.reference_layout = True
    if args.reference_layout:
        args.reference_op = True
    if args.config == "C4" and args.frames == 256:
        args.frames = 128
    if args.config == "C2":
        args.frames = 16
    if args.config == "C5":
        if args.frames == 256:
            args.frames = 2048
        args.corr = "pyramid"

    # DROID_BENCH_ONE_DEVICE=1 / DROID_BENCH_BACKEND=gloo: rehearse the N-rank path
    # with every rank on cuda:0 (a one-GPU box); the driver's runs use RCCL, one GPU per rank
    one_dev = os.environ.get("DROID_BENCH_ONE_DEVICE") == "1"
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` on its own: start the N ranks (one process per GPU,
        # as train.py:184-186 spawns its DDP workers) before anything touches the GPU
        sys.exit(launch_ranks(args.gpus, one_dev))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("error: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
        sys.exit(2)
    device = torch.device("cuda", 0 if one_dev else local_rank)
    torch.cuda.set_device(device)
    import torch.distributed as dist
    # DROID_BENCH_FORCE_DIST=1: the sharded path (process group, all-reduce of the
    # reduced system) even with one rank - exercises RCCL on a one-GPU box
    args.force_dist = os.environ.get("DROID_BENCH_FORCE_DIST") == "1"
    dist_on = world > 1 or args.force_dist
    if dist_on:
        if world == 1 and "RANK" not in os.environ:
            # a forced one-rank group started without a launcher: a local rendezvous
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        backend = os.environ.get("DROID_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    t_setup = time.time()
    video, graph, (ii, jj), e_local = build_state(args, rank, world, device)
    if rank == 0:
        log("setup %.1fs (local edges %d)" % (time.time() - t_setup, e_local))

    import droid_backends
    tiled_ref = graph.corr is not None and getattr(graph.corr, "tiled", False)
    LOOKUP_FN[0] = (("corr_pyramid_lookup_tiled" if tiled_ref else "corr_pyramid_lookup") if args.reference_op else
                    "corr_alt_ce0" if args.corr == "pyramid" or args.lowmem else "corr_lookup_ce0")
    if args.reference_api:
        LOOKUP_FN[0] = "corr_index_forward"
    lookup = graph.corr if args.reference_api else KernelTimer(droid_backends, LOOKUP_FN[0])
    zr = zrp = None
    if not args.reference_op or args.reference_layout:
        zr = KernelTimer(droid_backends, "conv_nhwc_f16", when=lambda *a, **k: k.get("epi") == droid_backends.EPI_GRU_ZR)
        zrp = KernelTimer(droid_backends, "conv_gru_pre_f16", when=lambda *a, **k: a[5] == droid_backends.EPI_GRU_ZR)

    with torch.no_grad():
        t_w = time.time()
        upd = dict(use_inactive=True) if args.config == "C2" else {}
        step_fn = (lambda: graph.update_lowmem(steps=1)) if args.lowmem else (lambda: graph.update(**upd))
        for _ in range(args.warmup):
            step_fn()
        torch.cuda.synchronize(device)
        if rank == 0:
            log("warmup %.1fs, peak HBM %.1f GB" % (time.time() - t_w, torch.cuda.max_memory_allocated(device) / 1e9))
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(device)
        lookup.active = True
        if zr:
            zr.active = zrp.active = True
        if graph.comm is not None:
            graph.comm["_ar_events"] = []
            graph.comm["_solve_events"] = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_fn()
        torch.cuda.synchronize(device)
        if dist_on:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        lookup.active = False
        if zr:
            zr.active = zrp.active = False
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    allreduce = serial = None
    if graph.comm is not None:
        evs, graph.comm["_ar_events"] = graph.comm["_ar_events"], None
        sevs, graph.comm["_solve_events"] = graph.comm["_solve_events"], None
        torch.cuda.synchronize(device)
        if evs:
            allreduce = {"collective": "all_reduce(SUM) of the reduced camera system's input tiles (fp64)",
                         "backend": dist.get_backend(), "payload_bytes": int(evs[0][2]),
                         "per_update": len(evs) // args.steps,
                         "ms_per_gn_iteration": float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))}
        if sevs:
            # the replicated part of a sharded GN iteration: every rank
            # damps and factors the same all-reduced system (dataflow Cholesky + back
            # solve, one launch) - per rank, gathered so the line shows the spread
            solve = torch.tensor([float(np.mean([a.elapsed_time(b) for a, b in sevs]))], dtype=torch.float64,
                                 device=device)
            every = [torch.zeros_like(solve) for _ in range(world)]
            dist.all_gather(every, solve)
            serial = {"solve_ms_per_gn_iteration_per_rank": [float(t.item()) for t in every],
                      "gn_per_update": len(sevs) // args.steps}
    finite = bool(torch.isfinite(video.poses).all() and torch.isfinite(video.disps).all())
    lookup_ms = lookup.mean_ms()
    zr_ms = zr.mean_ms() if zr else None
    factored = bool(zrp and zrp.mean_ms())
    if factored:
        zr_ms = zrp.mean_ms()
    breakdown = stage_breakdown(graph, video) if args.breakdown else None
    frontend = frontend_edge_change(graph, video) if args.config == "C2" else None

    if rank == 0:
        ms = 1000.0 * elapsed / args.steps
        bytes_per_launch = (LOOKUP_BYTES_PER_EDGE if args.reference_op else LOOKUP_CE0_BYTES_PER_EDGE) * e_local
        achieved = bytes_per_launch / (lookup_ms * 1e-3) / 1e9 if lookup_ms else None
        coop = (args.ht // 8) * (args.wd // 8) % 64 == 0   # the cooperative lookup's shape rule (corr_kernels.hip)
        ref_lookup = (("corr_lookup_coop_kernel<true> (cooperative 4-level lookup, NCHW out, 8x8-tiled volume pool)"
                       if coop else "corr_lookup_lvl_kernel<false, true> (4-level lookup, NCHW out, 8x8-tiled volume pool)")
                      if LOOKUP_FN[0] == "corr_pyramid_lookup_tiled" else
                      "corr_lookup_coop_kernel<false> (4-level lookup, NCHW out)" if coop
                      else "corr_lookup_lvl_kernel<false> (4-level lookup, NCHW out)")
        if args.reference_api:
            ref_lookup = ("CorrBlock.__call__ of modules/corr.py:40-50: 4 x corr_index_fwd_kernel<__half> "
                          "(droid_corr_index_forward, one level each, row-major volume) + torch.cat, per call")
        lookup_roof = {"kernel": (ref_lookup if args.reference_op else
                                  "corr_ce0_kernel (4-level lookup fused with corr_encoder[0] 1x1 196->128)"),
                       "bound": "hbm",
                       "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                       "frac": (achieved / PEAK_HBM_GBS) if achieved else None,
                       "traffic": (None if args.reference_api else
                                   load_traffic("corr_lookup_nchw", e_local, "corr_lookup_coop_kernel")
                                   if args.reference_op else load_traffic("corr_lookup", e_local, "corr_ce0_kernel<true>")),
                       "launch_ms": lookup_ms,
                       "algorithmic_bytes_per_launch": bytes_per_launch}
        if zr_ms:
            flops = (ZR_PRE_FLOPS_PER_PIXEL if factored else ZR_FLOPS_PER_PIXEL) * e_local * (args.ht // 8) * (args.wd // 8)
            tf = flops / (zr_ms * 1e-3) / 1e12
            roofline = {"kernel": "%s (ConvGRU z|r gates, 3x3 %d->256, fp16 MFMA%s)"
                                  % (ZR_KERNEL, 320 if factored else 448, ", inp term per source frame" if factored else ""),
                        "bound": "mfma", "achieved": tf, "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                        "frac": tf / PEAK_F16_TFLOPS, "traffic": load_traffic("conv_zr", e_local,
                                                                                ZRP_KERNEL_MATCH if factored else ZR_KERNEL_MATCH),
                        "launch_ms": zr_ms, "algorithmic_flops_per_launch": flops}
        else:
            roofline, lookup_roof = lookup_roof, None
        if args.lowmem or args.corr == "pyramid":
            lookup_roof["kernel"] = ("corr_alt2_kernel (on-demand 4-level correlation windows on MFMA from the "
                                     "feature pyramid, fused with corr_encoder[0] 1x1 196->128)")
            lookup_roof["algorithmic_bytes_per_launch"] = ALT_BYTES_PER_EDGE * e_local
            lookup_roof["achieved"] = ALT_BYTES_PER_EDGE * e_local / (lookup_ms * 1e-3) / 1e9 if lookup_ms else None
            lookup_roof["frac"] = lookup_roof["achieved"] / PEAK_HBM_GBS if lookup_ms else None
            lookup_roof["traffic"] = load_traffic("corr_alt", e_local, "corr_alt2_kernel")
        result = {
            "metric": ("factor_graph.update_lowmem() steps/sec at 256 KF x 2k edges, 384x512" if args.lowmem else "factor_graph.update() iters/sec at 256 KF x 2k edges, 384x512" if args.config == "C3"
                       else "factor_graph.update() iters/sec, C5 %d KF x %d edges, 384x512" % (args.frames, len(ii))
                       if args.config == "C5" else "factor_graph.update() iters/sec, C4 stereo %d KF x %d edges, 384x512" % (args.frames, len(ii))
                       if args.config == "C4" else
                       "factor_graph.update(use_inactive=True) iters/sec, C2 frontend 16-KF buffer x %d edges, 384x512"
                       % len(ii)),
            "value": 1000.0 / ms,
            "unit": "iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f16 (corr volume, update-operator convs) / f32 (BA linearisation, Schur) / f64 (reduced system)",
            "data": "synthetic (SURVEY.md §8d %s graph, random-init UpdateModule)" % args.config,
            "config": {"workload": {"C4": "C4 stereo graph", "C3": "C3 global graph", "C5": "C5 2048-KF global graph",
                                    "C2": "C2 frontend window (use_inactive=True)"}[args.config]
                                   + (": update_lowmem(steps=1, itrs=2), on-demand corr" if args.lowmem else
                                      ": update(itrs=2), %s corr" % args.corr)
                                   + (", reference update() layout + the reference's CorrBlock.__call__ over "
                                      "droid_backends.corr_index_forward + MI355X UpdateModule drop-in"
                                      if args.reference_api else
                                      ", reference update() layout + MI355X UpdateModule drop-in" if args.reference_layout
                                      else ", reference-structured torch UpdateModule" if args.reference_op else ""),
                       "keyframes": args.frames,
                       "edges": len(ii), "image": [args.ht, args.wd], "fmap": [args.ht // 8, args.wd // 8],
                       "parallelism": ("edge-sharded x%d (%s all-reduce of the reduced camera system)"
                                       % (world, "RCCL" if dist.get_backend() == "nccl" else dist.get_backend())
                                       if dist_on else "single GPU (no process group)")},
            "roofline": roofline,
            "state_finite": finite,
        }
        if lookup_roof:
            result["roofline_lookup"] = lookup_roof
        if allreduce:
            result["allreduce"] = allreduce
        if serial:
            # the serial term of the sharded step: replicated solve + all-reduce per GN
            # iteration (max over ranks), times GN iterations per update, over the step
            per_gn = max(serial["solve_ms_per_gn_iteration_per_rank"]) + (allreduce["ms_per_gn_iteration"]
                                                                          if allreduce else 0.0)
            serial["serial_ms_per_update"] = per_gn * serial["gn_per_update"]
            serial["serial_fraction"] = serial["serial_ms_per_update"] / ms
            result["serial"] = serial
        # whole-iteration fraction: max(HBM floor, MFMA floor) / measured update()
        hw = (args.ht // 8) * (args.wd // 8)
        # edges the update operator runs on (C2: the active window; the stored ones only join the BA)
        e_op = e_local if args.config == "C2" else len(ii)
        n_src = len(np.unique(graph._ii)) if args.config == "C2" else len(np.unique(ii))
        conv_flops = (CONV_FLOPS_PER_EDGE_PIXEL * e_op + CONV_FLOPS_PER_FRAME_PIXEL * n_src) * hw
        if factored:   # the algorithm run: the gate's inp term once per edge set (per source
            # frame, cached across updates - FusedUpdateModule._pre), not per edge and update
            conv_flops -= GATE_INP_FLOPS_PER_PIXEL * e_op * hw
        hbm_bytes = HBM_BYTES_PER_EDGE * e_op + HBM_BYTES_PER_FRAME * args.frames
        mfma_floor = conv_flops / (PEAK_F16_TFLOPS * 1e12) * 1e3 / world
        hbm_floor = hbm_bytes / (PEAK_HBM_GBS * 1e9) * 1e3 / world
        result["iteration_roofline"] = {
            "bound": "mfma" if mfma_floor >= hbm_floor else "hbm",
            "mfma_floor_ms": mfma_floor, "hbm_floor_ms": hbm_floor, "measured_ms": ms,
            "frac": max(mfma_floor, hbm_floor) / ms,
            "conv_flops_per_update": conv_flops, "hbm_bytes_per_update": hbm_bytes}
        if breakdown:
            op_ms = breakdown["update_op (convs)"]
            result["iteration_roofline"]["conv_stack"] = {
                "achieved_tflops": conv_flops / world / (op_ms * 1e-3) / 1e12, "peak": PEAK_F16_TFLOPS,
                "frac": conv_flops / world / (op_ms * 1e-3) / 1e12 / PEAK_F16_TFLOPS,
                "update_op_ms": op_ms, "note": "update_op includes the fused lookup + corr_encoder[0]"}
        if breakdown:
            result["breakdown_ms"] = breakdown
        if frontend:
            result["frontend"] = frontend
        if world == 1 and not args.no_cpu_baseline and args.config == "C3":
            try:
                result["cpu_baseline"] = cpu_baseline(graph, video, args)
            except Exception as ex:  # the baseline is reported, never fatal
                result["cpu_baseline"] = {"value": None, "error": repr(ex)}
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Frame graph + recurrent update (mirror of droid_slam/factor_graph.py).

Interface and semantics follow the reference FactorGraph
(factor_graph.py:11-369): edges (ii, jj) with per-edge state net/inp/corr/
target/weight/age, an inactive edge store, `update()` (the hot path,
:196-242) and `update_lowmem()` (:245-290).  Differences are in how, not
what: the edge list is mirrored on the host (numpy) so t0, unique(ii),
scatter indices and the BA plan never need a device->host sync; the motion
features come out of the fused reprojection kernel; the correlation lookup
is one kernel for all levels; BA runs fully on the GPU.
"""
import os
import warnings
import sys

import numpy as np
import torch

import droid_backends

from .corr import AltCorrBlock, CorrBlock, upload
from .fused import PendingAltLookup, PendingLookup, edge_segments


def _coords_grid(ht, wd, device):
    y, x = torch.meshgrid(torch.arange(ht, device=device, dtype=torch.float),
                          torch.arange(wd, device=device, dtype=torch.float), indexing="ij")
    return torch.stack([x, y], dim=-1)


_GRAPH_DEBUG = os.environ.get("DROID_GRAPH_DEBUG", "0") == "1"


class _PointerRecorder:
    """Diagnostics (DROID_GRAPH_DEBUG=1): every device pointer the captured body
    hands the C library (scalar arguments and pointer arrays), checked after the
    capture against the caching allocator's blocks - a pointer into a block that
    is no longer allocated is one the graph's replays would read or write stale."""

    def __init__(self):
        import ctypes
        self.ct = ctypes
        self.calls = []

    def install(self):
        real = droid_backends.lib
        rec = self

        class Proxy:
            def __getattr__(self, name):
                fn = getattr(real, name)
                if not name.startswith("droid_"):
                    return fn

                def wrapped(*a):
                    ptrs = []
                    for i, x in enumerate(a):
                        if isinstance(x, rec.ct.c_void_p) and x.value:
                            ptrs.append((i, x.value))
                        elif isinstance(x, rec.ct.Array) and getattr(x, "_type_", None) is rec.ct.c_void_p:
                            ptrs.extend((("%d[%d]" % (i, j)), v) for j, v in enumerate(x) if v)
                    rec.calls.append((name, ptrs))
                    return fn(*a)
                return wrapped
        self.real = real
        droid_backends.lib = Proxy()

    def remove(self):
        droid_backends.lib = self.real

    def report(self, pool):
        blocks = []
        for sg in torch.cuda.memory_snapshot():
            pid = tuple(sg.get("segment_pool_id", ()))
            for b in sg.get("blocks", []):
                blocks.append((b["address"], b["size"], b["state"], pid))
        blocks.sort()
        import bisect
        starts = [b[0] for b in blocks]
        bad, n = [], 0
        for name, ptrs in self.calls:
            for arg, v in ptrs:
                n += 1
                k = bisect.bisect_right(starts, v) - 1
                if k < 0 or v >= blocks[k][0] + blocks[k][1]:
                    if v < (1 << 40):   # a host handle (the stream), not device memory
                        continue
                    bad.append((name, arg, hex(v), "outside every segment"))
                elif blocks[k][2] != "active_allocated" and blocks[k][3] != tuple(pool):
                    bad.append((name, arg, hex(v), blocks[k][2], blocks[k][3]))
        print("[update graph] %d library calls, %d device pointers captured; stale (free outside the graph's "
              "pool): %s" % (len(self.calls), n, bad[:40]), file=sys.stderr, flush=True)


class FactorGraph:
    def __init__(self, video, update_op, device="cuda:0", corr_impl="volume", max_factors=-1):
        self.video = video
        self.update_op = update_op
        self.device = torch.device(device)
        self.max_factors = max_factors
        self.corr_impl = corr_impl
        self.ht = ht = video.ht // 8
        self.wd = wd = video.wd // 8
        self.coords0 = _coords_grid(ht, wd, self.device)
        self._ii = np.zeros(0, np.int64)   # host mirrors of the edge list
        self._jj = np.zeros(0, np.int64)
        self._ii_inac = np.zeros(0, np.int64)
        self._jj_inac = np.zeros(0, np.int64)
        self._ii_bad = np.zeros(0, np.int64)
        self._jj_bad = np.zeros(0, np.int64)
        self.age = torch.zeros(0, dtype=torch.long, device=self.device)
        self.corr, self.net, self.inp = None, None, None
        self.damping = 1e-6 * torch.ones_like(self.video.disps)
        self.target = torch.zeros([1, 0, ht, wd, 2], device=self.device, dtype=torch.float)
        self.weight = torch.zeros([1, 0, ht, wd, 2], device=self.device, dtype=torch.float)
        self.target_inac = torch.zeros([1, 0, ht, wd, 2], device=self.device, dtype=torch.float)
        self.weight_inac = torch.zeros([1, 0, ht, wd, 2], device=self.device, dtype=torch.float)
        self._dev_cache = {}
        # corr_impl "pyramid" (MI355X): no per-edge volume; update() computes the
        # correlation windows on demand from this feature pyramid of the frames
        self._alt_pyr = None
        self._inp_frames = None   # (inp tensor, first-edge bytes, per-source-frame inp rows)
        self.comm = None  # set for edge-sharded multi-GPU: dict(group, own=(lo,hi), t0, t1, version)
        # fused (MI355X) operator: per-edge hidden state kept channels-last (E,H,W,128)
        from .fused import FusedUpdateModule
        self.fused = isinstance(update_op, FusedUpdateModule)
        # CorrBlock(tiled=...): the volume pool in 8x8 tiles for every operator - the
        # fused lookup reads it, and so does CorrBlock.__call__ (the reference
        # operators' NCHW lookup, droid_corr_pyramid_lookup_tiled); the layout is
        # internal to the block (set False before add_factors for the reference
        # row-major layout)
        self.tiled_volume = True
        # the on-demand lookup's tile walk grouped by target frame (measured
        # within +-3 % of edge order, so off; see _alt_order)
        self.alt_order_by_target = False
        self._version = 0          # bumped by every edge edit
        self._ba_tw = None         # (key, BA target rows, BA weight rows), see _ba_inputs
        # HIP-graph replay of update() per edge set (fused operator, one device,
        # frontend-sized graphs where host issue and launch gaps dominate):
        # DROID_UPDATE_GRAPHS=1 enables it (off by default; see _update_graphed)
        self.graphs = os.environ.get("DROID_UPDATE_GRAPHS", "0") == "1"
        # a failed capture falls back to eager with one warning; strict re-raises (tests)
        self.graph_strict = os.environ.get("DROID_GRAPH_STRICT", "0") == "1"
        self._graph = None         # captured update: dict(key, graph, plan, state, keep)
        self._graph_warm = None    # key of the last eager call (the capture follows it)
        self._cap_stream = None

    # -- per-edge state layout ------------------------------------------------
    @property
    def _edim(self):
        return 0 if self.fused else 1

    def _edge_state(self, x):
        """(E,128,H,W) -> (1,E,128,H,W) (reference layout) or (E,H,W,128) (fused)."""
        if self.fused:
            return x.permute(0, 2, 3, 1).contiguous()
        return x.unsqueeze(0)

    # -- edge-list views ------------------------------------------------------
    def _up(self, arr):
        """host array -> device tensor without waiting for the stream (a copy from
        pageable memory first drains the stream; this one goes through pinned memory)."""
        return upload(arr, self.device)

    def _dev(self, name, arr):
        key = (name, arr.tobytes())
        t = self._dev_cache.get(name)
        if t is None or t[0] != key:
            t = (key, self._up(arr))
            self._dev_cache[name] = t
        return t[1]

    @property
    def ii(self):
        return self._dev("ii", self._ii)

    @property
    def jj(self):
        return self._dev("jj", self._jj)

    @property
    def ii_inac(self):
        return self._dev("ii_inac", self._ii_inac)

    @property
    def jj_inac(self):
        return self._dev("jj_inac", self._jj_inac)

    @staticmethod
    def _host(x):
        if isinstance(x, torch.Tensor):
            return x.detach().to("cpu", torch.long).numpy().reshape(-1)
        return np.asarray(x, dtype=np.int64).reshape(-1)

    # -- graph edits (factor_graph.py:43-193) ---------------------------------
    def _edited(self):
        """edge-set version (sharded BA: the global-edge cache key) - every edit,
        issued in lockstep on all ranks even when it leaves this rank's shard
        unchanged, bumps it, so all ranks agree on when to re-gather.  Drops a
        captured update graph."""
        self._version += 1
        self._drop_graph()
        if self.comm is not None:
            self.comm["version"] = self.comm.get("version", 0) + 1

    def _filter_repeated(self, ii, jj):
        seen = set(zip(self._ii.tolist(), self._jj.tolist())) | set(zip(self._ii_inac.tolist(),
                                                                      self._jj_inac.tolist()))
        keep = np.array([(a, b) not in seen for a, b in zip(ii.tolist(), jj.tolist())], dtype=bool)
        return ii[keep], jj[keep]

    def print_edges(self):
        order = np.argsort(self._ii, kind="stable")
        w = torch.mean(self.weight, dim=[0, 2, 3, 4]).cpu().numpy()
        for e in zip(self._ii[order], self._jj[order], w[order]):
            print(e)
        print()

    def filter_edges(self):
        conf = torch.mean(self.weight, dim=[0, 2, 3, 4]).cpu().numpy()
        mask = (np.abs(self._ii - self._jj) > 2) & (conf < 0.001)
        self._ii_bad = np.concatenate([self._ii_bad, self._ii[mask]])
        self._jj_bad = np.concatenate([self._jj_bad, self._jj[mask]])
        self.rm_factors(mask, store=False)

    def clear_edges(self):
        self.rm_factors(np.ones(len(self._ii), dtype=bool))
        self.net = None
        self.inp = None

    def add_factors(self, ii, jj, remove=False):
        self._edited()
        ii, jj = self._filter_repeated(self._host(ii), self._host(jj))
        if ii.shape[0] == 0:
            return
        if (self.max_factors > 0 and len(self._ii) + len(ii) > self.max_factors
                and self.corr is not None and remove):
            # factor_graph.py:105-106 masks POSITION k by argsort(age)[k] (kept literally)
            order = np.argsort(self.age.cpu().numpy(), kind="stable")
            self.rm_factors(order >= self.max_factors - len(ii), store=True)

        dij = self._up(np.stack([ii, jj]).astype(np.int64))   # one upload
        dii, djj = dij[0], dij[1]
        net = self._edge_state(self.video.nets[dii].to(self.device))
        if self.corr_impl == "volume":
            # the new edges' pyramids from the frames' NHWC features / 4 (one kernel;
            # the stereo edge (i, i) correlates against the right image,
            # factor_graph.py:112-114); the fused operator reads the 8x8-tiled layout
            # only the frames the new edges touch (one keyframe's edges touch a few)
            num, rig, ch, ht, wd = self.video.fmaps.shape
            rows_1 = (rig * ii).astype(np.int64)
            rows_2 = (rig * jj + ((ii == jj) & (rig > 1))).astype(np.int64)
            used, inv = np.unique(np.concatenate([rows_1, rows_2]), return_inverse=True)
            up = self._up(np.concatenate([used, inv]).astype(np.int32))   # one upload
            fm = self.video.fmaps.reshape(num * rig, ch, ht, wd).index_select(0, up[:len(used)])
            frames = torch.empty((len(used), ht, wd, ch), dtype=torch.float16, device=self.device)
            torch.mul(fm.permute(0, 2, 3, 1), 0.25, out=frames)     # NHWC / 4 in one pass (exact in fp16)
            f1, f2 = up[len(used):len(used) + len(ii)], up[len(used) + len(ii):]
            tiled = self.tiled_volume
            if droid_backends.corr_volume_pyramid_supported(ht, wd, tiled and wd // 8 % 8 == 0):
                corr = CorrBlock.from_frames(frames, f1, f2, tiled=tiled)
            else:
                c = self._up((ii == jj).astype(np.int64))
                corr = CorrBlock(self.video.fmaps[dii, 0].unsqueeze(0), self.video.fmaps[djj, c].unsqueeze(0),
                                 tiled=tiled)
            self.corr = corr if self.corr is None else self.corr.cat(corr)
        if self.corr_impl == "pyramid":
            self._alt_pyr = None   # frames may have changed: rebuilt at the next update
        if self.corr_impl in ("volume", "pyramid"):
            inp = self._edge_state(self.video.inps[dii].to(self.device))
            self.inp = inp if self.inp is None else torch.cat([self.inp, inp], self._edim)

        target, _ = self.video.reproject(dii, djj)
        weight = torch.zeros_like(target)
        self._ii = np.concatenate([self._ii, ii])
        self._jj = np.concatenate([self._jj, jj])
        self.age = torch.cat([self.age, torch.zeros_like(dii)], 0)
        self.net = net if self.net is None else torch.cat([self.net, net], self._edim)
        self.target = torch.cat([self.target, target], 1)
        self.weight = torch.cat([self.weight, weight], 1)

    def rm_factors(self, mask, store=False):
        # the reference frontend passes device bool tensors (droid_frontend.py:42,106)
        if isinstance(mask, torch.Tensor):
            mask = mask.detach().cpu().numpy()
        mask = np.asarray(mask, dtype=bool).reshape(-1)
        self._edited()
        keep = ~mask
        # host index lists, one upload: a device bool mask would sync per tensor (nonzero)
        nk = int(keep.sum())
        both = self._up(np.concatenate([np.flatnonzero(keep), np.flatnonzero(mask)]))
        dkeep, dgone = both[:nk], both[nk:]
        if store:
            self._ii_inac = np.concatenate([self._ii_inac, self._ii[mask]])
            self._jj_inac = np.concatenate([self._jj_inac, self._jj[mask]])
            self.target_inac = torch.cat([self.target_inac, self.target.index_select(1, dgone)], 1)
            self.weight_inac = torch.cat([self.weight_inac, self.weight.index_select(1, dgone)], 1)
        self._ii = self._ii[keep]
        self._jj = self._jj[keep]
        self.age = self.age.index_select(0, dkeep)
        if self.corr_impl == "volume" and self.corr is not None:
            self.corr = self.corr.select(keep)   # a slot pool: frees rows, copies nothing
        if self.net is not None:
            self.net = self.net.index_select(0 if self.fused else 1, dkeep)
        if self.inp is not None:
            self.inp = self.inp.index_select(0 if self.fused else 1, dkeep)
        self.target = self.target.index_select(1, dkeep)
        self.weight = self.weight.index_select(1, dkeep)

    def rm_keyframe(self, ix):
        self._edited()
        self._alt_pyr = None   # frames shift
        v = self.video
        with v.get_lock():
            for buf in (v.images, v.poses, v.disps, v.disps_sens, v.intrinsics, v.nets, v.inps, v.fmaps):
                buf[ix] = buf[ix + 1]
        m = (self._ii_inac == ix) | (self._jj_inac == ix)
        self._ii_inac = np.where(self._ii_inac >= ix, self._ii_inac - 1, self._ii_inac)
        self._jj_inac = np.where(self._jj_inac >= ix, self._jj_inac - 1, self._jj_inac)
        if m.any():
            dm = self._up(np.flatnonzero(~m))
            self._ii_inac = self._ii_inac[~m]
            self._jj_inac = self._jj_inac[~m]
            self.target_inac = self.target_inac.index_select(1, dm)
            self.weight_inac = self.weight_inac.index_select(1, dm)
        m = (self._ii == ix) | (self._jj == ix)
        self._ii = np.where(self._ii >= ix, self._ii - 1, self._ii)
        self._jj = np.where(self._jj >= ix, self._jj - 1, self._jj)
        self.rm_factors(m, store=False)

    # -- the hot path (factor_graph.py:196-242) -------------------------------
    def update(self, t0=None, t1=None, itrs=2, use_inactive=False, EP=1e-7, motion_only=False):
        args = (t0, t1, itrs, use_inactive, EP, motion_only)
        if self.graphs and self.fused and self.comm is None and 0 < len(self._ii) <= 512:
            return self._update_graphed(args)
        self._update(*args)

    def _drop_graph(self):
        """Release the captured update graph.  The caller's stream is synchronised
        first: no replay may still be running when the graph's executable and its
        private memory pool go."""
        if self._graph is not None:
            torch.cuda.current_stream(self.device).synchronize()
            self._graph = None
        self._graph_warm = None

    def _graph_keep(self):
        """Strong references to every tensor the captured body reads or writes
        by raw pointer (caches that a later call could replace and free while
        the graph still holds their addresses)."""
        keep = dict(dev=dict(self._dev_cache), inp=self.inp, inp_frames=self._inp_frames, ba_tw=self._ba_tw,
                    damping=self.damping, target_inac=self.target_inac, weight_inac=self.weight_inac,
                    pre=getattr(self.update_op, "_pre", None), packed=getattr(self.update_op, "_packed", None))
        if self.corr is not None:
            keep["corr"] = (list(getattr(self.corr, "_pyr", [])), getattr(self.corr, "_slot_dev", None))
        return keep

    def _graph_pool_report(self, graph, static):
        """Diagnostics (DROID_GRAPH_DEBUG=1): every live CUDA tensor whose memory
        lies in the just-captured graph's private pool (an allocation made inside
        the capture that outlived it), named by where this graph, its module,
        correlation block, video or droid_backends hold it.  With
        DROID_GRAPH_DEBUG_STOP=n the n-th capture raises after the report."""
        import gc
        torch.cuda.synchronize(self.device)
        pid = tuple(graph.pool())
        segs = [(sg["address"], sg["total_size"]) for sg in torch.cuda.memory_snapshot()
                if tuple(sg.get("segment_pool_id", ())) == pid]
        inpool = lambda t: any(a <= t.data_ptr() < a + n for a, n in segs)
        live = [t for t in gc.get_objects() if isinstance(t, torch.Tensor) and t.is_cuda and inpool(t)]
        owners = dict(graph=self.__dict__, update_op=self.update_op.__dict__, video=self.video.__dict__,
                      backends=vars(droid_backends))
        if self.corr is not None:
            owners["corr"] = self.corr.__dict__

        def walk(x, path, out, depth=0):
            if isinstance(x, torch.Tensor):
                if x.is_cuda and inpool(x):
                    out.append(path)
            elif depth < 4 and isinstance(x, dict):
                for k, v in list(x.items())[:200]:
                    walk(v, "%s[%r]" % (path, k), out, depth + 1)
            elif depth < 4 and isinstance(x, (list, tuple)):
                for i, v in enumerate(list(x)[:200]):
                    walk(v, "%s[%d]" % (path, i), out, depth + 1)
        named = []
        for nm, d in owners.items():
            for k, v in list(d.items()):
                walk(v, "%s.%s" % (nm, k), named)
        print("[update graph] pool %s: %d segments, %d live tensors in the pool; held by: %s" % (
            pid, len(segs), len(live), named[:40]), file=sys.stderr, flush=True)
        self._n_captures = getattr(self, "_n_captures", 0) + 1

    def _update_graphed(self, args):
        """update() through a HIP graph of this edge set: the first call is eager
        (it fills every cache the body reads: edge-list uploads, the BA plan,
        the per-frame inp rows and gate term), the second captures the body and
        replays it, later ones only replay.  The per-edge state (net, target,
        weight) lives in static buffers the graph reads and refills, so replay
        t+1 sees replay t's output; an edge edit drops the graph.

        Capture safety (round 4): nothing may be uploaded or
        allocated for the body's inputs inside the capture - a host-to-device
        copy captured from a pinned staging buffer would re-read that buffer at
        every replay after the host allocator had recycled it (stale indices),
        and a BA plan built inside the capture would live in the graph's pool.
        upload() and get_plan() raise during a capture; the capture then falls
        back to eager for good.  Every tensor the graph addresses is kept alive
        by the graph record, and a graph is only released after its stream is
        synchronised."""
        key = (self._version, self.video.counter.value) + args
        dbg = _GRAPH_DEBUG

        def trace(phase):
            if dbg:   # diagnostics: each phase synchronised and named (never inside a capture)
                torch.cuda.synchronize(self.device)
                print("[update graph] %s key=%s" % (phase, key), file=sys.stderr, flush=True)
        g = self._graph
        if g is not None and g["key"] == key:
            for name in ("net", "target", "weight"):      # state replaced from outside: copy it in
                cur = getattr(self, name)
                if cur is not g[name]:
                    g[name].copy_(cur)
                    setattr(self, name, g[name])
            trace("replay begin")
            g["graph"].replay()
            g["plan"]._record_status()
            self.age += 1
            trace("replay done")
            return
        if self._cap_stream is None:
            self._cap_stream = torch.cuda.Stream(device=self.device)
        cs, main = self._cap_stream, torch.cuda.current_stream(self.device)
        if self._graph_warm != key:
            # eager warm-up on the capture stream (torch's rule: lazily created
            # per-stream state must not be born inside the capture), ordered both ways
            trace("warm begin")
            self._drop_graph()
            self._graph_warm = key
            cs.wait_stream(main)
            with torch.cuda.stream(cs):
                self._update(*args)
            main.wait_stream(cs)
            trace("warm done")
            return
        trace("capture begin")
        droid_backends.check_status()        # no host wait may happen inside the capture
        saved = (self.net, self.target, self.weight)
        static = dict(net=self.net, target=self.target, weight=self.weight.clone())
        self.weight = static["weight"]
        graph = torch.cuda.CUDAGraph()
        cs.wait_stream(main)
        rec = _PointerRecorder() if dbg else None
        try:
            with torch.cuda.graph(graph, stream=cs):
                if rec is not None:
                    rec.install()
                plan = self._update(*args, age=False)
                for name in ("net", "target", "weight"):   # this update's state -> the static inputs
                    static[name].copy_(getattr(self, name))
                if rec is not None:
                    rec.remove()
        except Exception as exc:
            if rec is not None:
                rec.remove()
            # capture unsupported here (an upload, a plan build, an op that syncs): stay
            # eager, and say so once - or re-raise when capture safety is under test
            main.wait_stream(cs)
            self.net, self.target, self.weight = saved
            self.graphs = False
            if self.graph_strict:
                raise
            warnings.warn("FactorGraph: HIP-graph capture of update() failed (%s: %s); update() runs eagerly "
                          "from now on" % (type(exc).__name__, exc), RuntimeWarning, stacklevel=3)
            self._update(*args)
            return
        main.wait_stream(cs)
        trace("captured")
        self.net, self.target, self.weight = static["net"], static["target"], static["weight"]
        if dbg:
            self._graph_pool_report(graph, static)
            rec.report(graph.pool())
        self._graph = dict(key=key, graph=graph, plan=plan, keep=self._graph_keep(), **static)
        if dbg:   # integrity of what the graph only reads: unchanged by a replay?
            ro = {"plan.ints": plan.ints_region()}
            for nm, (_, t) in self._dev_cache.items():
                ro["dev." + nm] = t
            if self.corr is not None and getattr(self.corr, "_slot_dev", None) is not None:
                ro["corr.slots"] = self.corr._slot_dev
            before = {nm: t.clone() for nm, t in ro.items()}
            # do allocations made after the capture land in the graph's private pool?
            pid = tuple(graph.pool())
            segs = [(sg["address"], sg["total_size"]) for sg in torch.cuda.memory_snapshot()
                    if tuple(sg.get("segment_pool_id", ())) == pid]
            probe = [torch.empty(n, dtype=torch.uint8, device=self.device) for n in (512, 4096, 65536, 1 << 20, 4 << 20)]
            inside = [nm for nm, t in list(before.items()) + [("probe%d" % i, t) for i, t in enumerate(probe)]
                      if any(a <= t.data_ptr() < a + n for a, n in segs)]
            print("[update graph] post-capture allocations inside the graph's pool: %s" % (inside,), file=sys.stderr,
                  flush=True)
            del probe
            if os.environ.get("DROID_GRAPH_DEBUG_STOP_BEFORE_REPLAY", "0") == "1":
                raise RuntimeError("graph debug stop before the first replay")
        graph.replay()
        plan._record_status()
        self.age += 1
        trace("first replay done")
        if dbg:
            changed = [nm for nm, t in ro.items() if not torch.equal(t, before[nm])]
            print("[update graph] read-only inputs changed by the replay: %s" % (changed,), file=sys.stderr, flush=True)
            stop = int(os.environ.get("DROID_GRAPH_DEBUG_STOP", "0"))
            if stop and self._n_captures >= stop:
                raise RuntimeError("graph debug stop after capture %d" % self._n_captures)

    def _update(self, t0=None, t1=None, itrs=2, use_inactive=False, EP=1e-7, motion_only=False, age=True):
        ht, wd = self.ht, self.wd
        E = len(self._ii)
        ii, jj = self.ii, self.jj
        with torch.autocast("cuda", enabled=False):
            coords1, _, motn = droid_backends.projective_transform(
                self.video.poses, self.video.disps, self.video.intrinsics, ii, jj,
                target=self.target.view(E, ht, wd, 2), with_valid=False)
            coords1 = coords1.view(1, E, ht, wd, 2)
            motn = motn.view(1, E, 4, ht, wd)

        uniq, inverse = np.unique(self._ii, return_inverse=True)
        dinv = self._dev("inverse", inverse.astype(np.int64))
        if self.fused:
            if self.corr_impl == "pyramid":
                corr = self._pending_alt_lookup(coords1)   # windows computed on demand (no volume)
            else:
                corr = PendingLookup(self.corr, coords1)   # lookup runs fused with corr_encoder[0]
            ptr, idx = edge_segments(inverse, len(uniq))
            segs = (self._dev("seg_ptr", ptr), self._dev("seg_idx", idx))
            # every edge leaving a frame holds the same context features (video.inps[ii],
            # factor_graph.py:118): one row per source frame - the first edge of its
            # segment - lets the gate convs compute their inp term once per frame
            inp_frames = None
            if self.inp is not None:
                # the per-frame rows change only with the edge set (add/rm_factors)
                # (the cache holds self.inp itself: a new edge set is a new tensor object)
                first = idx[ptr[:-1]]
                c = self._inp_frames
                if c is None or c[0] is not self.inp or c[1] != first.tobytes():
                    c = self._inp_frames = (self.inp, first.tobytes(),
                                            self.inp.index_select(0, self._dev("seg_first", first)))
                inp_frames = c[2]
            raw = hasattr(self.update_op, "head_bias")
            self.net, delta, weight, damping = self.update_op(self.net, self.inp, corr, motn[0], dinv, len(uniq),
                                                              segments=segs, inp_frames=inp_frames, raw_head=raw)
        else:
            corr = self.corr(coords1)
            with torch.autocast("cuda", enabled=True):
                self.net, delta, weight, damping, upmask = self.update_op(
                    self.net, self.inp, corr, motn, ii, jj, inverse=dinv, num_unique=len(uniq))

        if t0 is None:
            t0 = self.comm["t0"] if self.comm is not None else max(1, int(self._ii.min()) + 1)

        with torch.autocast("cuda", enabled=False):
            if use_inactive:
                m = (self._ii_inac >= t0 - 3) & (self._jj_inac >= t0 - 3)
                ii_h = np.concatenate([self._ii_inac[m], self._ii])
                jj_h = np.concatenate([self._jj_inac[m], self._jj])
            else:
                m = None
                ii_h, jj_h = self._ii, self._jj
            if self.fused and weight is None:
                # fused heads: one kernel adds the bias, takes the sigmoid, forms
                # target = coords1 + delta and writes both maps straight into the
                # BA's (rows,2,H,W) inputs, whose inactive rows are filled once
                # per edge set (no per-update transposes or concatenation)
                target, weight = self._ba_inputs(m, E)
                n_in = target.shape[0] - E
                t_act, w_act = droid_backends.head_finish(delta, self.update_op.head_bias(), coords1[0], target,
                                                          weight, n_in)
                self.target, self.weight = t_act.unsqueeze(0), w_act.unsqueeze(0)
            else:
                self.target = coords1 + delta.to(dtype=torch.float)
                self.weight = weight.to(dtype=torch.float)
                if use_inactive:
                    # the selection as a cached index (a boolean mask would sync on its count)
                    if m.all():
                        t_in, w_in = self.target_inac, self.weight_inac
                    else:
                        sel = self._dev("inac_sel", np.nonzero(m)[0].astype(np.int64))
                        t_in, w_in = self.target_inac.index_select(1, sel), self.weight_inac.index_select(1, sel)
                    target = torch.cat([t_in, self.target], 1)
                    weight = torch.cat([w_in, self.weight], 1)
                else:
                    target, weight = self.target, self.weight
                target = target.view(-1, ht, wd, 2).permute(0, 3, 1, 2).contiguous()
                weight = weight.view(-1, ht, wd, 2).permute(0, 3, 1, 2).contiguous()
            uniq_ba = np.unique(ii_h)
            if damping.dtype == torch.float16:
                # the fused module's raw eta conv: one kernel applies 0.01 softplus, stores
                # the frames' damping and gathers 0.2 damping + EP for the BA's frames
                rows = np.searchsorted(uniq, uniq_ba)
                hit = (rows < len(uniq)) & (uniq[np.minimum(rows, len(uniq) - 1)] == uniq_ba)
                K = len(uniq_ba)
                mf = self._dev("eta_map", np.concatenate([np.where(hit, rows, -1), uniq_ba]).astype(np.int32))
                damping = droid_backends.eta_damping(damping, mf[:K], mf[K:], self.damping, EP)
            else:
                self.damping[self._dev("uniq", uniq)] = damping[0].to(torch.float)
                damping = 0.2 * self.damping[self._dev("uniq_ba", uniq_ba)].contiguous() + EP
            self.video.ba(target, weight, damping, self._dev("ii_ba", ii_h), self._dev("jj_ba", jj_h),
                          t0, t1, itrs=itrs, lm=1e-4, ep=0.1, motion_only=motion_only,
                          ii_host=ii_h, jj_host=jj_h, comm=self.comm,
                          edge_tag="update+inactive" if use_inactive else "update")
        if age:
            self.age += 1
        return droid_backends.last_plan()

    def _ba_inputs(self, m, E):
        """The BA's target / weight inputs (rows,2,H,W) f32 for update(): the
        selected inactive edges' rows first (mask m over the inactive store, or
        None), filled once per edge set and selection, then E rows the heads'
        finish writes every update."""
        key = (self._version, E, None if m is None else m.tobytes())
        c = self._ba_tw
        if c is None or c[0] != key:
            ht, wd = self.ht, self.wd
            sel = np.zeros(0, np.int64) if m is None else np.nonzero(m)[0]
            n_in = len(sel)
            rows = n_in + E
            # storage reused across edge sets while it is large enough (rows rounded
            # up to 32): an edit then costs the inactive rows' refill, not an allocation
            if c is None or c[3].shape[0] < rows:
                cap = (rows + 31) // 32 * 32
                st = torch.empty((cap, 2, ht, wd), dtype=torch.float32, device=self.device)
                sw = torch.empty_like(st)
            else:
                st, sw = c[3], c[4]
            tb, wb = st[:rows], sw[:rows]
            if n_in:
                idx = self._dev("inac_sel", sel)
                tb[:n_in] = self.target_inac[0].index_select(0, idx).permute(0, 3, 1, 2)
                wb[:n_in] = self.weight_inac[0].index_select(0, idx).permute(0, 3, 1, 2)
            c = self._ba_tw = (key, tb, wb, st, sw)
        return c[1], c[2]

    def _pending_alt_lookup(self, coords1):
        """corr_impl "pyramid": AltCorrBlock pyramid of the frames (built once per
        edge-set change) + per-edge pyramid rows: f1 = fmaps[ii, 0], f2 =
        fmaps[jj, ii == jj] (the stereo edge reads the right image,
        factor_graph.py:112-114)."""
        num, rig = self.video.fmaps.shape[:2]
        n = max(int(self.video.counter.value), int(max(self._ii.max(), self._jj.max())) + 1)
        if self._alt_pyr is None or self._alt_pyr[0] != n:
            f = self.video.fmaps[:n]
            blk = AltCorrBlock(f.reshape((1, n * rig) + tuple(f.shape[2:])))
            self._alt_pyr = (n, [lv.view((-1,) + tuple(lv.shape[2:])) for lv in blk.pyramid])
        f1 = self._dev("alt_f1", (rig * self._ii).astype(np.int32))
        f2h = (rig * self._jj + ((self._ii == self._jj) & (rig > 1))).astype(np.int32)
        f2 = self._dev("alt_f2", f2h)
        return PendingAltLookup(self._alt_pyr[1], f1, f2, coords1, order=self._alt_order(f2h))

    def _alt_order(self, f2h):
        """the on-demand lookup's tile walk, opt-in (alt_order_by_target): edges
        grouped by target frame (stable sort), so the tiles that read one frame's
        pyramid rows run together.  Measured at C3 (profiles/r04/r04n_alt_time.txt):
        within +-3 % of edge order for every XCD chunk size - the kernel is bound
        by its per-tile phases, not by L2 misses - so edge order is the default."""
        if not self.alt_order_by_target:
            return None
        return self._dev("alt_order", np.argsort(f2h, kind="stable").astype(np.int32))

    def update_lowmem(self, t0=None, t1=None, itrs=2, use_inactive=False, EP=1e-7, steps=8):
        """factor_graph.py:245-290: `steps` x [reprojection, on-the-fly (alt)
        correlation + update operator, BA over poses [1, t) with lm=1e-5,
        ep=1e-2] - the global-BA backend's update (droid_backend.py:31-38).

        The reference walks the source frames in chunks of 8 to bound the memory
        of its fp32 correlation; every per-edge stage and GraphAgg's per-frame
        mean are independent across chunks, so the fused path runs all edges in
        one pass: the lookup is corr_alt_ce0 (windows computed on demand from the
        feature pyramid of the frames, fused with corr_encoder[0]) and the gate
        convs take the context term per source frame (video.inps[ii])."""
        t = self.video.counter.value
        num, rig, ch, ht, wd = self.video.fmaps.shape
        E = len(self._ii)
        if self.fused:
            f = self.video.fmaps[:num]
            blk = AltCorrBlock(f.reshape((1, num * rig) + tuple(f.shape[2:])))
            pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in blk.pyramid]
            f1 = self._dev("alt_f1", (rig * self._ii).astype(np.int32))
            f2h = (rig * self._jj + ((self._ii == self._jj) & (rig > 1))).astype(np.int32)
            f2 = self._dev("alt_f2", f2h)
            alt_order = self._alt_order(f2h)
            uniq, inverse = np.unique(self._ii, return_inverse=True)
            dinv = self._dev("inverse", inverse.astype(np.int64))
            ptr, idx = edge_segments(inverse, len(uniq))
            segs = (self._dev("seg_ptr", ptr), self._dev("seg_idx", idx))
            duniq = self._dev("uniq", uniq)
            # the source frames' context features: the same tensor for every step
            # (the update operator caches its per-frame gate term on it)
            inp_frames = self.video.inps[duniq].permute(0, 2, 3, 1).contiguous()
        else:
            corr_op = AltCorrBlock(self.video.fmaps.view(1, num * rig, ch, ht, wd))
        for _ in range(steps):
            with torch.autocast("cuda", enabled=False):
                coords1, _, motn = droid_backends.projective_transform(
                    self.video.poses, self.video.disps, self.video.intrinsics, self.ii, self.jj,
                    target=self.target.view(E, ht, wd, 2), with_valid=False)
                coords1 = coords1.view(1, E, ht, wd, 2)
                motn = motn.view(1, E, 4, ht, wd)
            if self.fused:
                corr = PendingAltLookup(pyr, f1, f2, coords1, order=alt_order)
                self.net, delta, weight, damping = self.update_op(self.net, None, corr, motn[0], dinv, len(uniq),
                                                                  segments=segs, inp_frames=inp_frames)
                with torch.autocast("cuda", enabled=False):
                    self.target = coords1 + delta.to(dtype=torch.float)
                    self.weight = weight.to(dtype=torch.float)
                    self.damping[duniq] = damping[0].to(torch.float)
            else:
                self._lowmem_chunks(corr_op, coords1, motn, rig)
            damping = 0.2 * self.damping[self._dev("uniq_all", np.unique(self._ii))].contiguous() + EP
            target = self.target.view(-1, ht, wd, 2).permute(0, 3, 1, 2).contiguous()
            weight = self.weight.view(-1, ht, wd, 2).permute(0, 3, 1, 2).contiguous()
            self.video.ba(target, weight, damping, self.ii, self.jj, 1, t, itrs=itrs, lm=1e-5, ep=1e-2,
                          motion_only=False, ii_host=self._ii, jj_host=self._jj, comm=self.comm, edge_tag="lowmem")
            self.video.dirty[:t] = True

    def _lowmem_chunks(self, corr_op, coords1, motn, rig):
        """the reference-structured operator: chunks of 8 source frames (factor_graph.py:262-280)."""
        s = 8
        for i in range(0, int(self._jj.max()) + 1, s):
            vh = (self._ii >= i) & (self._ii < i + s)
            if not vh.any():
                continue
            v = self._up(vh)
            iis_h, jjs_h = self._ii[vh], self._jj[vh]
            iis = self._up(iis_h)
            jjs = self._up(jjs_h)
            src = self._up(rig * iis_h)
            dst = self._up(rig * jjs_h + (iis_h == jjs_h))
            corr1 = corr_op(coords1[:, v], src, dst)
            uq, inv = np.unique(iis_h, return_inverse=True)
            dinv = self._up(inv)
            with torch.autocast("cuda", enabled=True):
                net, delta, weight, damping, _ = self.update_op(
                    self.net[:, v], self.video.inps[None, iis], corr1, motn[:, v], iis, jjs,
                    inverse=dinv, num_unique=len(uq))
            self.net[:, v] = net
            self.target[:, v] = coords1[:, v] + delta.float()
            self.weight[:, v] = weight.float()
            self.damping[self._up(uq)] = damping[0].float()

    # -- edge construction (factor_graph.py:292-369) --------------------------
    def add_neighborhood_factors(self, t0, t1, r=3):
        ii, jj = np.meshgrid(np.arange(t0, t1), np.arange(t0, t1), indexing="ij")
        ii, jj = ii.reshape(-1), jj.reshape(-1)
        c = 1 if self.video.stereo else 0
        keep = (np.abs(ii - jj) > c) & (np.abs(ii - jj) <= r)
        self.add_factors(ii[keep], jj[keep])

    def proximity_factor_list(self, t0=0, t1=0, rad=2, nms=2, beta=0.25, thresh=16.0):
        """the edge list add_proximity_factors adds (factor_graph.py:305-368):
        the meshgrid distances on the device (droid_frame_distance, both
        directions), then proximity_edge_list -> (k, 2) int64 numpy."""
        t = self.video.counter.value
        dev = self.video.poses.device
        ii, jj = torch.meshgrid(torch.arange(t0, t, device=dev), torch.arange(t1, t, device=dev), indexing="ij")
        d = self.video.distance(ii.reshape(-1), jj.reshape(-1), beta=beta)
        return proximity_edge_list(d, t0, t1, t, rad, nms, thresh, np.concatenate([self._ii, self._ii_bad, self._ii_inac]),
                                   np.concatenate([self._jj, self._jj_bad, self._jj_inac]), self.video.stereo,
                                   self.max_factors)

    def add_proximity_factors(self, t0=0, t1=0, rad=2, nms=2, beta=0.25, thresh=16.0, remove=False):
        """factor_graph.py:305-369 (proximity_factor_list, then add_factors)."""
        es = self.proximity_factor_list(t0, t1, rad, nms, beta, thresh)
        self.add_factors(es[:, 0], es[:, 1], remove)


def proximity_edge_list(d, t0, t1, t, rad, nms, thresh, ii_all, jj_all, stereo, max_factors):
    """The edge list add_proximity_factors hands to add_factors
    (factor_graph.py:312-369) from the device distances d ((t-t0)*(t-t1), f32):
    the candidate mask, the NMS suppression around ii_all/jj_all (the graph's
    ii|ii_bad|ii_inac), the sort and the greedy accept-and-suppress walk run in
    droid_proximity_select (csrc/proximity_kernels.hip); only the accepted
    pairs come back.  The static neighbour edges are built here, in the
    reference's order, and lead the list.  -> (k, 2) int64 numpy."""
    es = []
    for i in range(t0, t):                  # :333-341
        if stereo:
            es.append((i, i))
        for j in range(max(i - rad - 1, 0), i):
            es.append((i, j))
            es.append((j, i))
    # :355-356 - a candidate is appended while len(es) <= max_factors
    n_cap = (max_factors - len(es)) // 2 + 1 if max_factors >= len(es) else 0
    n_cap = min(n_cap, (t - t0) * (t - t1))
    dev = d.device
    ei = torch.from_numpy(np.asarray(ii_all).astype(np.int32)).to(dev)
    ej = torch.from_numpy(np.asarray(jj_all).astype(np.int32)).to(dev)
    pairs = droid_backends.proximity_select(d.float().contiguous(), t0, t1, t, rad, nms, thresh, ei, ej, stereo,
                                            n_cap).cpu().numpy().astype(np.int64)
    es = np.asarray(es, dtype=np.int64).reshape(-1, 2)
    both = np.stack([pairs, pairs[:, ::-1]], 1).reshape(-1, 2)   # (i, j), (j, i) per accepted pair
    return np.concatenate([es, both], 0)

"""Generate golden input/output vectors by importing the REFERENCE's own Python.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

It imports /root/reference/droid_slam with import-only stubs for the
un-vendored / CUDA-only modules (`droid_backends`, `lietorch`) and a
restatement of `torch_scatter.scatter_mean` (third-party, not installed;
restated below as an index_add mean).  Every fixture is
computed in fp32 on CPU by the reference code itself:

  corr_pyramid.npz   CorrBlock(fmap1, fmap2).corr_pyramid   (modules/corr.py:24-38,63-71)
  alt_pyramid.npz    AltCorrBlock(fmaps).pyramid            (modules/corr.py:92-104)
  update_module.npz  UpdateModule.forward(...)              (droid_net.py:111-143, gru.py:19-32)
  convgru.npz        ConvGRU.forward(...)                   (modules/gru.py:19-32)
  cvx_upsample.npz   cvx_upsample(...)                      (droid_net.py:21-35)

Weights come from tests/golden/fill.py (RNG-free), inputs from a seeded numpy
generator; both are stored in the fixture so the tests never re-derive them.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/droid_slam"
sys.path.insert(0, HERE)
from fill import det_fill  # noqa: E402


def _install_stubs():
    for name in ["droid_backends", "lietorch", "torch_scatter"]:
        sys.modules[name] = types.ModuleType(name)
    lt = sys.modules["lietorch"]
    lt.SE3 = lt.Sim3 = lt.SO3 = type("Stub", (), {})

    def scatter_mean(src, index, dim=-1, dim_size=None):
        # torch_scatter.scatter_mean restated: mean of src slices sharing an index.
        dim = dim % src.dim()
        n = int(index.max()) + 1 if dim_size is None else dim_size
        shape = list(src.shape)
        shape[dim] = n
        out = torch.zeros(shape, dtype=src.dtype)
        out.index_add_(dim, index, src)
        cnt = torch.zeros(n, dtype=src.dtype)
        cnt.index_add_(0, index, torch.ones_like(index, dtype=src.dtype))
        view = [1] * src.dim()
        view[dim] = n
        return out / cnt.clamp(min=1).view(view)

    ts = sys.modules["torch_scatter"]
    ts.scatter_mean = scatter_mean
    ts.scatter_sum = None


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    from modules.corr import CorrBlock, AltCorrBlock
    from modules.gru import ConvGRU
    import droid_net

    torch.set_grad_enabled(False)
    rng = np.random.default_rng(2024)

    # --- CorrBlock pyramid (all-pairs volume + avg-pool levels) ---------------
    f1 = rng.standard_normal((1, 2, 128, 16, 16)).astype(np.float32)
    f2 = rng.standard_normal((1, 2, 128, 16, 16)).astype(np.float32)
    cb = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=4, radius=3)
    np.savez_compressed(os.path.join(HERE, "corr_pyramid.npz"), fmap1=f1, fmap2=f2,
                        **{f"level{i}": cb.corr_pyramid[i].numpy() for i in range(4)})

    # --- AltCorrBlock feature pyramid -----------------------------------------
    fm = rng.standard_normal((1, 3, 128, 16, 16)).astype(np.float32)
    ab = AltCorrBlock(torch.from_numpy(fm), num_levels=4, radius=3)
    np.savez_compressed(os.path.join(HERE, "alt_pyramid.npz"), fmaps=fm,
                        **{f"level{i}": ab.pyramid[i].numpy() for i in range(4)})

    # --- ConvGRU (small planes) ------------------------------------------------
    gru = ConvGRU(16, 24)
    det_fill(gru)
    h = np.tanh(rng.standard_normal((2, 16, 6, 8))).astype(np.float32)
    x1 = rng.standard_normal((2, 10, 6, 8)).astype(np.float32)
    x2 = rng.standard_normal((2, 14, 6, 8)).astype(np.float32)
    out = gru(torch.from_numpy(h), torch.from_numpy(x1), torch.from_numpy(x2))
    np.savez_compressed(os.path.join(HERE, "convgru.npz"), h=h, x1=x1, x2=x2, out=out.numpy())

    # --- UpdateModule (full planes, tiny spatial size) -------------------------
    um = droid_net.UpdateModule()
    det_fill(um)
    E, H, W = 5, 6, 8
    net = np.tanh(rng.standard_normal((1, E, 128, H, W))).astype(np.float32)
    inp = np.maximum(rng.standard_normal((1, E, 128, H, W)), 0).astype(np.float32)
    corr = rng.standard_normal((1, E, 196, H, W)).astype(np.float32)
    flow = np.clip(4.0 * rng.standard_normal((1, E, 4, H, W)), -64, 64).astype(np.float32)
    ii = np.array([0, 0, 1, 2, 2], dtype=np.int64)
    jj = np.array([1, 2, 0, 1, 3], dtype=np.int64)
    net_o, delta, weight, eta, upmask = um(
        torch.from_numpy(net), torch.from_numpy(inp), torch.from_numpy(corr),
        torch.from_numpy(flow), torch.from_numpy(ii), torch.from_numpy(jj))
    np.savez_compressed(os.path.join(HERE, "update_module.npz"), net=net, inp=inp, corr=corr,
                        flow=flow, ii=ii, jj=jj, net_out=net_o.numpy(), delta=delta.numpy(),
                        weight=weight.numpy(), eta=eta.numpy(), upmask=upmask.numpy())

    # --- convex upsampling (used by DepthVideo.upsample) -----------------------
    data = rng.standard_normal((2, 6, 8, 1)).astype(np.float32)
    mask = rng.standard_normal((2, 576, 6, 8)).astype(np.float32)
    up = droid_net.cvx_upsample(torch.from_numpy(data), torch.from_numpy(mask))
    np.savez_compressed(os.path.join(HERE, "cvx_upsample.npz"), data=data, mask=mask, up=up.numpy())
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()

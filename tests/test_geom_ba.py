"""The differentiable training-path BA (droid_mi355x.dense_ba: BA, MoBA, the
implicit-gradient LLT) vs the reference's own geom/ba.py (tests/golden/
geom_ba.npz, run by make_golden.py with an independent SE3 stand-in whose Exp
is a matrix exponential): poses, disparities and the gradients of a fixed
linear functional w.r.t. target, weight and eta - float64 on the CPU, float32
on the GPU."""
import os

import numpy as np
import pytest
import torch


def _run(z, dev, dtype):
    from droid_mi355x.dense_ba import BA, MoBA
    from droid_mi355x.lie import SE3
    T = lambda k: torch.from_numpy(z[k]).to(device=dev, dtype=dtype)
    ii, jj = torch.from_numpy(z["ii"]).to(dev), torch.from_numpy(z["jj"]).to(dev)
    Gs = SE3(T("poses"))
    target = T("target").requires_grad_()
    weight = T("weight").requires_grad_()
    eta = T("eta").requires_grad_()
    p1, d1 = BA(target, weight, eta, Gs, T("disps"), T("intrinsics"), ii, jj, fixedp=1)
    loss = (p1.data * T("c_pose")).sum() + (d1 * T("c_disp")).sum()
    gt, gw, ge = torch.autograd.grad(loss, [target, weight, eta])
    t2 = T("target").requires_grad_()
    p2 = MoBA(t2, T("weight"), T("eta"), Gs, T("disps"), T("intrinsics"), ii, jj, fixedp=1)
    g2, = torch.autograd.grad((p2.data * T("c_pose")).sum(), [t2])
    f = lambda t: t.detach().double().cpu().numpy()
    return dict(ba_poses=f(p1.data), ba_disps=f(d1), grad_target=f(gt), grad_weight=f(gw), grad_eta=f(ge),
                moba_poses=f(p2.data), moba_grad_target=f(g2))


def _check(z, got, rtol, atol):
    for k, v in got.items():
        ref = z[k]
        np.testing.assert_allclose(v, ref, rtol=rtol, atol=atol * max(1.0, np.abs(ref).max()), err_msg=k)


def test_geom_ba_matches_reference_cpu(golden_dir):
    z = np.load(os.path.join(golden_dir, "geom_ba.npz"))
    _check(z, _run(z, "cpu", torch.float64), rtol=1e-7, atol=1e-8)


@pytest.mark.gpu
def test_geom_ba_matches_reference_gpu(golden_dir):
    z = np.load(os.path.join(golden_dir, "geom_ba.npz"))
    _check(z, _run(z, "cuda:0", torch.float64), rtol=1e-7, atol=1e-8)
    _check(z, _run(z, "cuda:0", torch.float32), rtol=2e-3, atol=2e-3)

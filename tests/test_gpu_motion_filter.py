"""MotionFilter on the MI355X: the fused instance-norm kernel vs torch, the
channels-last fp16 encoders vs the reference BasicEncoder outputs
(tests/golden/encoders.npz) and MotionFilter.track vs the reference's own
track() on the same frames (tests/golden/motion_filter.npz: per-frame motion,
keyframe decisions, stored features)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fill import det_fill
from gpu_util import host

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("N,C,H,W", [(2, 32, 24, 40), (1, 64, 48, 64), (2, 128, 12, 16), (1, 256, 8, 8)])
def test_instance_norm_act(N, C, H, W):
    import droid_backends as nb
    g = torch.Generator(device=DEV).manual_seed(C + H)
    x = (torch.randn((N, C, H, W), generator=g, device=DEV) * 2 + 0.5).half().contiguous(memory_format=torch.channels_last)
    r = torch.randn((N, C, H, W), generator=g, device=DEV).half().contiguous(memory_format=torch.channels_last)
    n = F.instance_norm(x.float(), eps=1e-5).half().float()
    refs = {nb.NORM_RELU: torch.relu(n), nb.NORM_RES_RELU: torch.relu(r.float() + torch.relu(n)),
            nb.NORM_ADD_RELU: torch.relu(n + r.float()), nb.NORM_ONLY: n}
    for mode, ref in refs.items():
        out = nb.instance_norm_act_f16(x, mode, res=r)
        assert out.is_contiguous(memory_format=torch.channels_last)
        np.testing.assert_allclose(host(out.float()), host(ref), atol=4e-3, rtol=4e-3, err_msg="mode %d" % mode)
    # in place
    y = x.clone(memory_format=torch.channels_last)
    nb.instance_norm_act_f16(y, nb.NORM_RELU, out=y)
    np.testing.assert_allclose(host(y.float()), host(refs[nb.NORM_RELU]), atol=4e-3, rtol=4e-3)


def test_encoders_match_reference(golden_dir):
    """The fast path vs the reference fixture (fp32), judged against the drift
    the reference's own module shows under the autocast it runs in
    (motion_filter.py:31-40): fp16 convolutions through ~20 layers."""
    from droid_mi355x.extractor import BasicEncoder
    z = np.load(os.path.join(golden_dir, "encoders.npz"))
    x = torch.from_numpy(z["x"]).to(DEV)
    for name, dim, norm in (("fnet", 128, "instance"), ("cnet", 256, "none")):
        enc = BasicEncoder(output_dim=dim, norm_fn=norm).to(DEV)
        det_fill(enc)
        with torch.no_grad():
            out = enc(x)
            with torch.autocast("cuda", enabled=True):
                auto = enc.forward_reference(x.clone())
        assert out.dtype == torch.float16 and out.shape == z[name].shape
        ref = z[name]
        scale = np.abs(ref).max()
        e_fast = np.abs(host(out.float()) - ref)
        e_auto = np.abs(host(auto.float()) - ref)
        print("%s: |fast - fp32 ref| max %.4f mean %.5f; |autocast ref - fp32 ref| max %.4f mean %.5f (scale %.3f)"
              % (name, e_fast.max(), e_fast.mean(), e_auto.max(), e_auto.mean(), scale))
        assert e_fast.mean() < 1.5 * e_auto.mean() + 1e-3 * scale, name
        assert e_fast.max() < 2.5 * e_auto.max() + 2e-2 * scale, name


def test_motion_filter_track_matches_reference(golden_dir):
    from types import SimpleNamespace as NS
    from droid_mi355x import DroidNet, MotionFilter
    z = np.load(os.path.join(golden_dir, "motion_filter.npz"))
    net = DroidNet().to(DEV)
    det_fill(net)
    frames, intr = torch.from_numpy(z["frames"]), torch.from_numpy(z["intrinsics"])
    for tag, th in (("all", 0.0), ("none", float("inf"))):
        appended, feats, motion = [], [], []
        video = NS(counter=NS(value=0))

        def append(*item):
            appended.append(float(item[0]))
            if len(feats) < 3:
                feats.append((host(item[6].float()), host(item[7].float()), host(item[8].float())))
            video.counter.value += 1
        video.append = append
        f = MotionFilter(net, video, thresh=th, device=DEV)
        for k in range(len(frames)):
            f.track(float(k), frames[k][None], intrinsics=intr)
            if k > 0:
                motion.append(f.last_motion)
        np.testing.assert_array_equal(np.array(appended), z["appended_" + tag])
        np.testing.assert_allclose(np.array(motion), z["motion_" + tag], rtol=2e-3, atol=1e-4)
        if tag == "all":
            # the stored features vs the fixture, judged against the drift of the
            # reference-structured encoders under autocast on the same frame
            mean = torch.as_tensor([0.485, 0.456, 0.406], device=DEV)[:, None, None]
            std = torch.as_tensor([0.229, 0.224, 0.225], device=DEV)[:, None, None]
            with torch.no_grad(), torch.autocast("cuda", enabled=True):
                for q in range(3):
                    img = frames[q][None, None, [2, 1, 0]].to(DEV) / 255.0
                    img = (img - mean) / std
                    g_ref = net.fnet.forward_reference(img.clone())[0]
                    c = net.cnet.forward_reference(img.clone())[0]
                    n_ref, i_ref = torch.tanh(c[:, :128]), torch.relu(c[:, 128:])
                    if q == 0:   # the reference's first-frame quirk: net[0, 0], inp[0, 0] (channel 0)
                        n_ref, i_ref = n_ref[0, 0], i_ref[0, 0]
                    else:
                        n_ref, i_ref = n_ref[0], i_ref[0]
                    for nm, got, auto in zip(("gmap", "net", "inp"), feats[q], (g_ref, n_ref, i_ref)):
                        ref = z["%s%d" % (nm, q)]
                        e_fast = np.abs(got - ref)
                        e_auto = np.abs(host(auto.float()) - ref)
                        scale = max(1.0, np.abs(ref).max())
                        assert e_fast.mean() < 1.5 * e_auto.mean() + 1e-3 * scale, (nm, q, e_fast.mean(), e_auto.mean())
                        # (single outliers of two fp16 roundings paths differ more than their means)
                        assert e_fast.max() < 2.5 * e_auto.max() + 2e-2 * scale, (nm, q, e_fast.max(), e_auto.max())

"""MotionFilter encoders on CPU: the module tree matches the reference's
DroidNet parameter layout, and forward_reference (fp32) reproduces the
reference BasicEncoder outputs (tests/golden/encoders.npz, made by importing
modules/extractor.py)."""
import os

import numpy as np
import torch

from fill import det_fill


def test_droidnet_state_dict_layout(golden_dir):
    from droid_mi355x import DroidNet
    z = np.load(os.path.join(golden_dir, "encoders.npz"))
    sd = DroidNet().state_dict()
    assert list(sd.keys()) == list(z["droidnet_keys"])
    assert [",".join(map(str, v.shape)) for v in sd.values()] == list(z["droidnet_shapes"])


def test_basic_encoder_reference_path(golden_dir):
    from droid_mi355x.extractor import BasicEncoder
    z = np.load(os.path.join(golden_dir, "encoders.npz"))
    x = torch.from_numpy(z["x"])
    for name, dim, norm in (("fnet", 128, "instance"), ("cnet", 256, "none")):
        enc = BasicEncoder(output_dim=dim, norm_fn=norm)
        det_fill(enc)
        with torch.no_grad():
            out = enc(x)   # CPU input: the reference ops
        np.testing.assert_allclose(out.numpy(), z[name], rtol=1e-4, atol=1e-4, err_msg=name)

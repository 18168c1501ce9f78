"""DroidNet's module container (droid_net.py:146-150): fnet = BasicEncoder(128,
'instance'), cnet = BasicEncoder(256, 'none'), update = UpdateModule - the
attribute and parameter names of the reference, so its droid.pth state dict
loads unchanged - plus extract_features (:153-168)."""
import torch
import torch.nn as nn

from .extractor import BasicEncoder
from .update import UpdateModule


class DroidNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.fnet = BasicEncoder(output_dim=128, norm_fn="instance")
        self.cnet = BasicEncoder(output_dim=256, norm_fn="none")
        self.update = UpdateModule()

    def extract_features(self, images):
        """images (b, n, 3, H, W) uint8/float BGR -> fmaps, net, inp at 1/8."""
        images = images[:, :, [2, 1, 0]] / 255.0
        mean = torch.as_tensor([0.485, 0.456, 0.406], device=images.device)
        std = torch.as_tensor([0.229, 0.224, 0.225], device=images.device)
        images = images.sub_(mean[:, None, None]).div_(std[:, None, None])
        fmaps = self.fnet(images)
        net = self.cnet(images)
        net, inp = net.split([128, 128], dim=2)
        return fmaps, torch.tanh(net), torch.relu(inp)

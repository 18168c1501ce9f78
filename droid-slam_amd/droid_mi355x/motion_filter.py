"""MotionFilter (motion_filter.py:12-82): normalise each incoming frame,
extract its correlation features (fnet) and - for keyframes - its context
features (cnet), and keep the frame only if one update iteration against the
last keyframe predicts a mean flow above `thresh`.  The encoders run on the
MI355X path of droid_mi355x.extractor (channels-last fp16, fused instance
norm), the flow check on the library's correlation volume + lookup and the
UpdateModule; the control flow, the autocast scope and the DepthVideo.append
calls are the reference's.  lietorch-free: the identity pose is [0,0,0,0,0,0,1].
"""
import torch

from .corr import CorrBlock


def coords_grid(ht, wd, device):
    y, x = torch.meshgrid(torch.arange(ht, device=device, dtype=torch.float),
                          torch.arange(wd, device=device, dtype=torch.float), indexing="ij")
    return torch.stack([x, y], dim=-1)


class MotionFilter:
    """Keyframe gate in front of the frame graph: every frame gets its
    matching features; only a frame whose predicted flow against the last
    kept frame exceeds `thresh` pixels is appended to the DepthVideo (with its
    context features)."""

    def __init__(self, net, video, thresh=2.5, device="cuda:0"):
        self.cnet = net.cnet
        self.fnet = net.fnet
        self.update = net.update
        self.video = video
        self.thresh = thresh
        self.device = device
        self.count = 0
        self.MEAN = torch.as_tensor([0.485, 0.456, 0.406], device=self.device)[:, None, None]
        self.STDV = torch.as_tensor([0.229, 0.224, 0.225], device=self.device)[:, None, None]
        self.last_motion = None   # mean |delta| of the last check (for tests / logging)

    def _context_encoder(self, image):
        net, inp = self.cnet(image).split([128, 128], dim=2)
        return net.tanh().squeeze(0), inp.relu().squeeze(0)

    def _feature_encoder(self, image):
        return self.fnet(image).squeeze(0)

    @torch.no_grad()
    def track(self, tstamp, image, depth=None, intrinsics=None):
        """Encode one frame and decide whether it becomes a keyframe
        (reference control flow: motion_filter.py:47-82).  The first frame is
        always kept with the identity pose; later frames are kept when the mean
        |delta| of one update against the last keyframe's features is above
        `thresh`, otherwise only `count` grows."""
        Id = torch.as_tensor([0, 0, 0, 0, 0, 0, 1.0])
        ht = image.shape[-2] // 8
        wd = image.shape[-1] // 8
        with torch.autocast("cuda", enabled=True):
            inputs = image[None, :, [2, 1, 0]].to(self.device) / 255.0
            inputs = inputs.sub_(self.MEAN).div_(self.STDV)
            gmap = self._feature_encoder(inputs)
            if self.video.counter.value == 0:
                net, inp = self._context_encoder(inputs[:, [0]])
                self.net, self.inp, self.fmap = net, inp, gmap
                self.video.append(tstamp, image[0], Id, 1.0, depth, intrinsics / 8.0, gmap, net[0, 0], inp[0, 0])
            else:
                coords0 = coords_grid(ht, wd, device=self.device)[None, None]
                corr = CorrBlock(self.fmap[None, [0]], gmap[None, [0]])(coords0)
                _, delta, weight = self.update(self.net[None], self.inp[None], corr)
                self.last_motion = delta.norm(dim=-1).mean().item()
                if self.last_motion > self.thresh:
                    self.count = 0
                    net, inp = self._context_encoder(inputs[:, [0]])
                    self.net, self.inp, self.fmap = net, inp, gmap
                    self.video.append(tstamp, image[0], None, None, depth, intrinsics / 8.0, gmap, net[0], inp[0])
                else:
                    self.count += 1

"""Per-frame latency of the MotionFilter on the MI355X at 384x512: the feature
encoder (fnet, instance norm), the context encoder (cnet) and a full
track() call (fnet + the 1-edge correlation + update check, plus cnet when the
frame becomes a keyframe), fast path vs the reference-structured modules under
autocast.  Random frames, deterministic (untrained) weights."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
import json  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from droid_mi355x import DepthVideo, DroidNet, MotionFilter  # noqa: E402
from fill import det_fill  # noqa: E402

dev = torch.device("cuda:0")
H, W = 384, 512
net = DroidNet().to(dev)
det_fill(net)
x = torch.randn((1, 1, 3, H, W), device=dev)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


res = {}
with torch.no_grad():
    res["fnet_ms"] = timed(lambda: net.fnet(x))
    res["cnet_ms"] = timed(lambda: net.cnet(x))
    with torch.autocast("cuda", enabled=True):
        res["fnet_reference_autocast_ms"] = timed(lambda: net.fnet.forward_reference(x.clone()))
        res["cnet_reference_autocast_ms"] = timed(lambda: net.cnet.forward_reference(x.clone()))
rng = np.random.default_rng(0)
frames = torch.from_numpy(rng.integers(0, 255, (40, 3, H, W), dtype=np.uint8))
intr = torch.as_tensor([320.0, 320.0, W / 2, H / 2])
for tag, th in (("track_keyframe_ms", 0.0), ("track_skip_ms", float("inf"))):
    video = DepthVideo(image_size=(H, W), buffer=64, device="cuda:0")
    f = MotionFilter(net, video, thresh=th, device="cuda:0")
    ts = []
    for k in range(40):
        if video.counter.value >= 60:
            break
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        f.track(float(k), frames[k][None], intrinsics=intr)
        e.record()
        torch.cuda.synchronize()
        if k >= 3:
            ts.append(s.elapsed_time(e))
    res[tag] = float(np.median(ts))
res["image"] = [H, W]
print(json.dumps(res))

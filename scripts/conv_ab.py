"""A/B of the update operator's conv execution on MIOpen: layout x find mode.
Times UpdateModule.forward (fp16 autocast) at E edges of 48x64."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import torch

from droid_mi355x.update import UpdateModule

E = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
H, W = 48, 64
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = UpdateModule().to(dev).eval()
net = torch.tanh(torch.randn(1, E, 128, H, W, device=dev)).half()
inp = torch.relu(torch.randn(1, E, 128, H, W, device=dev)).half()
corr = torch.randn(1, E, 196, H, W, device=dev).half()
flow = torch.randn(1, E, 4, H, W, device=dev)
ii = torch.arange(E, device=dev) // 8
inv = ii.clone()
nu = int(E // 8)


def run(tag, cl, bench):
    torch.backends.cudnn.benchmark = bench
    mm = m.to(memory_format=torch.channels_last) if cl else m.to(memory_format=torch.contiguous_format)
    args = [net, inp, corr, flow]
    with torch.no_grad(), torch.autocast("cuda", enabled=True):
        t = time.time()
        mm(*args, ii, ii, inverse=inv, num_unique=nu)
        torch.cuda.synchronize()
        first = time.time() - t
        ts = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            mm(*args, ii, ii, inverse=inv, num_unique=nu)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
    print("%-28s first %.1fs  steady %.2f ms  (%.0f TFLOP/s)" % (tag, first, min(ts), 14.03e9 * E / (min(ts) * 1e-3) / 1e12),
          flush=True)


run("nchw, benchmark=False", False, False)
run("nchw, benchmark=True", False, True)
run("channels_last, bench=False", True, False)
run("channels_last, bench=True", True, True)

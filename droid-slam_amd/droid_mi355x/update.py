"""Update operator (mirror of droid_net.py:21-143, modules/gru.py, modules/clipping.py).

Module tree and parameter names are identical to the reference so a
`droid.pth` state dict (after droid.py:45-59's key fix-ups) loads unchanged.
The convolutions run on MIOpen through PyTorch (fp16 under autocast, as in
the reference); GraphAgg's scatter_mean takes a host-computed inverse index
so no device->host sync (torch.unique) is needed on the hot path.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

GRAD_CLIP = 0.01


class GradClip(torch.autograd.Function):
    """modules/clipping.py:7-18: identity forward; backward zeroes |g| > 0.01 and NaN."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        z = torch.zeros_like(g)
        g = torch.where(g.abs() > GRAD_CLIP, z, g)
        return torch.where(torch.isnan(g), z, g)


class GradientClip(nn.Module):
    def forward(self, x):
        return GradClip.apply(x)


class ConvGRU(nn.Module):
    """modules/gru.py:5-32 (gated conv GRU with a global-context branch)."""

    def __init__(self, h_planes=128, i_planes=128):
        super().__init__()
        self.do_checkpoint = False
        self.convz = nn.Conv2d(h_planes + i_planes, h_planes, 3, padding=1)
        self.convr = nn.Conv2d(h_planes + i_planes, h_planes, 3, padding=1)
        self.convq = nn.Conv2d(h_planes + i_planes, h_planes, 3, padding=1)
        self.w = nn.Conv2d(h_planes, h_planes, 1, padding=0)
        self.convz_glo = nn.Conv2d(h_planes, h_planes, 1, padding=0)
        self.convr_glo = nn.Conv2d(h_planes, h_planes, 1, padding=0)
        self.convq_glo = nn.Conv2d(h_planes, h_planes, 1, padding=0)

    def forward(self, net, *inputs):
        inp = torch.cat(inputs, dim=1)
        net_inp = torch.cat([net, inp], dim=1)
        b, c, h, w = net.shape
        glo = (torch.sigmoid(self.w(net)) * net).view(b, c, h * w).mean(-1).view(b, c, 1, 1)
        z = torch.sigmoid(self.convz(net_inp) + self.convz_glo(glo))
        r = torch.sigmoid(self.convr(net_inp) + self.convr_glo(glo))
        q = torch.tanh(self.convq(torch.cat([r * net, inp], dim=1)) + self.convq_glo(glo))
        return (1 - z) * net + z * q


def scatter_mean(src, index, dim, dim_size):
    """torch_scatter.scatter_mean restated (index_add mean)."""
    shape = list(src.shape)
    shape[dim] = dim_size
    out = torch.zeros(shape, dtype=src.dtype, device=src.device).index_add_(dim, index, src)
    cnt = torch.zeros(dim_size, dtype=src.dtype, device=src.device)
    cnt.index_add_(0, index, torch.ones(index.shape[0], dtype=src.dtype, device=src.device))
    view = [1] * src.dim()
    view[dim] = dim_size
    return out / cnt.clamp(min=1).view(view)


class GraphAgg(nn.Module):
    """droid_net.py:44-75: per-source-frame damping eta and upsampling mask."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(128, 128, 3, padding=1)
        self.conv2 = nn.Conv2d(128, 128, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.eta = nn.Sequential(nn.Conv2d(128, 1, 3, padding=1), GradientClip(), nn.Softplus())
        self.upmask = nn.Sequential(nn.Conv2d(128, 8 * 8 * 9, 1, padding=0))

    def forward(self, net, ii, inverse=None, num_unique=None):
        batch, num, ch, ht, wd = net.shape
        net = net.view(batch * num, ch, ht, wd)
        if inverse is None:
            uniq, inverse = torch.unique(ii, return_inverse=True)
            num_unique = uniq.shape[0]
        net = self.relu(self.conv1(net)).view(batch, num, 128, ht, wd)
        net = scatter_mean(net, inverse, 1, num_unique).view(-1, 128, ht, wd)
        net = self.relu(self.conv2(net))
        eta = self.eta(net).view(batch, -1, ht, wd)
        upmask = self.upmask(net).view(batch, -1, 8 * 8 * 9, ht, wd)
        return 0.01 * eta, upmask


class UpdateModule(nn.Module):
    """droid_net.py:78-143 (RAFT-SLAM update operator)."""

    def __init__(self):
        super().__init__()
        cor_planes = 4 * (2 * 3 + 1) ** 2
        self.corr_encoder = nn.Sequential(
            nn.Conv2d(cor_planes, 128, 1, padding=0), nn.ReLU(inplace=True),
            nn.Conv2d(128, 128, 3, padding=1), nn.ReLU(inplace=True))
        self.flow_encoder = nn.Sequential(
            nn.Conv2d(4, 128, 7, padding=3), nn.ReLU(inplace=True),
            nn.Conv2d(128, 64, 3, padding=1), nn.ReLU(inplace=True))
        self.weight = nn.Sequential(
            nn.Conv2d(128, 128, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(128, 2, 3, padding=1), GradientClip(), nn.Sigmoid())
        self.delta = nn.Sequential(
            nn.Conv2d(128, 128, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(128, 2, 3, padding=1), GradientClip())
        self.gru = ConvGRU(128, 128 + 128 + 64)
        self.agg = GraphAgg()

    def forward(self, net, inp, corr, flow=None, ii=None, jj=None, inverse=None, num_unique=None):
        batch, num, ch, ht, wd = net.shape
        if flow is None:
            flow = torch.zeros(batch, num, 4, ht, wd, device=net.device)
        out_dim = (batch, num, -1, ht, wd)
        net = net.view(batch * num, -1, ht, wd)
        inp = inp.view(batch * num, -1, ht, wd)
        corr = corr.view(batch * num, -1, ht, wd)
        flow = flow.view(batch * num, -1, ht, wd)
        corr = self.corr_encoder(corr)
        flow = self.flow_encoder(flow)
        net = self.gru(net, inp, corr, flow)
        delta = self.delta(net).view(*out_dim)
        weight = self.weight(net).view(*out_dim)
        delta = delta.permute(0, 1, 3, 4, 2)[..., :2].contiguous()
        weight = weight.permute(0, 1, 3, 4, 2)[..., :2].contiguous()
        net = net.view(*out_dim)
        if ii is None:
            return net, delta, weight
        eta, upmask = self.agg(net, ii.to(net.device), inverse, num_unique)
        return net, delta, weight, eta, upmask


def cvx_upsample(data, mask):
    """droid_net.py:21-35: convex 8x upsampling of a per-pixel field."""
    batch, ht, wd, dim = data.shape
    data = data.permute(0, 3, 1, 2)
    mask = torch.softmax(mask.view(batch, 1, 9, 8, 8, ht, wd), dim=2)
    up = F.unfold(data, [3, 3], padding=1).view(batch, dim, 9, 1, 1, ht, wd)
    up = torch.sum(mask * up, dim=2).permute(0, 4, 2, 5, 3, 1)
    return up.reshape(batch, 8 * ht, 8 * wd, dim)


def upsample_disp(disp, mask):
    """droid_net.py:37-41."""
    batch, num, ht, wd = disp.shape
    disp = disp.view(batch * num, ht, wd, 1)
    mask = mask.view(batch * num, -1, ht, wd)
    return cvx_upsample(disp, mask).view(batch, num, 8 * ht, 8 * wd)

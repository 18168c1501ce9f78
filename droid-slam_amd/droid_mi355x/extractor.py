"""MotionFilter feature encoders (modules/extractor.py:1-198, droid_net.py:149-150)
on the MI355X: the same module tree (parameter names match, so the
reference's droid.pth loads), run channels-last fp16 - the convolutions on
MIOpen through torch, every InstanceNorm2d together with the ReLU / residual
add around it in one hand-written pass pair (droid_instance_norm_act_f16,
csrc/norm_kernels.hip).  `forward` keeps the reference's signature and output
(b, n, C, H/8, W/8); `forward_reference` is the module run op by op as the
reference runs it (the parity bridge for the tests).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

import droid_backends

DIM = 32


def _norm(kind, planes):
    if kind == "group":
        return nn.GroupNorm(num_groups=planes // 8, num_channels=planes)
    if kind == "batch":
        return nn.BatchNorm2d(planes)
    if kind == "instance":
        return nn.InstanceNorm2d(planes)
    return nn.Sequential()


class ResidualBlock(nn.Module):
    """extractor.py:6-55 (3x3 conv - norm - ReLU twice, 1x1 strided shortcut)."""

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, planes)
        self.norm2 = _norm(norm_fn, planes)
        if stride != 1:
            self.norm3 = _norm(norm_fn, planes)
        self.downsample = None if stride == 1 else nn.Sequential(
            nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward_reference(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)

    def forward_fast(self, x):
        """channels_last fp16 in and out (instance or no norm)."""
        nb = droid_backends
        if self.norm_fn == "instance":
            y = nb.instance_norm_act_f16(_conv(self.conv1, x), nb.NORM_RELU)
            y2 = _conv(self.conv2, y)
            if self.downsample is None:
                return nb.instance_norm_act_f16(y2, nb.NORM_RES_RELU, res=x)           # relu(x + relu(n(y2)))
            y = nb.instance_norm_act_f16(y2, nb.NORM_RELU)
            return nb.instance_norm_act_f16(_conv(self.downsample[0], x), nb.NORM_ADD_RELU, res=y)
        y = torch.relu_(_conv(self.conv1, x))
        y = torch.relu_(_conv(self.conv2, y))
        if self.downsample is not None:
            x = _conv(self.downsample[0], x)
        return torch.relu_(x + y)


def _conv(conv, x):
    """nn.Conv2d on a channels_last fp16 map (MIOpen), fp16 weights as under
    autocast (cast once per parameter version)."""
    key = (conv.weight.data_ptr(), conv.weight._version,
           None if conv.bias is None else (conv.bias.data_ptr(), conv.bias._version))
    c = getattr(conv, "_f16", None)
    if c is None or c[0] != key:
        c = (key, conv.weight.detach().to(torch.float16).contiguous(memory_format=torch.channels_last),
             None if conv.bias is None else conv.bias.detach().to(torch.float16))
        conv._f16 = c
    y = F.conv2d(x, c[1], c[2], conv.stride, conv.padding)
    return y.contiguous(memory_format=torch.channels_last)


class BasicEncoder(nn.Module):
    """extractor.py:120-198 (multidim=False, as DroidNet builds it)."""

    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0, multidim=False):
        super().__init__()
        if multidim:
            raise NotImplementedError("BasicEncoder(multidim=True) is not used by DroidNet")
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, DIM) if norm_fn != "group" else nn.GroupNorm(num_groups=8, num_channels=DIM)
        self.conv1 = nn.Conv2d(3, DIM, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = DIM
        self.layer1 = self._make_layer(DIM, stride=1)
        self.layer2 = self._make_layer(2 * DIM, stride=2)
        self.layer3 = self._make_layer(4 * DIM, stride=2)
        self.conv2 = nn.Conv2d(4 * DIM, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim, stride=1):
        layers = (ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride),
                  ResidualBlock(dim, dim, self.norm_fn, stride=1))
        self.in_planes = dim
        return nn.Sequential(*layers)

    def forward_reference(self, x):
        b, n, c1, h1, w1 = x.shape
        x = x.view(b * n, c1, h1, w1)
        x = self.relu1(self.norm1(self.conv1(x)))
        for layer in (self.layer1, self.layer2, self.layer3):
            for blk in layer:
                x = blk.forward_reference(x)
        x = self.conv2(x)
        _, c2, h2, w2 = x.shape
        return x.view(b, n, c2, h2, w2)

    def forward(self, x):
        """(b, n, 3, H, W) -> (b, n, C, H/8, W/8) fp16: the MI355X path for the
        norms DroidNet uses (instance: fnet, none: cnet - no running statistics,
        so train and eval mode agree; the reference never applies its dropout).
        Training (gradients through the encoder) runs the reference ops."""
        if (self.norm_fn not in ("instance", "none") or not x.is_cuda
                or (torch.is_grad_enabled() and self.conv1.weight.requires_grad)):
            return self.forward_reference(x)
        b, n, c1, h1, w1 = x.shape
        x = x.reshape(b * n, c1, h1, w1).to(torch.float16).contiguous(memory_format=torch.channels_last)
        with torch.autocast("cuda", enabled=False):
            x = _conv(self.conv1, x)
            if self.norm_fn == "instance":
                x = droid_backends.instance_norm_act_f16(x, droid_backends.NORM_RELU)
            else:
                x = torch.relu_(x)
            for layer in (self.layer1, self.layer2, self.layer3):
                for blk in layer:
                    x = blk.forward_fast(x)
            x = _conv(self.conv2, x)
        _, c2, h2, w2 = x.shape
        return x.contiguous().view(b, n, c2, h2, w2)

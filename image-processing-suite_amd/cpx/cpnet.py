"""CPnet — the Cellpose (<= v3) residual U-Net: the architecture, its weights and the fp32 module.

Architecture restated from Cellpose's resnet_torch.CPnet (the model behind
``models.CellposeModel(model_type='nuclei')``, Cellpose_GPU_s3fs.py:28,108): nbase = [2, 32, 64,
128, 256], 3x3 convs, 4 BN-ReLU-conv per residual block (down path with 1x1 projection), global
style vector (mean-pool + L2-normalise) added through Linear layers in the up path, nearest x2
upsampling, 1x1 output head -> (dy, dx, cellprob).

This module is the network's definition, not the product forward: the pipeline runs it on
libcpx's native split-fp16 MFMA kernels at the fp32 network's accuracy (cpx.cpnet_x3, the
default "f16x3" precision); the eager fp32 module here is the named "fp32" variant (and the
per-FOV re-run when a split-fp16 activation overflows), the CPU reference of the tests and the
CPU baseline's network; the bf16 kernels (cpx.cpnet_fused) are a named variant off every default.

Weights: Cellpose's pretrained weights are a network fetch (unavailable offline), so the model is
built with a seeded random initialisation of this architecture or loaded from a local state_dict
(the bench uses cpx/weights/cpnet_nuclei_synth.pt, trained on the synthetic plates).  Eval-mode
BatchNorm is an affine per channel.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _bnconv(cin, cout, k, relu=True):
    layers = [nn.BatchNorm2d(cin, eps=1e-5, momentum=0.05)]
    if relu:
        layers.append(nn.ReLU(inplace=True))
    layers.append(nn.Conv2d(cin, cout, k, padding=k // 2))
    return nn.Sequential(*layers)


class ResDown(nn.Module):
    def __init__(self, cin, cout, k=3):
        super().__init__()
        self.proj = _bnconv(cin, cout, 1, relu=False)
        self.conv = nn.ModuleList([_bnconv(cin if t == 0 else cout, cout, k) for t in range(4)])

    def forward(self, x):
        x = self.proj(x) + self.conv[1](self.conv[0](x))
        return x + self.conv[3](self.conv[2](x))


class BnConvStyle(nn.Module):
    def __init__(self, cin, cout, style_ch, k=3):
        super().__init__()
        self.conv = _bnconv(cin, cout, k)
        self.full = nn.Linear(style_ch, cout)

    def forward(self, style, x, y=None):
        if y is not None:
            x = x + y
        return self.conv(x + self.full(style)[:, :, None, None])


class ResUp(nn.Module):
    def __init__(self, cin, cout, style_ch, k=3):
        super().__init__()
        self.conv0 = _bnconv(cin, cout, k)
        self.conv1 = BnConvStyle(cout, cout, style_ch, k)
        self.conv2 = BnConvStyle(cout, cout, style_ch, k)
        self.conv3 = BnConvStyle(cout, cout, style_ch, k)
        self.proj = _bnconv(cin, cout, 1, relu=False)

    def forward(self, x, y, style):
        x = self.proj(x) + self.conv1(style, self.conv0(x), y=y)
        return x + self.conv3(style, self.conv2(style, x))


class CPnet(nn.Module):
    def __init__(self, nbase=(2, 32, 64, 128, 256), nout=3, k=3, diam_mean=17.0):
        super().__init__()
        nbase = list(nbase)
        self.nbase = nbase
        self.down = nn.ModuleList([ResDown(nbase[n], nbase[n + 1], k) for n in range(len(nbase) - 1)])
        up = nbase[1:] + [nbase[-1]]
        self.up = nn.ModuleList([ResUp(up[n], up[n - 1], up[-1], k) for n in range(1, len(up))])
        self.output = _bnconv(up[0], nout, 1)
        self.diam_mean = diam_mean

    def forward(self, x):
        xd = []
        for n, blk in enumerate(self.down):
            xd.append(blk(x if n == 0 else F.max_pool2d(xd[n - 1], 2, 2)))
        style = F.avg_pool2d(xd[-1], kernel_size=xd[-1].shape[-2:]).flatten(1)
        style = style / torch.sum(style ** 2, dim=1, keepdim=True) ** 0.5
        x = self.up[-1](xd[-1], xd[-1], style)
        for n in range(len(self.up) - 2, -1, -1):
            x = F.interpolate(x, scale_factor=2, mode="nearest")
            x = self.up[n](x, xd[n], style)
        return self.output(x)


def build_cpnet(seed: int = 0, model: str = "nuclei", state_dict_path: str | None = None) -> CPnet:
    """Seeded random init of the architecture (BatchNorm running stats set to a plausible
    eval-mode affine), or a local state_dict if given."""
    diam = {"nuclei": 17.0, "cyto": 30.0, "cyto2": 30.0, "cyto3": 30.0}[model]
    g = torch.Generator().manual_seed(seed)
    net = CPnet(diam_mean=diam)
    if state_dict_path:
        net.load_state_dict(torch.load(state_dict_path, map_location="cpu", weights_only=True))
    else:
        with torch.no_grad():
            for m in net.modules():
                if isinstance(m, nn.Conv2d):
                    fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
                    m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.01)
                elif isinstance(m, nn.Linear):
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (1.0 / m.in_features) ** 0.5)
                    m.bias.zero_()
                elif isinstance(m, nn.BatchNorm2d):
                    m.running_mean.copy_(torch.randn(m.running_mean.shape, generator=g) * 0.1)
                    m.running_var.copy_(1.0 + torch.rand(m.running_var.shape, generator=g))
                    m.weight.copy_(1.0 + 0.1 * torch.randn(m.weight.shape, generator=g))
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
    return net.eval()


def count_flops(tile: int = 224, nbase=(2, 32, 64, 128, 256), nout=3) -> float:
    """Multiply-add FLOPs (2 per MAC) of one CPnet forward on a tile x tile input."""
    total = 0.0
    hw = tile * tile
    nb = list(nbase)
    for n in range(len(nb) - 1):
        cin, cout = nb[n], nb[n + 1]
        total += 2 * hw * cin * cout  # 1x1 proj
        total += 2 * hw * 9 * (cin * cout + 3 * cout * cout)
        if n < len(nb) - 2:
            hw //= 4
    up = nb[1:] + [nb[-1]]
    hw_levels = [tile * tile // (4 ** n) for n in range(len(up) - 1)]
    for n in range(1, len(up)):
        cin, cout = up[n], up[n - 1]
        hw = hw_levels[n - 1]
        total += 2 * hw * cin * cout + 2 * hw * 9 * (cin * cout + 3 * cout * cout)
    total += 2 * tile * tile * up[0] * nout
    return total

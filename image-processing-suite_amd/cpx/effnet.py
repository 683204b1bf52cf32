"""EfficientNetV2-L feature extractor — the embedding model of the reference's consumer
(Cellpose_GPU_s3fs.py:27,109-110,184-194: ``AutoModel.from_pretrained("timm/tf_efficientnetv2_l.in21k")``
run under fp16 autocast, ``outputs.pooler_output`` = 1280 features per image).

The weights are a remote download by model name, unavailable here, so the architecture is
restated (timm's ``tf_efficientnetv2_l``: TF 'same' padding, BatchNorm eps 1e-3, SiLU) and
built with a seeded initialisation or loaded from a local state_dict; parity with the trained
checkpoint is unpinned.  transformers' TimmWrapperModel builds the timm
model with num_classes=0, so ``pooler_output = forward_head(forward_features(x))`` = global
average pool of the 1280-channel head:

  stem   conv3x3/2 3->32, BN, SiLU
  stage  cn_r4_k3_s1_e1_c32 | er_r7_k3_s2_e4_c64 | er_r7_k3_s2_e4_c96 |
         ir_r10_k3_s2_e4_c192_se0.25 | ir_r19_k3_s1_e6_c224_se0.25 |
         ir_r25_k3_s2_e6_c384_se0.25 | ir_r7_k3_s1_e6_c640_se0.25
  head   conv1x1 640->1280, BN, SiLU, global average pool
  cn = conv3x3+BN+SiLU; er (fused MBConv) = conv3x3 expand +BN+SiLU, conv1x1 project +BN;
  ir (MBConv) = conv1x1 expand +BN+SiLU, depthwise 3x3 +BN+SiLU, squeeze-excite (reduce to
  in*0.25, SiLU, sigmoid gate), conv1x1 project +BN; residual when stride 1 and in == out.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

BN_EPS = 1e-3
FEATURE_LENGTH = 1280        # Cellpose_GPU_s3fs.py:29
INPUT_SIZE = 384             # pretrained_cfg input_size (3, 384, 384), crop_pct 1.0
MEAN = (0.5, 0.5, 0.5)
STD = (0.5, 0.5, 0.5)
ARCH = [  # (block type, repeats, stride, expansion, out channels, se ratio)
    ("cn", 4, 1, 1, 32, 0.0),
    ("er", 7, 2, 4, 64, 0.0),
    ("er", 7, 2, 4, 96, 0.0),
    ("ir", 10, 2, 4, 192, 0.25),
    ("ir", 19, 1, 6, 224, 0.25),
    ("ir", 25, 2, 6, 384, 0.25),
    ("ir", 7, 1, 6, 640, 0.25),
]


class Conv2dSame(nn.Conv2d):
    """TF 'same' padding: static (k-1)/2 for stride 1; for stride 2 the input is padded
    max((ceil(i/s)-1)*s + k - i, 0) with the extra pixel at the bottom / right."""

    def forward(self, x):
        s = self.stride[0]
        if s == 1:
            return F.conv2d(x, self.weight, self.bias, 1, self.kernel_size[0] // 2, 1, self.groups)
        ih, iw = x.shape[-2:]
        k = self.kernel_size[0]
        ph = max((math.ceil(ih / s) - 1) * s + k - ih, 0)
        pw = max((math.ceil(iw / s) - 1) * s + k - iw, 0)
        x = F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
        return F.conv2d(x, self.weight, self.bias, s, 0, 1, self.groups)


def _conv(cin, cout, k, s=1, groups=1, bias=False):
    return Conv2dSame(cin, cout, k, s, padding=0, groups=groups, bias=bias)


def _bn(c):
    return nn.BatchNorm2d(c, eps=BN_EPS)


class SqueezeExcite(nn.Module):
    def __init__(self, chs, rd):
        super().__init__()
        self.conv_reduce = nn.Conv2d(chs, rd, 1, bias=True)
        self.conv_expand = nn.Conv2d(rd, chs, 1, bias=True)

    def forward(self, x):
        s = x.mean((2, 3), keepdim=True)
        s = self.conv_expand(F.silu(self.conv_reduce(s)))
        return x * torch.sigmoid(s)


class ConvBnAct(nn.Module):  # 'cn'
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv = _conv(cin, cout, 3, stride)
        self.bn1 = _bn(cout)
        self.skip = stride == 1 and cin == cout

    def forward(self, x):
        y = F.silu(self.bn1(self.conv(x)))
        return y + x if self.skip else y


class EdgeResidual(nn.Module):  # 'er' (fused MBConv)
    def __init__(self, cin, cout, stride, exp):
        super().__init__()
        mid = cin * exp
        self.conv_exp = _conv(cin, mid, 3, stride)
        self.bn1 = _bn(mid)
        self.conv_pwl = _conv(mid, cout, 1)
        self.bn2 = _bn(cout)
        self.skip = stride == 1 and cin == cout

    def forward(self, x):
        y = F.silu(self.bn1(self.conv_exp(x)))
        y = self.bn2(self.conv_pwl(y))
        return y + x if self.skip else y


class InvertedResidual(nn.Module):  # 'ir' (MBConv)
    def __init__(self, cin, cout, stride, exp, se):
        super().__init__()
        mid = cin * exp
        self.conv_pw = _conv(cin, mid, 1)
        self.bn1 = _bn(mid)
        self.conv_dw = _conv(mid, mid, 3, stride, groups=mid)
        self.bn2 = _bn(mid)
        # timm: se_ratio / exp_ratio of the expanded channels = in_chs * se_ratio
        self.se = SqueezeExcite(mid, round(mid * se / exp)) if se else nn.Identity()
        self.conv_pwl = _conv(mid, cout, 1)
        self.bn3 = _bn(cout)
        self.skip = stride == 1 and cin == cout

    def forward(self, x):
        y = F.silu(self.bn1(self.conv_pw(x)))
        y = F.silu(self.bn2(self.conv_dw(y)))
        y = self.se(y)
        y = self.bn3(self.conv_pwl(y))
        return y + x if self.skip else y


class EfficientNetV2L(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv_stem = _conv(3, 32, 3, 2)
        self.bn1 = _bn(32)
        blocks = []
        cin = 32
        for bt, r, s, e, cout, se in ARCH:
            stage = []
            for i in range(r):
                st = s if i == 0 else 1
                if bt == "cn":
                    stage.append(ConvBnAct(cin, cout, st))
                elif bt == "er":
                    stage.append(EdgeResidual(cin, cout, st, e))
                else:
                    stage.append(InvertedResidual(cin, cout, st, e, se))
                cin = cout
            blocks.append(nn.Sequential(*stage))
        self.blocks = nn.Sequential(*blocks)
        self.conv_head = _conv(cin, FEATURE_LENGTH, 1)
        self.bn2 = _bn(FEATURE_LENGTH)

    def forward_features(self, x):
        x = F.silu(self.bn1(self.conv_stem(x)))
        x = self.blocks(x)
        return F.silu(self.bn2(self.conv_head(x)))

    def forward(self, x):
        """pixel_values [N, 3, 384, 384] -> pooler_output [N, 1280]."""
        return self.forward_features(x).mean((2, 3))


def build_effnet(seed: int = 0, state_dict_path: str | None = None) -> EfficientNetV2L:
    """Eval-mode model: seeded initialisation (He-normal convs, BN statistics drawn near
    identity so activations stay O(1) through the 99 blocks) or a local state_dict."""
    m = EfficientNetV2L()
    if state_dict_path:
        m.load_state_dict(torch.load(state_dict_path, map_location="cpu", weights_only=True))
    else:
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, nn.Conv2d):
                    fan = mod.in_channels // mod.groups * mod.kernel_size[0] * mod.kernel_size[1]
                    mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) * math.sqrt(1.0 / fan))
                    if mod.bias is not None:
                        mod.bias.copy_(0.1 * torch.randn(mod.bias.shape, generator=g))
                elif isinstance(mod, nn.BatchNorm2d):
                    c = mod.num_features
                    mod.weight.copy_(1.0 + 0.1 * torch.randn(c, generator=g))
                    mod.bias.copy_(0.1 * torch.randn(c, generator=g))
                    mod.running_mean.copy_(0.1 * torch.randn(c, generator=g))
                    mod.running_var.copy_(1.0 + 0.1 * torch.rand(c, generator=g))
            # residual branches start small (as a trained network's): the last BN of every
            # block with a skip scales its branch down
            for mod in m.modules():
                if isinstance(mod, (EdgeResidual, InvertedResidual)) and mod.skip:
                    last = mod.bn2 if isinstance(mod, EdgeResidual) else mod.bn3
                    last.weight.mul_(0.2)
    return m.eval()


def count_flops(size: int = INPUT_SIZE) -> int:
    """Multiply-add x 2 of the convolutions (+ SE GEMVs) for one size x size image."""
    m = EfficientNetV2L()
    total = 0
    h = size

    def conv_flops(conv, hin):
        s = conv.stride[0]
        ho = math.ceil(hin / s)
        k = conv.kernel_size[0]
        return 2 * ho * ho * conv.out_channels * (conv.in_channels // conv.groups) * k * k, ho

    f, h = conv_flops(m.conv_stem, h)
    total += f
    for stage in m.blocks:
        for b in stage:
            for name in ("conv", "conv_exp", "conv_pw", "conv_dw", "conv_pwl"):
                c = getattr(b, name, None)
                if c is not None:
                    f, h2 = conv_flops(c, h)
                    total += f
                    if c.stride[0] == 2:
                        h = h2
            if isinstance(getattr(b, "se", None), SqueezeExcite):
                total += 4 * b.se.conv_reduce.in_channels * b.se.conv_reduce.out_channels
    f, _ = conv_flops(m.conv_head, h)
    return total + f

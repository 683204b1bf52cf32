"""EfficientNetV2-L forward on libcpx's hand-written kernels (k_effnet.hip) — the embedding
model of Cellpose_GPU_s3fs.py:109-110,184-194 (timm tf_efficientnetv2_l under fp16 autocast,
``pooler_output``), replacing the PyTorch/MIOpen module on the GPU.

The architecture and its weights come from ``cpx.effnet.EfficientNetV2L`` (a seeded initialisation
or a local state_dict): every BatchNorm is folded to an fp32 per-channel scale / shift, 3x3 and
1x1 convolution weights are stored fp16 as [cout][ky][kx][cin], depthwise and squeeze-excite
weights fp32.  Activations are NHWC fp16 [N][H][W][C]; per block:

  cn   conv3x3 + BN + SiLU (+ input)                               cpx_effnet_conv
  er   conv3x3 expand + BN + SiLU -> conv1x1 + BN (+ input)        cpx_effnet_conv x 2
  ir   conv1x1 + BN + SiLU -> depthwise 3x3 + BN + SiLU (channel sums) -> SE gate ->
       conv1x1 on the gated input + BN (+ input)                   conv, dw, se, conv
  head conv1x1 640 -> 1280 + BN + SiLU -> global average pool     conv, pool
"""
from __future__ import annotations

import torch

from . import effnet
from ._lib import check
from .device import _ptr


def _fold(bn):
    """eval BatchNorm -> (scale, shift) fp32, computed in fp64."""
    g, b = bn.weight.detach().double(), bn.bias.detach().double()
    m, v = bn.running_mean.detach().double(), bn.running_var.detach().double()
    sc = g / torch.sqrt(v + bn.eps)
    return sc.float(), (b - m * sc).float()


def _w16(conv):
    """[cout][cin][kh][kw] -> fp16 [cout][kh][kw][cin]."""
    return conv.weight.detach().permute(0, 2, 3, 1).contiguous().half()


class EffNetHip:
    """Callable: fp16 [N, 3, H, W] pixel values (device) -> fp32 [N, 1280] pooler_output."""

    def __init__(self, model: "effnet.EfficientNetV2L", dev):
        self.dev, self.lib = dev, dev.lib
        td = dev.torch_device
        t = lambda x: x.to(td).contiguous()  # noqa: E731
        sc, sh = _fold(model.bn1)
        self.stem = dict(w=t(model.conv_stem.weight.detach().float().reshape(-1)), sc=t(sc), sh=t(sh))

        def conv(c, bn, act):
            s, h = _fold(bn)
            return dict(w=t(_w16(c)), sc=t(s), sh=t(h), cin=c.in_channels, cout=c.out_channels,
                        ks=c.kernel_size[0], stride=c.stride[0], act=int(act))

        self.blocks = []
        for stage in model.blocks:
            for b in stage:
                if isinstance(b, effnet.ConvBnAct):
                    self.blocks.append(dict(kind="cn", skip=b.skip, c=conv(b.conv, b.bn1, True)))
                elif isinstance(b, effnet.EdgeResidual):
                    self.blocks.append(dict(kind="er", skip=b.skip, exp=conv(b.conv_exp, b.bn1, True),
                                            pwl=conv(b.conv_pwl, b.bn2, False)))
                else:
                    s2, h2 = _fold(b.bn2)
                    mid = b.conv_dw.out_channels
                    se = b.se
                    self.blocks.append(dict(
                        kind="ir", skip=b.skip, pw=conv(b.conv_pw, b.bn1, True), pwl=conv(b.conv_pwl, b.bn3, False),
                        dw=dict(w=t(b.conv_dw.weight.detach().float().reshape(mid, 9)), sc=t(s2), sh=t(h2),
                                stride=b.conv_dw.stride[0], C=mid),
                        se=dict(wr=t(se.conv_reduce.weight.detach().float().reshape(se.conv_reduce.out_channels, mid)),
                                br=t(se.conv_reduce.bias.detach().float()),
                                we=t(se.conv_expand.weight.detach().float().reshape(mid, se.conv_expand.in_channels)),
                                be=t(se.conv_expand.bias.detach().float()), rd=se.conv_reduce.out_channels)))
        self.head = conv(model.conv_head, model.bn2, True)

    def _conv(self, x, p, res=None, gate=None):
        N, H, W, _ = x.shape
        Ho, Wo = -(-H // p["stride"]), -(-W // p["stride"])
        out = torch.empty((N, Ho, Wo, p["cout"]), dtype=torch.float16, device=x.device)
        check(self.lib.cpx_effnet_conv(self.dev.h, _ptr(x), N, H, W, p["cin"], p["cout"], p["ks"], p["stride"],
                                       _ptr(p["w"]), _ptr(p["sc"]), _ptr(p["sh"]), p["act"], _ptr(res), _ptr(gate),
                                       _ptr(out)), "cpx_effnet_conv")
        return out

    def _dw_se(self, x, dw, se):
        N, H, W, C = x.shape
        s = dw["stride"]
        Ho, Wo = -(-H // s), -(-W // s)
        nb = self.lib.cpx_effnet_dw_blocks(H, W, s)
        out = torch.empty((N, Ho, Wo, C), dtype=torch.float16, device=x.device)
        part = torch.empty((N, nb, C), dtype=torch.float32, device=x.device)
        check(self.lib.cpx_effnet_dw(self.dev.h, _ptr(x), N, H, W, C, s, _ptr(dw["w"]), _ptr(dw["sc"]),
                                     _ptr(dw["sh"]), _ptr(out), _ptr(part)), "cpx_effnet_dw")
        gate = torch.empty((N, C), dtype=torch.float32, device=x.device)
        check(self.lib.cpx_effnet_se(self.dev.h, _ptr(part), N, nb, Ho * Wo, C, se["rd"], _ptr(se["wr"]),
                                     _ptr(se["br"]), _ptr(se["we"]), _ptr(se["be"]), _ptr(gate)), "cpx_effnet_se")
        return out, gate

    @torch.no_grad()
    def __call__(self, x):
        assert x.dtype == torch.float16 and x.is_contiguous() and x.shape[1] == 3
        self.dev._bind_stream()
        N, _, H, W = x.shape
        h = torch.empty((N, -(-H // 2), -(-W // 2), 32), dtype=torch.float16, device=x.device)
        check(self.lib.cpx_effnet_stem(self.dev.h, _ptr(x), N, H, W, _ptr(self.stem["w"]), _ptr(self.stem["sc"]),
                                       _ptr(self.stem["sh"]), _ptr(h)), "cpx_effnet_stem")
        for b in self.blocks:
            res = h if b["skip"] else None
            if b["kind"] == "cn":
                h = self._conv(h, b["c"], res=res)
            elif b["kind"] == "er":
                h = self._conv(self._conv(h, b["exp"]), b["pwl"], res=res)
            else:
                d, gate = self._dw_se(self._conv(h, b["pw"]), b["dw"], b["se"])
                h = self._conv(d, b["pwl"], res=res, gate=gate)
        h = self._conv(h, self.head)
        N, Hh, Wh, C = h.shape
        out = torch.empty((N, C), dtype=torch.float32, device=x.device)
        check(self.lib.cpx_effnet_pool(self.dev.h, _ptr(h), N, Hh * Wh, C, _ptr(out)), "cpx_effnet_pool")
        return out

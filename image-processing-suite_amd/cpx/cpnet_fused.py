"""CPnet inference schedule: MIOpen convolutions + libcpx fused epilogues (bf16 NHWC).

Same network as cpx.cpnet.CPnet (Cellpose resnet_torch.CPnet, eval mode), re-scheduled for
MI355X: each 3x3 convolution runs without bias through MIOpen (implicit-GEMM on MFMA), and ONE
libcpx pass (cpx_cpnet_epilogue, k_cpnet.hip) applies bias + residual + style + the next
BatchNorm + ReLU, writing the residual stream and the next convolution's input together.
Further rewrites, all exact in real arithmetic:
  * the 1x1 projection's BatchNorm (no ReLU) is folded into its weights; its bias joins the
    bias of the convolution whose epilogue adds the projection;
  * nearest 2x upsampling commutes with per-pixel ops, so the up path's projection runs at the
    low resolution (read back nearest-upsampled by the epilogue) and the next block's
    BatchNorm+ReLU is applied before upsampling, written straight to the upsampled tensor;
  * the down path's 2x2 max-pool is fused with the next block's BatchNorm+ReLU
    (cpx_cpnet_pool).
Eager PyTorch runs ~9 full-tensor passes per convolution; this runs ~2.
"""
from __future__ import annotations

import ctypes as ct

import torch
import torch.nn.functional as F

from ._lib import check
from .cpnet import CPnet

CL = torch.channels_last


def _p(t):
    if t is None:
        return None
    assert t.is_cuda
    assert t.is_contiguous() or t.is_contiguous(memory_format=CL), "dense NCHW/NHWC tensor expected"
    return ct.c_void_p(t.data_ptr())


def _bn_affine(bn, dev):
    scale = bn.weight.detach().double().cpu() / torch.sqrt(bn.running_var.double().cpu() + bn.eps)
    shift = bn.bias.detach().double().cpu() - bn.running_mean.double().cpu() * scale
    return scale.float().to(dev).contiguous(), shift.float().to(dev).contiguous()


def _conv_w(conv, dev):
    return conv.weight.detach().to(dev, torch.bfloat16).contiguous(memory_format=CL)


def _bias(conv, dev):
    return conv.bias.detach().float().to(dev).contiguous()


def _fold_proj(seq, dev):
    """BatchNorm (no ReLU) -> 1x1 conv  ==  1x1 conv with w * scale[in], b + w @ shift."""
    bn, conv = seq[0], seq[-1]
    scale, shift = _bn_affine(bn, "cpu")
    w = conv.weight.detach().double().cpu()[:, :, 0, 0]
    wf = (w * scale.double()[None, :])
    bf = conv.bias.detach().double().cpu() + w @ shift.double()
    wt = wf[:, :, None, None].to(dev, torch.bfloat16).contiguous(memory_format=CL)
    return wt, bf.float().to(dev)


class FusedCPnet:
    def __init__(self, net: CPnet, dev):
        self.dev = dev
        self.lib = dev.lib
        td = dev.torch_device
        net = net.float().eval()
        self.down = []
        for blk in net.down:
            wp, bp = _fold_proj(blk.proj, td)
            d = dict(wp=wp,
                     bn=[_bn_affine(blk.conv[t][0], td) for t in range(4)],
                     w=[_conv_w(blk.conv[t][-1], td) for t in range(4)],
                     b=[_bias(blk.conv[t][-1], td) for t in range(4)])
            d["b1p"] = (d["b"][1] + bp).contiguous()
            self.down.append(d)
        self.up = []
        for blk in net.up:
            wp, bp = _fold_proj(blk.proj, td)
            convs = [blk.conv0, blk.conv1.conv, blk.conv2.conv, blk.conv3.conv]
            u = dict(wp=wp,
                     bn=[_bn_affine(c[0], td) for c in convs],
                     w=[_conv_w(c[-1], td) for c in convs],
                     b=[_bias(c[-1], td) for c in convs],
                     full=[(m.full.weight.detach().float().to(td), m.full.bias.detach().float().to(td))
                           for m in (blk.conv1, blk.conv2, blk.conv3)])
            u["b1p"] = (u["b"][1] + bp).contiguous()
            self.up.append(u)
        self.bn_out = _bn_affine(net.output[0], td)
        self.w_out = _conv_w(net.output[-1], td)
        self.b_out = net.output[-1].bias.detach().to(td, torch.bfloat16)

    # -- libcpx passes -------------------------------------------------------------------------
    def _epi(self, conv, bias, res=None, res_up=False, style=None, bn=None, relu=True,
             y=False, z=True, z_up=False):
        N, C, H, W = conv.shape
        assert conv.is_contiguous(memory_format=CL), "epilogue input must be NHWC"
        yo = torch.empty_like(conv, memory_format=CL) if y else None
        zo = None
        if z:
            zo = (torch.empty((N, C, 2 * H, 2 * W), dtype=conv.dtype, device=conv.device,
                              memory_format=CL) if z_up else torch.empty_like(conv, memory_format=CL))
        scale, shift = bn if bn is not None else (None, None)
        check(self.lib.cpx_cpnet_epilogue(self.dev.h, _p(conv), _p(bias), _p(res), int(res_up),
                                          _p(style), _p(scale), _p(shift), int(relu), N, H, W, C,
                                          _p(yo), _p(zo), int(z_up)), "cpx_cpnet_epilogue")
        return yo, zo

    def _pool(self, x, bn):
        N, C, H, W = x.shape
        xo = torch.empty((N, C, H // 2, W // 2), dtype=x.dtype, device=x.device, memory_format=CL)
        zo = torch.empty_like(xo, memory_format=CL)
        scale, shift = bn
        check(self.lib.cpx_cpnet_pool(self.dev.h, _p(x), _p(scale), _p(shift), 1, N, H // 2, W // 2,
                                      C, _p(xo), _p(zo)), "cpx_cpnet_pool")
        return xo, zo

    # -- forward -------------------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, x):
        """x: [N, 2, H, W] bf16 channels_last (H, W multiples of 16) -> [N, 3, H, W] bf16 NHWC."""
        self.dev._bind_stream()
        assert x.is_contiguous(memory_format=CL)
        xd = []
        zu = None
        for n, d in enumerate(self.down):
            if n == 0:
                xin = x
                _, z0 = self._epi(x, None, bn=d["bn"][0])
            else:
                xin, z0 = self._pool(xd[-1], d["bn"][0])
            p = F.conv2d(xin, d["wp"])
            h = F.conv2d(z0, d["w"][0], padding=1)
            _, z = self._epi(h, d["b"][0], bn=d["bn"][1])
            h = F.conv2d(z, d["w"][1], padding=1)
            x1, z = self._epi(h, d["b1p"], res=p, bn=d["bn"][2], y=True)
            h = F.conv2d(z, d["w"][2], padding=1)
            _, z = self._epi(h, d["b"][2], bn=d["bn"][3])
            h = F.conv2d(z, d["w"][3], padding=1)
            if n < len(self.down) - 1:
                xo, _ = self._epi(h, d["b"][3], res=x1, y=True, z=False)
            else:  # deepest level also feeds the first up block's BatchNorm+ReLU
                xo, zu = self._epi(h, d["b"][3], res=x1, bn=self.up[-1]["bn"][0], y=True)
            xd.append(xo)
        style = xd[-1].float().mean(dim=(2, 3))
        style = style / torch.sum(style ** 2, dim=1, keepdim=True) ** 0.5
        x_small, z0 = xd[-1], zu
        out_in = None
        for n in range(len(self.up) - 1, -1, -1):
            u = self.up[n]
            s = [(style @ w.t() + b).contiguous() for (w, b) in u["full"]]
            p = F.conv2d(x_small, u["wp"])
            h = F.conv2d(z0, u["w"][0], padding=1)
            _, z = self._epi(h, u["b"][0], res=xd[n], style=s[0], bn=u["bn"][1])
            h = F.conv2d(z, u["w"][1], padding=1)
            x1, z = self._epi(h, u["b1p"], res=p, res_up=(n < len(self.up) - 1), style=s[1],
                              bn=u["bn"][2], y=True)
            h = F.conv2d(z, u["w"][2], padding=1)
            _, z = self._epi(h, u["b"][2], style=s[2], bn=u["bn"][3])
            h = F.conv2d(z, u["w"][3], padding=1)
            if n > 0:
                x_small, z0 = self._epi(h, u["b"][3], res=x1, bn=self.up[n - 1]["bn"][0], y=True,
                                        z_up=True)
            else:
                _, out_in = self._epi(h, u["b"][3], res=x1, bn=self.bn_out)
        return F.conv2d(out_in, self.w_out, self.b_out)

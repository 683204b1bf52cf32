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
Every 3x3 convolution with 32..256 channels runs as ONE native launch (cpx_cpnet_conv3x3,
k_conv.hip: MFMA implicit GEMM with the epilogue applied to the fp32 accumulators); the stem
(input BatchNorm+ReLU, 2-channel 3x3 convolution + epilogue and the first 1x1 projection) is
one native pass (cpx_cpnet_stem) and the output 1x1 convolution runs in the last 3x3
convolution's epilogue (cpx_cpnet_conv3x3_head); only the inner blocks' 1x1 projections stay on
MIOpen.  Eager PyTorch runs ~9 full-tensor passes per convolution; this runs one.
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


def _pack3x3(lib, w, dev):
    """[cout][cin][3][3] -> the cpx_cpnet_conv3x3 layout [cout/bn][cin/ck][ky][kx][bn][ck] bf16,
    or None when the native kernel has no instance for (cin, cout)."""
    cout, cin = w.shape[0], w.shape[1]
    bn, ck = ct.c_int(), ct.c_int()
    if lib is None or lib.cpx_cpnet_conv_cfg(cin, cout, ct.byref(bn), ct.byref(ck)) != 0:
        return None
    bn, ck = bn.value, ck.value
    t = w.detach().float().cpu().reshape(cout // bn, bn, cin // ck, ck, 3, 3)
    t = t.permute(0, 2, 4, 5, 1, 3).contiguous()
    return t.to(dev, torch.bfloat16).contiguous()


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
    def __init__(self, net: CPnet, dev, native_conv: bool = True):
        self.dev = dev
        self.lib = dev.lib
        td = dev.torch_device
        net = net.float().eval()
        lib = self.lib if native_conv else None
        self.down = []
        for blk in net.down:
            wp, bp = _fold_proj(blk.proj, td)
            d = dict(wp=wp,
                     bn=[_bn_affine(blk.conv[t][0], td) for t in range(4)],
                     w=[_conv_w(blk.conv[t][-1], td) for t in range(4)],
                     b=[_bias(blk.conv[t][-1], td) for t in range(4)],
                     pk=[_pack3x3(lib, blk.conv[t][-1].weight, td) for t in range(4)])
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
                     pk=[_pack3x3(lib, c[-1].weight, td) for c in convs],
                     full=[(m.full.weight.detach().float().to(td), m.full.bias.detach().float().to(td))
                           for m in (blk.conv1, blk.conv2, blk.conv3)])
            u["b1p"] = (u["b"][1] + bp).contiguous()
            self.up.append(u)
        self.bn_out = _bn_affine(net.output[0], td)
        self.w_out = _conv_w(net.output[-1], td)
        self.b_out = net.output[-1].bias.detach().to(td, torch.bfloat16)
        # native stem (input BN+ReLU, 3x3 2->32 conv + epilogue, 1x1 projection in one pass) and
        # output head (1x1 32->nout fused into the last conv's epilogue); operands are the
        # bf16-rounded weights the MIOpen path uses, in fp32
        d0 = self.down[0]
        self.native = lib is not None and d0["w"][0].shape[1] == 2 and self.up[0]["pk"][3] is not None
        if self.native:
            self.stem_w = d0["w"][0].float().contiguous()                      # [32][2][3][3]
            self.stem_wp = d0["wp"].float().reshape(d0["wp"].shape[0], -1).contiguous()  # [32][2]
            self.head_w = self.w_out.float().reshape(self.w_out.shape[0], -1).contiguous()  # [nout][32]
            self.head_b = self.b_out.float().contiguous()

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

    def _conv(self, x, blk, i, bias, res=None, res_up=False, style=None, bn=None, relu=True,
              y=False, z=True, z_up=False):
        """3x3 conv i of block blk + fused epilogue: one native MFMA launch when packed weights
        exist, else MIOpen + cpx_cpnet_epilogue."""
        pk = blk["pk"][i]
        if pk is None:
            return self._epi(F.conv2d(x, blk["w"][i], padding=1), bias, res=res, res_up=res_up,
                             style=style, bn=bn, relu=relu, y=y, z=z, z_up=z_up)
        N, Cin, H, W = x.shape
        Cout = blk["w"][i].shape[0]
        assert x.is_contiguous(memory_format=CL)
        yo = torch.empty((N, Cout, H, W), dtype=x.dtype, device=x.device, memory_format=CL) if y else None
        zo = None
        if z:
            zs = (N, Cout, 2 * H, 2 * W) if z_up else (N, Cout, H, W)
            zo = torch.empty(zs, dtype=x.dtype, device=x.device, memory_format=CL)
        scale, shift = bn if bn is not None else (None, None)
        check(self.lib.cpx_cpnet_conv3x3(self.dev.h, _p(x), N, H, W, Cin, Cout, _p(pk), _p(bias),
                                         _p(res), int(res_up), _p(style), _p(scale), _p(shift),
                                         int(relu), _p(yo), _p(zo), int(z_up)), "cpx_cpnet_conv3x3")
        return yo, zo

    def _pool(self, x, bn):
        N, C, H, W = x.shape
        xo = torch.empty((N, C, H // 2, W // 2), dtype=x.dtype, device=x.device, memory_format=CL)
        zo = torch.empty_like(xo, memory_format=CL)
        scale, shift = bn
        check(self.lib.cpx_cpnet_pool(self.dev.h, _p(x), _p(scale), _p(shift), 1, N, H // 2, W // 2,
                                      C, _p(xo), _p(zo)), "cpx_cpnet_pool")
        return xo, zo

    def _stem(self, x, d):
        N, _, H, W = x.shape
        p = torch.empty((N, 32, H, W), dtype=x.dtype, device=x.device, memory_format=CL)
        z = torch.empty_like(p, memory_format=CL)
        (s0, h0), (s1, h1) = d["bn"][0], d["bn"][1]
        check(self.lib.cpx_cpnet_stem(self.dev.h, _p(x), N, H, W, _p(s0), _p(h0), _p(self.stem_w),
                                      _p(d["b"][0]), _p(s1), _p(h1), _p(self.stem_wp), _p(p), _p(z)),
              "cpx_cpnet_stem")
        return p, z

    def _head(self, z, u, x1):
        """last up conv + output BatchNorm/ReLU + output 1x1 conv in one native launch."""
        N, Cin, H, W = z.shape
        nout = self.head_w.shape[0]
        out = torch.empty((N, nout, H, W), dtype=z.dtype, device=z.device, memory_format=CL)
        scale, shift = self.bn_out
        check(self.lib.cpx_cpnet_conv3x3_head(self.dev.h, _p(z), N, H, W, Cin, u["w"][3].shape[0],
                                              _p(u["pk"][3]), _p(u["b"][3]), _p(x1), 0, None,
                                              _p(scale), _p(shift), 1, None, _p(self.head_w),
                                              _p(self.head_b), nout, _p(out)), "cpx_cpnet_conv3x3_head")
        return out

    @staticmethod
    def _proj(x, w):
        """1x1 projection of an NHWC (channels_last) tensor as one GEMM [pixels, cin] x [cin, cout]
        (hipBLASLt, fixed reduction order).  MIOpen's fast 1x1 solvers split K with atomic
        accumulation, which makes the bf16 outputs — and so the masks — differ run to run."""
        N, C, H, W = x.shape
        y = torch.matmul(x.permute(0, 2, 3, 1).reshape(-1, C), w.reshape(w.shape[0], C).t())
        return y.view(N, H, W, -1).permute(0, 3, 1, 2)

    # -- forward -------------------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, x):
        """x: [N, 2, H, W] bf16 channels_last (H, W multiples of 16) -> [N, 3, H, W] bf16 NHWC."""
        self.dev._bind_stream()
        assert x.is_contiguous(memory_format=CL)
        xd = []
        zu = None
        for n, d in enumerate(self.down):
            if n == 0 and self.native:
                p, z = self._stem(x, d)
            else:
                if n == 0:
                    xin = x
                    _, z0 = self._epi(x, None, bn=d["bn"][0])
                else:
                    xin, z0 = self._pool(xd[-1], d["bn"][0])
                p = self._proj(xin, d["wp"])
                _, z = self._conv(z0, d, 0, d["b"][0], bn=d["bn"][1])
            x1, z = self._conv(z, d, 1, d["b1p"], res=p, bn=d["bn"][2], y=True)
            _, z = self._conv(z, d, 2, d["b"][2], bn=d["bn"][3])
            if n < len(self.down) - 1:
                xo, _ = self._conv(z, d, 3, d["b"][3], res=x1, y=True, z=False)
            else:  # deepest level also feeds the first up block's BatchNorm+ReLU
                xo, zu = self._conv(z, d, 3, d["b"][3], res=x1, bn=self.up[-1]["bn"][0], y=True)
            xd.append(xo)
        style = xd[-1].float().mean(dim=(2, 3))
        style = style / torch.sum(style ** 2, dim=1, keepdim=True) ** 0.5
        x_small, z0 = xd[-1], zu
        out_in = None
        for n in range(len(self.up) - 1, -1, -1):
            u = self.up[n]
            s = [(style @ w.t() + b).contiguous() for (w, b) in u["full"]]
            p = self._proj(x_small, u["wp"])
            _, z = self._conv(z0, u, 0, u["b"][0], res=xd[n], style=s[0], bn=u["bn"][1])
            x1, z = self._conv(z, u, 1, u["b1p"], res=p, res_up=(n < len(self.up) - 1), style=s[1],
                               bn=u["bn"][2], y=True)
            _, z = self._conv(z, u, 2, u["b"][2], style=s[2], bn=u["bn"][3])
            if n > 0:
                x_small, z0 = self._conv(z, u, 3, u["b"][3], res=x1, bn=self.up[n - 1]["bn"][0],
                                         y=True, z_up=True)
            elif self.native:
                return self._head(z, u, x1)
            else:
                _, out_in = self._conv(z, u, 3, u["b"][3], res=x1, bn=self.bn_out)
        return F.conv2d(out_in, self.w_out, self.b_out)

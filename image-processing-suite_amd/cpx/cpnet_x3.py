"""CPnet forward at the reference's precision on the fp16 matrix cores ("f16x3").

The reference runs Cellpose's U-Net in fp32 (CellposeModel(gpu, model_type='nuclei') without
half precision, Cellpose_GPU_s3fs.py:108,143); the masks and object IDs that north_star asks to
reproduce depend on the flows to fp32 rounding (a bf16 network moves mask boundaries and IDs:
DESIGN.md §6).  This schedule is FusedCPnet's (cpx.cpnet_fused) on split activations: every
tensor between two kernels holds hi = f16(a) and lo = f16((a - hi) * 2^11) per value (libcpx
"split" layout, include/cpx.h), every weight is split the same way on the host, and each
product is formed as wh*xh + (wh*xl + wl*xh) * 2^-11 with fp32 accumulation — three fp16 MFMAs
per 16 channels, ~2^-22 relative per operand.  Everything is native libcpx
(k_conv_x3.hip): the stem, the 3x3 convolutions with their fused epilogues, the 1x1 block
projections (BatchNorm folded), the max-pools, the style vector with the up path's Linear
layers, and the fp32 output head; no PyTorch compute.
"""
from __future__ import annotations

import ctypes as ct

import numpy as np
import torch

from ._lib import check
from .cpnet import CPnet

# The network's build choices (module constants: the constructor's `variant` / `zvariant`
# arguments and the tests select the others):
X3_VARIANT = 0
# the convolutions that write only the next input z (no residual stream y) run as variant 3 at the
# 112^2 and deeper levels (BM 64: two channel slices per wave, one slab buffer): 5-12 % faster
# there, slower where the epilogue also stores y (tools/conv_bench_x3.py, gpurun_out/r05c);
# bit-identical outputs.  -1 keeps every convolution at X3_VARIANT
X3_ZVARIANT = 3
# each down block's last convolution also max-pools its output for the next block (the pooled
# tensor and its BatchNorm+ReLU from the staged tile: no read of y back); False keeps the
# separate pool kernel
X3_POOL_FUSE = True
# fold each down block's (and the deepest up block's) 1x1 residual projection into the block's
# second 3x3 convolution (cpx_cpnet_x3_conv_proj); False keeps the separate 1x1 pass
X3_FOLD = True


def split_f16(w: np.ndarray):
    """fp32 array -> (hi, lo) float16 with w ~= hi + lo * 2^-11 (hi, lo round to nearest)."""
    w = np.asarray(w, np.float32)
    if not np.all(np.abs(w) < 65504.0):
        raise ValueError("weights outside the fp16 range cannot be split")
    hi = w.astype(np.float16)
    lo = ((w - hi.astype(np.float32)) * np.float32(2048.0)).astype(np.float16)
    return hi, lo


def join_f16(hi: np.ndarray, lo: np.ndarray) -> np.ndarray:
    return (hi.astype(np.float32) + lo.astype(np.float32) * np.float32(1.0 / 2048.0)).astype(np.float32)


def pack_conv(w: np.ndarray, bm: int) -> np.ndarray:
    """[cout][cin][ks][ks] fp32 -> split [cout/bm][cin/16][ky][kx][bm][hi|lo][16] float16."""
    cout, cin, ks, _ = w.shape
    hi, lo = split_f16(w)
    parts = []
    for a in (hi, lo):
        t = a.reshape(cout // bm, bm, cin // 16, 16, ks, ks).transpose(0, 2, 4, 5, 1, 3)
        parts.append(t)
    return np.ascontiguousarray(np.stack(parts, axis=-2))  # [..., bm, 2, 16]


def to_split(x: np.ndarray) -> np.ndarray:
    """fp32 NHWC [..., C] -> split layout as float16 [..., C/16, 2, 16] (test helper)."""
    hi, lo = split_f16(x)
    s = x.shape[:-1] + (x.shape[-1] // 16, 16)
    return np.ascontiguousarray(np.stack([hi.reshape(s), lo.reshape(s)], axis=-2))


def from_split(t: np.ndarray) -> np.ndarray:
    """split float16 [..., C/16, 2, 16] (or its raw [..., C] int32 view) -> fp32 [..., C]."""
    if t.dtype != np.float16:
        t = t.view(np.float16)
        t = t.reshape(t.shape[:-1] + (t.shape[-1] // 32, 2, 16))
    v = join_f16(t[..., 0, :], t[..., 1, :])
    return v.reshape(v.shape[:-2] + (-1,))


def _bn_affine(bn):
    scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.double() + bn.eps)
    shift = bn.bias.detach().double() - bn.running_mean.double() * scale
    return scale.float(), shift.float()


def _fold_proj(seq):
    """BatchNorm (no ReLU) -> 1x1 conv  ==  1x1 conv with w * scale[in], b + w @ shift (fp64)."""
    bn, conv = seq[0], seq[-1]
    scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.double() + bn.eps)
    shift = bn.bias.detach().double() - bn.running_mean.double() * scale
    w = conv.weight.detach().double()[:, :, 0, 0]
    return (w * scale[None, :]).float()[:, :, None, None], (conv.bias.detach().double() + w @ shift).float()


def _p(t):
    return None if t is None else ct.c_void_p(t.data_ptr())


class FusedCPnetX3:
    """Native split-fp16 CPnet forward: __call__(x fp32 [N, by, bx, 2] NHWC) -> fp32 [N, by, bx, 3]."""

    def __init__(self, net: CPnet, dev, variant: int | None = None, zvariant: int | None = None):
        self.dev = dev
        self.lib = dev.lib
        self.variant = X3_VARIANT if variant is None else int(variant)
        td = dev.torch_device
        self.td = td
        net = net.float().eval().cpu()
        if list(net.nbase) != [2, 32, 64, 128, 256]:
            raise ValueError("FusedCPnetX3: the native kernels cover nbase (2, 32, 64, 128, 256)")

        def dv(t):
            return t.detach().float().contiguous().to(td)

        def conv_pack(w, ks, cfg_cin=None, variant=None):
            """pack for the tile configuration of a ks x ks conv of cfg_cin (default: w's own
            input channels) -> w's output channels, in `variant` (default self.variant)"""
            cout, cin = w.shape[0], w.shape[1]
            bm = ct.c_int()
            check(self.lib.cpx_cpnet_x3_cfg(ks, cin if cfg_cin is None else cfg_cin, cout,
                                            self.variant if variant is None else variant,
                                            ct.byref(bm)), "cpx_cpnet_x3_cfg")
            return torch.from_numpy(pack_conv(w.detach().float().numpy(), bm.value)).to(td)

        # z-only convolutions (each block's conv0 and conv2) in X3_ZVARIANT when the default is 0
        zvar = X3_ZVARIANT if zvariant is None else int(zvariant)
        zv = zvar if (self.variant == 0 and zvar >= 0) else self.variant

        def zconv(w):
            """(packed weights, variant) of a z-only 3x3 convolution"""
            v = zv if w.shape[0] >= 64 else self.variant  # the 224^2 level keeps its kernels
            return (conv_pack(w, 3, variant=v), v)

        # the folded projections exist for variant 0's tile configurations
        self.fold = X3_FOLD and self.variant != 1

        self.down = []
        for blk in net.down:
            wp, bp = _fold_proj(blk.proj)
            bns = [_bn_affine(blk.conv[t][0]) for t in range(4)]
            b = [blk.conv[t][-1].bias.detach().float() for t in range(4)]
            cout_b = blk.conv[0][-1].out_channels
            d = dict(bn=[(dv(s), dv(h)) for s, h in bns], b=[dv(x) for x in b], b1p=dv(b[1] + bp),
                     pk=[None if t == 0 and blk is net.down[0] else
                         (zconv(blk.conv[t][-1].weight) if t in (0, 2) else conv_pack(blk.conv[t][-1].weight, 3))
                         for t in range(4)],
                     wp=None if blk is net.down[0] else conv_pack(wp, 1), cout=cout_b,
                     # the projection packed as extra one-tap slabs of the block's second conv
                     wpf=None if blk is net.down[0] or not self.fold else conv_pack(wp, 3, cfg_cin=cout_b))
            if blk is net.down[0]:
                d["stem_w"] = dv(blk.conv[0][-1].weight.reshape(32, 18))
                d["stem_wp"] = dv(wp.reshape(32, 2))
            self.down.append(d)
        # style Linear layers of the up path, concatenated: rows [J][256]
        lin_w, lin_b, self.style_off = [], [], []
        off = 0
        for blk in net.up:
            offs = []
            for m in (blk.conv1, blk.conv2, blk.conv3):
                lin_w.append(m.full.weight.detach().float())
                lin_b.append(m.full.bias.detach().float())
                offs.append(off)
                off += m.full.out_features
            self.style_off.append(offs)
        self.J = off
        self.lin_w = dv(torch.cat(lin_w, 0))
        self.lin_b = dv(torch.cat(lin_b, 0))
        self.up = []
        for blk in net.up:
            wp, bp = _fold_proj(blk.proj)
            convs = [blk.conv0, blk.conv1.conv, blk.conv2.conv, blk.conv3.conv]
            bns = [_bn_affine(c[0]) for c in convs]
            b = [c[-1].bias.detach().float() for c in convs]
            cout_b = convs[0][-1].out_channels
            self.up.append(dict(bn=[(dv(s), dv(h)) for s, h in bns], b=[dv(x) for x in b], b1p=dv(b[1] + bp),
                                pk=[zconv(c[-1].weight) if t in (0, 2) else conv_pack(c[-1].weight, 3)
                                    for t, c in enumerate(convs)], wp=conv_pack(wp, 1),
                                cout=cout_b,
                                # the deepest up block reads its projection input at full size:
                                # folded like the down blocks' (the others read it upsampled)
                                wpf=conv_pack(wp, 3, cfg_cin=cout_b) if self.fold and blk is net.up[-1] else None))
        self.bn_out = tuple(dv(x) for x in _bn_affine(net.output[0]))
        self.head_w = dv(net.output[-1].weight.reshape(net.output[-1].out_channels, -1))
        self.head_b = dv(net.output[-1].bias)
        self.nout = net.output[-1].out_channels
        # per network image (tile): non-zero once one of its activations left the fp16 range;
        # sized and cleared by every forward (the clear is part of a captured graph)
        self.ovf = torch.zeros(1, dtype=torch.int32, device=td)

    # -- libcpx passes ----------------------------------------------------------------------------
    def _ovf_p(self, N):
        """The per-image overflow flags, at least N of them (a pass called on its own)."""
        if self.ovf.numel() < N:
            self.ovf = torch.zeros(N, dtype=torch.int32, device=self.td)
        return _p(self.ovf)

    def _empty(self, N, H, W, C):
        return torch.empty((N, H, W, C), dtype=torch.int32, device=self.td)  # split: 4 B per channel

    def _conv(self, x, pk, cout, bias, ks=3, res=None, res_up=False, style=None, bn=None, relu=True,
              y=False, z=True, z_up=False, head=False, in_up=False):
        variant = self.variant
        if isinstance(pk, tuple):  # (weights, variant) of a z-only convolution
            pk, variant = pk
        N, H, W, cin = x.shape
        if in_up:  # x is read 2x nearest-upsampled: the output has twice its size
            H, W = 2 * H, 2 * W
        yo = self._empty(N, H, W, cout) if y else None
        zo = None
        if z and not head:
            zo = self._empty(N, 2 * H, 2 * W, cout) if z_up else self._empty(N, H, W, cout)
        ho = torch.empty((N, H, W, self.nout), dtype=torch.float32, device=self.td) if head else None
        scale, shift = bn if bn is not None else (None, None)
        st, st_stride = (None, 0) if style is None else style
        check(self.lib.cpx_cpnet_x3_conv(
            self.dev.h, ks, variant, _p(x), int(in_up), N, H, W, cin, cout, _p(pk), _p(bias), _p(res), int(res_up),
            st, st_stride, _p(scale), _p(shift), int(relu), _p(yo), _p(zo), int(z_up),
            _p(self.head_w) if head else None, _p(self.head_b) if head else None, self.nout if head else 0,
            _p(ho), self._ovf_p(N)), "cpx_cpnet_x3_conv")
        return (ho,) if head else (yo, zo)

    def _conv_proj(self, x, pk, cout, bias, x2, pk2, style=None, bn=None, y=True):
        """3x3 conv of x + the folded 1x1 projection of x2 (cpx_cpnet_x3_conv_proj)."""
        N, H, W, cin = x.shape
        yo = self._empty(N, H, W, cout) if y else None
        zo = self._empty(N, H, W, cout)
        scale, shift = bn if bn is not None else (None, None)
        st, st_stride = (None, 0) if style is None else style
        check(self.lib.cpx_cpnet_x3_conv_proj(
            self.dev.h, self.variant, _p(x), N, H, W, cin, cout, _p(pk), _p(x2), x2.shape[-1], _p(pk2), _p(bias),
            st, st_stride, _p(scale), _p(shift), 1, _p(yo), _p(zo), 0, self._ovf_p(N)), "cpx_cpnet_x3_conv_proj")
        return yo, zo

    def _conv_pool(self, x, pk, cout, bias, res, bn):
        """A down block's last convolution (residual, y) with the next block's max-pool and its
        BatchNorm+ReLU fused into the epilogue (cpx_cpnet_x3_conv_pool): (y, pooled, z)."""
        N, H, W, cin = x.shape
        yo = self._empty(N, H, W, cout)
        xo = self._empty(N, H // 2, W // 2, cout)
        zo = self._empty(N, H // 2, W // 2, cout)
        check(self.lib.cpx_cpnet_x3_conv_pool(
            self.dev.h, self.variant, _p(x), N, H, W, cin, cout, _p(pk), _p(bias), _p(res), _p(yo), _p(xo), _p(zo),
            _p(bn[0]), _p(bn[1]), self._ovf_p(N)), "cpx_cpnet_x3_conv_pool")
        return yo, xo, zo

    def _proj(self, x, blk):
        return self._conv(x, blk["wp"], blk["cout"], None, ks=1, relu=False, y=True, z=False)[0]

    def _pool(self, x, bn):
        N, H, W, C = x.shape
        xo = self._empty(N, H // 2, W // 2, C)
        zo = self._empty(N, H // 2, W // 2, C)
        scale, shift = bn
        check(self.lib.cpx_cpnet_x3_pool(self.dev.h, _p(x), _p(scale), _p(shift), 1, N, H // 2, W // 2, C,
                                         _p(xo), _p(zo), self._ovf_p(N)), "cpx_cpnet_x3_pool")
        return xo, zo

    def _stem(self, x, d):
        N, H, W, _ = x.shape
        p = self._empty(N, H, W, 32)
        z = self._empty(N, H, W, 32)
        (s0, h0), (s1, h1) = d["bn"][0], d["bn"][1]
        check(self.lib.cpx_cpnet_x3_stem(self.dev.h, _p(x), N, H, W, _p(s0), _p(h0), _p(d["stem_w"]),
                                         _p(d["b"][0]), _p(s1), _p(h1), _p(d["stem_wp"]), _p(p), _p(z),
                                         self._ovf_p(N)), "cpx_cpnet_x3_stem")
        return p, z

    def _style(self, x):
        N, H, W, C = x.shape
        S = torch.empty((N, self.J), dtype=torch.float32, device=self.td)
        check(self.lib.cpx_cpnet_x3_style(self.dev.h, _p(x), N, H, W, C, _p(self.lin_w), _p(self.lin_b),
                                          self.J, _p(S)), "cpx_cpnet_x3_style")
        return S

    # -- forward ----------------------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, x):
        """x: fp32 [N, by, bx, 2] NHWC (CPX_TILE_F32_NHWC tiles) -> fp32 [N, by, bx, nout] NHWC."""
        self.dev._bind_stream()
        assert x.dtype == torch.float32 and x.is_contiguous() and x.shape[-1] == 2
        if self.ovf.numel() != x.shape[0]:
            self.ovf = torch.zeros(x.shape[0], dtype=torch.int32, device=self.td)
        self.ovf.zero_()
        xd = []
        zu = None
        nd = len(self.down)
        pooled = None  # (xin, z0) of the next block from the fused pool
        for n, d in enumerate(self.down):
            if n == 0:
                p, z = self._stem(x, d)
                x1, z = self._conv(z, d["pk"][1], d["cout"], d["b1p"], res=p, bn=d["bn"][2], y=True)
            else:
                xin, z0 = pooled if pooled is not None else self._pool(xd[-1], d["bn"][0])
                _, z = self._conv(z0, d["pk"][0], d["cout"], d["b"][0], bn=d["bn"][1])
                if d["wpf"] is not None:
                    x1, z = self._conv_proj(z, d["pk"][1], d["cout"], d["b1p"], xin, d["wpf"], bn=d["bn"][2])
                else:
                    p = self._proj(xin, d)
                    x1, z = self._conv(z, d["pk"][1], d["cout"], d["b1p"], res=p, bn=d["bn"][2], y=True)
            _, z = self._conv(z, d["pk"][2], d["cout"], d["b"][2], bn=d["bn"][3])
            if n < nd - 1 and X3_POOL_FUSE:
                xo, xin_n, z0_n = self._conv_pool(z, d["pk"][3], d["cout"], d["b"][3], x1, self.down[n + 1]["bn"][0])
                pooled = (xin_n, z0_n)
            elif n < nd - 1:
                xo, _ = self._conv(z, d["pk"][3], d["cout"], d["b"][3], res=x1, y=True, z=False)
            else:  # deepest level also feeds the first up block's BatchNorm+ReLU
                xo, zu = self._conv(z, d["pk"][3], d["cout"], d["b"][3], res=x1, bn=self.up[-1]["bn"][0], y=True)
            xd.append(xo)
        S = self._style(xd[-1])
        J = self.J
        x_small, z0 = xd[-1], zu
        for n in range(len(self.up) - 1, -1, -1):
            u = self.up[n]
            so = self.style_off[n]
            sty = [(ct.c_void_p(S.data_ptr() + 4 * o), J) for o in so]
            p = None if u["wpf"] is not None else self._proj(x_small, u)
            # below the deepest level the block input is nn.Upsample(x_small): z0 (its
            # BatchNorm+ReLU, pointwise) stays at the small size and is read upsampled
            _, z = self._conv(z0, u["pk"][0], u["cout"], u["b"][0], res=xd[n], style=sty[0], bn=u["bn"][1],
                              in_up=(n < len(self.up) - 1))
            if p is None:
                x1, z = self._conv_proj(z, u["pk"][1], u["cout"], u["b1p"], x_small, u["wpf"], style=sty[1],
                                        bn=u["bn"][2])
            else:
                x1, z = self._conv(z, u["pk"][1], u["cout"], u["b1p"], res=p, res_up=(n < len(self.up) - 1),
                                   style=sty[1], bn=u["bn"][2], y=True)
            _, z = self._conv(z, u["pk"][2], u["cout"], u["b"][2], style=sty[2], bn=u["bn"][3])
            if n > 0:
                x_small, z0 = self._conv(z, u["pk"][3], u["cout"], u["b"][3], res=x1, bn=self.up[n - 1]["bn"][0],
                                         y=True)
            else:
                out = self._conv(z, u["pk"][3], u["cout"], u["b"][3], res=x1, bn=self.bn_out, head=True)[0]
                N, H, W, nout = out.shape
                check(self.lib.cpx_cpnet_x3_mask_overflow(self.dev.h, _p(out), N, H, W, nout, _p(self.ovf)),
                      "cpx_cpnet_x3_mask_overflow")
                return out

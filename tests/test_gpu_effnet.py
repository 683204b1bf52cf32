"""f3 EfficientNetV2-L kernels (k_effnet.hip) against fp32 PyTorch on the CPU: the implicit-GEMM
convolution (1x1 / 3x3, stride 1 / 2 with TF 'same' padding, BatchNorm scale/shift, SiLU,
residual, squeeze-excite gate on the input), the stem, the depthwise convolution with its channel
sums, the squeeze-excite gate and the pool — inputs fp16, outputs fp16 (one rounding), so the
tolerance is fp16's (rel 2^-10 of the magnitude of the terms).  The whole forward is compared with
the fp32 module in tests/test_embed.py."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _same(x, k, s):
    """timm Conv2dSame padding of an NCHW tensor."""
    ih, iw = x.shape[-2:]
    ph = max((math.ceil(ih / s) - 1) * s + k - ih, 0)
    pw = max((math.ceil(iw / s) - 1) * s + k - iw, 0)
    return F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])


def _P(t):
    import ctypes as ct
    return None if t is None else ct.c_void_p(t.data_ptr())


@pytest.mark.parametrize("ks,stride,cin,cout,H,W,act,res,gate", [
    (3, 1, 32, 32, 20, 18, 1, True, False), (3, 2, 32, 128, 24, 22, 1, False, False),
    (3, 2, 64, 96, 17, 19, 1, False, False), (1, 1, 96, 384, 12, 12, 1, False, False),
    (1, 1, 384, 192, 12, 12, 0, True, True), (1, 1, 1344, 224, 7, 9, 0, True, True),
    (1, 1, 640, 1280, 6, 6, 1, False, False)])
def test_effnet_conv_vs_torch(dev, ks, stride, cin, cout, H, W, act, res, gate):
    td = dev.torch_device
    g = torch.Generator().manual_seed(ks * 7 + stride + cin + cout)
    N = 2
    x = torch.randn(N, cin, H, W, generator=g).half()
    w = (torch.randn(cout, cin, ks, ks, generator=g) / math.sqrt(cin * ks * ks)).half()
    sc = 1 + 0.2 * torch.randn(cout, generator=g)
    sh = 0.1 * torch.randn(cout, generator=g)
    gt = torch.sigmoid(torch.randn(N, cin, generator=g)) if gate else None
    Ho, Wo = -(-H // stride), -(-W // stride)
    r = torch.randn(N, cout, Ho, Wo, generator=g).half() if res else None
    # reference: fp32 on the fp16 operands; the gate multiplies the weights (as the kernel)
    xr = x.float() if gt is None else x.float()
    y = torch.zeros(N, cout, Ho, Wo)
    for n in range(N):
        wn = w.float() if gt is None else (w.float() * gt[n][None, :, None, None]).half().float()
        y[n] = F.conv2d(_same(xr[n:n + 1], ks, stride), wn, stride=stride)[0]
    y = y * sc[None, :, None, None] + sh[None, :, None, None]
    if act:
        y = F.silu(y)
    if res:
        y = y + r.float()
    xd = x.permute(0, 2, 3, 1).contiguous().to(td)
    wd = w.permute(0, 2, 3, 1).contiguous().to(td)
    out = torch.empty(N, Ho, Wo, cout, dtype=torch.float16, device=td)
    rd = r.permute(0, 2, 3, 1).contiguous().to(td) if res else None
    gd = gt.contiguous().to(td) if gate else None
    scd, shd = sc.to(td), sh.to(td)  # held: a temporary's memory is reused by the next one
    rc = dev.lib.cpx_effnet_conv(dev.h, _P(xd), N, H, W, cin, cout, ks, stride, _P(wd), _P(scd), _P(shd), act,
                                 _P(rd), _P(gd), _P(out))
    assert rc == 0, dev.lib.cpx_last_error()
    got = out.float().cpu().permute(0, 3, 1, 2)
    mag = y.abs() + 1.0
    assert ((got - y).abs() <= 2e-3 * mag).all(), float((got - y).abs().max())


def test_effnet_stem_dw_se_pool_vs_torch(dev):
    td = dev.torch_device
    g = torch.Generator().manual_seed(3)
    N, H, W = 2, 38, 36
    x = torch.randn(N, 3, H, W, generator=g).half()
    w = torch.randn(32, 3, 3, 3, generator=g) / math.sqrt(27)
    sc, sh = 1 + 0.1 * torch.randn(32, generator=g), 0.1 * torch.randn(32, generator=g)
    ref = F.silu(F.conv2d(_same(x.float(), 3, 2), w, stride=2) * sc[None, :, None, None] + sh[None, :, None, None])
    Ho, Wo = -(-H // 2), -(-W // 2)
    out = torch.empty(N, Ho, Wo, 32, dtype=torch.float16, device=td)
    dv = [t.to(td).contiguous() for t in (x, w.reshape(-1), sc, sh)]  # held for the call
    assert dev.lib.cpx_effnet_stem(dev.h, _P(dv[0]), N, H, W, _P(dv[1]), _P(dv[2]), _P(dv[3]), _P(out)) == 0
    got = out.float().cpu().permute(0, 3, 1, 2)
    assert ((got - ref).abs() <= 2e-3 * (ref.abs() + 1)).all()
    # depthwise (stride 1 and 2) + channel sums + SE gate + pool
    C, rdc = 128, 24
    for s in (1, 2):
        xi = torch.randn(N, C, 15, 14, generator=g).half()
        wd = torch.randn(C, 1, 3, 3, generator=g) / 3
        dsc, dsh = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
        dref = F.silu(F.conv2d(_same(xi.float(), 3, s), wd, stride=s, groups=C) * dsc[None, :, None, None] +
                      dsh[None, :, None, None])
        Hd, Wd = -(-15 // s), -(-14 // s)
        nb = dev.lib.cpx_effnet_dw_blocks(15, 14, s)
        o = torch.empty(N, Hd, Wd, C, dtype=torch.float16, device=td)
        part = torch.empty(N, nb, C, dtype=torch.float32, device=td)
        dd = [t.to(td).contiguous() for t in (xi.permute(0, 2, 3, 1), wd.reshape(C, 9), dsc, dsh)]
        assert dev.lib.cpx_effnet_dw(dev.h, _P(dd[0]), N, 15, 14, C, s, _P(dd[1]), _P(dd[2]), _P(dd[3]), _P(o),
                                     _P(part)) == 0
        dgot = o.float().cpu().permute(0, 3, 1, 2)
        assert ((dgot - dref).abs() <= 2e-3 * (dref.abs() + 1)).all(), float((dgot - dref).abs().max())
        wr, br = torch.randn(rdc, C, generator=g) / math.sqrt(C), 0.1 * torch.randn(rdc, generator=g)
        we, be = torch.randn(C, rdc, generator=g) / math.sqrt(rdc), 0.1 * torch.randn(C, generator=g)
        gate = torch.empty(N, C, dtype=torch.float32, device=td)
        sd = [t.to(td).contiguous() for t in (wr, br, we, be)]
        assert dev.lib.cpx_effnet_se(dev.h, _P(part), N, nb, Hd * Wd, C, rdc, _P(sd[0]), _P(sd[1]), _P(sd[2]),
                                     _P(sd[3]), _P(gate)) == 0
        mean = dgot.mean((2, 3))  # the stored (fp16) outputs, as the kernel sums them
        gref = torch.sigmoid(F.silu(mean @ wr.T + br) @ we.T + be)
        np.testing.assert_allclose(gate.cpu().numpy(), gref.numpy(), rtol=1e-5, atol=1e-6)
        pooled = torch.empty(N, C, dtype=torch.float32, device=td)
        assert dev.lib.cpx_effnet_pool(dev.h, _P(o), N, Hd * Wd, C, _P(pooled)) == 0
        np.testing.assert_allclose(pooled.cpu().numpy(), mean.numpy(), rtol=1e-5, atol=1e-6)

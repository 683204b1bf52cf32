"""The reference-precision CPnet (split fp16, "f16x3", k_conv_x3.hip / cpx.cpnet_x3) against
fp64 / fp32 references of the same operations.

  * split format: hi + lo * 2^-11 within 2^-22 relative (CPU);
  * every convolution instance (3x3 and the 1x1 projections, each tile configuration) with the
    fused epilogue (bias, split residual incl. nearest-upsampled reads, style, BatchNorm, ReLU,
    2x upsampled next input, the fp32 output head) vs fp64 arithmetic on the same split
    operands: error within fp32 accumulation noise (1e-6 of sum |w x|);
  * stem, pool and style kernels vs fp64;
  * the whole forward vs Cellpose's CPnet in fp32 on the CPU (the reference's precision,
    Cellpose_GPU_s3fs.py:108,143): max error <= 1e-5 of the output range, and bit-identical
    across two runs.
"""
import ctypes as ct

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cpx.cpnet_x3 import from_split, join_f16, pack_conv, split_f16, to_split


def test_split_roundtrip_error():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(100000) * np.exp(rng.uniform(-12, 10, 100000))).astype(np.float32)
    x = x[np.abs(x) < 65000]
    hi, lo = split_f16(x)
    v = join_f16(hi, lo).astype(np.float64)
    err = np.abs(v - x.astype(np.float64))
    assert np.all(err <= 2.0 ** -22 * np.abs(x) + 2.0 ** -35)


def test_pack_conv_layout():
    rng = np.random.default_rng(1)
    w = rng.standard_normal((64, 32, 3, 3)).astype(np.float32)
    pk = pack_conv(w, 32)  # [cout/bm][cin/16][ky][kx][bm][2][16]
    assert pk.shape == (2, 2, 3, 3, 32, 2, 16) and pk.dtype == np.float16
    hi, lo = split_f16(w)
    assert pk[1, 0, 2, 1, 5, 0, 7] == hi[32 + 5, 7, 2, 1]
    assert pk[0, 1, 0, 2, 31, 1, 3] == lo[31, 16 + 3, 0, 2]


def test_split_tensor_helpers():
    rng = np.random.default_rng(2)
    x = rng.standard_normal((2, 5, 7, 64)).astype(np.float32)
    s = to_split(x)
    raw = s.reshape(2, 5, 7, 64 * 2).view(np.int32)  # the device storage (4 bytes per channel)
    np.testing.assert_array_equal(from_split(s), from_split(raw))
    assert np.abs(from_split(s) - x).max() <= 2.0 ** -22 * np.abs(x).max()


# ---------------------------------------------------------------------------------------------
def _dev_split(x32, td):
    return torch.from_numpy(to_split(x32).reshape(x32.shape[:-1] + (x32.shape[-1] * 2,)).view(np.int32)).to(td)


def _host_split(t):
    return from_split(t.cpu().numpy())


def _ref(v):
    """fp64 value of a split-representable fp32 tensor (what the kernel multiplies)."""
    return torch.from_numpy(from_split(to_split(v)).astype(np.float64))


CONFIGS = [  # ks, cin, cout, H, W, variant
    (3, 32, 32, 40, 70, 0), (3, 64, 32, 24, 36, 0), (3, 32, 64, 28, 20, 0), (3, 64, 64, 20, 18, 1),
    (3, 128, 64, 16, 16, 0), (3, 64, 128, 30, 29, 0), (3, 128, 128, 28, 28, 1), (3, 256, 128, 14, 14, 0),
    (3, 128, 256, 14, 28, 0), (3, 256, 256, 16, 12, 1), (1, 32, 64, 20, 22, 0), (1, 64, 128, 17, 16, 0),
    (1, 128, 256, 14, 14, 0), (1, 256, 256, 9, 7, 0), (1, 256, 128, 8, 8, 0), (1, 128, 64, 12, 16, 0),
    (1, 64, 32, 16, 16, 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("ks,cin,cout,H,W,variant", CONFIGS)
def test_x3_conv_epilogue_vs_fp64(dev, ks, cin, cout, H, W, variant):
    lib, td = dev.lib, dev.torch_device
    rng = np.random.default_rng(ks * 1000 + cin + cout + variant)
    N = 2
    bm = ct.c_int()
    assert lib.cpx_cpnet_x3_cfg(ks, cin, cout, variant, ct.byref(bm)) == 0
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, cin, ks, ks)) * (2.0 / (cin * ks * ks)) ** 0.5).astype(np.float32)
    bias = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    res_up = ks == 3 and H % 2 == 0 and W % 2 == 0 and cin == 64
    z_up = ks == 3 and cout <= 128 and not res_up
    rh, rw = (H // 2, W // 2) if res_up else (H, W)
    res = rng.standard_normal((N, rh, rw, cout)).astype(np.float32)
    style = (0.3 * rng.standard_normal((N, cout + 8))).astype(np.float32)  # stride cout + 8
    scale = (1 + 0.2 * rng.standard_normal(cout)).astype(np.float32)
    shift = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    pk = torch.from_numpy(pack_conv(w, bm.value)).to(td)
    xd, resd = _dev_split(x, td), _dev_split(res, td)
    yd = torch.empty((N, H, W, cout), dtype=torch.int32, device=td)
    zd = torch.empty((N, 2 * H, 2 * W, cout) if z_up else (N, H, W, cout), dtype=torch.int32, device=td)
    bd, sd, scd, shd = (torch.from_numpy(a).to(td) for a in (bias, style, scale, shift))
    ovf = torch.zeros(N, dtype=torch.int32, device=td)  # one flag per image
    P = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    rc = lib.cpx_cpnet_x3_conv(dev.h, ks, variant, P(xd), 0, N, H, W, cin, cout, P(pk), P(bd), P(resd),
                               int(res_up), P(sd), cout + 8, P(scd), P(shd), 1, P(yd), P(zd), int(z_up), None,
                               None, 0, None, P(ovf))
    assert rc == 0, lib.cpx_last_error()
    torch.cuda.synchronize()
    # fp64 reference on the split-representable operands
    hi, lo = split_f16(w)
    w64 = torch.from_numpy(hi.astype(np.float64) + lo.astype(np.float64) / 2048.0)
    x64 = _ref(x).permute(0, 3, 1, 2)
    conv = F.conv2d(x64, w64, padding=ks // 2)
    mag = F.conv2d(x64.abs(), w64.abs(), padding=ks // 2)
    r64 = _ref(res).permute(0, 3, 1, 2)
    if res_up:
        r64 = r64.repeat_interleave(2, 2).repeat_interleave(2, 3)
    t = conv + torch.from_numpy(bias.astype(np.float64))[None, :, None, None] + r64
    u = t + torch.from_numpy(style[:, :cout].astype(np.float64))[:, :, None, None]
    z = torch.relu(torch.from_numpy(scale.astype(np.float64))[None, :, None, None] * u +
                   torch.from_numpy(shift.astype(np.float64))[None, :, None, None])
    tol_t = 1e-6 * (mag + r64.abs() + 1.0) + 2.0 ** -21 * t.abs()
    y_got = torch.from_numpy(_host_split(yd)).permute(0, 3, 1, 2).double()
    assert ((y_got - t).abs() <= tol_t).all(), float((y_got - t).abs().max())
    z_got = torch.from_numpy(_host_split(zd)).permute(0, 3, 1, 2).double()
    if z_up:
        z_ref = z.repeat_interleave(2, 2).repeat_interleave(2, 3)
        tol = (tol_t * scale.astype(np.float64).__abs__().max() + 2.0 ** -21 * z.abs()).repeat_interleave(2, 2) \
            .repeat_interleave(2, 3)
    else:
        z_ref = z
        tol = tol_t * np.abs(scale).max() + 2.0 ** -21 * z.abs()
    assert ((z_got - z_ref).abs() <= tol).all(), float((z_got - z_ref).abs().max())
    assert int(ovf.sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cin2,H,W,with_style", [(64, 32, 20, 18, False), (128, 64, 30, 29, False),
                                                     (256, 128, 14, 14, False), (256, 256, 16, 12, True)])
def test_x3_conv_proj_vs_fp64(dev, cin, cin2, H, W, with_style):
    """cpx_cpnet_x3_conv_proj: a 3x3 convolution with the block's 1x1 projection folded in as
    extra one-tap slabs (every down block's second convolution and the deepest up block's) vs
    fp64 conv3x3(x) + conv1x1(x2) + bias (+ style), BatchNorm, ReLU on the same split operands."""
    lib, td = dev.lib, dev.torch_device
    rng = np.random.default_rng(cin + cin2)
    N, cout = 2, cin
    bm = ct.c_int()
    assert lib.cpx_cpnet_x3_cfg(3, cin, cout, 0, ct.byref(bm)) == 0
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    x2 = rng.standard_normal((N, H, W, cin2)).astype(np.float32)
    w = (rng.standard_normal((cout, cin, 3, 3)) * (2.0 / (cin * 9)) ** 0.5).astype(np.float32)
    wp = (rng.standard_normal((cout, cin2, 1, 1)) * (2.0 / cin2) ** 0.5).astype(np.float32)
    bias = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    style = (0.3 * rng.standard_normal((N, cout + 8))).astype(np.float32)
    scale = (1 + 0.2 * rng.standard_normal(cout)).astype(np.float32)
    shift = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    pk, pk2 = (torch.from_numpy(pack_conv(a, bm.value)).to(td) for a in (w, wp))
    xd, x2d = _dev_split(x, td), _dev_split(x2, td)
    yd = torch.empty((N, H, W, cout), dtype=torch.int32, device=td)
    zd = torch.empty((N, H, W, cout), dtype=torch.int32, device=td)
    bd, sd, scd, shd = (torch.from_numpy(a).to(td) for a in (bias, style, scale, shift))
    ovf = torch.zeros(N, dtype=torch.int32, device=td)
    P = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    rc = lib.cpx_cpnet_x3_conv_proj(dev.h, 0, P(xd), N, H, W, cin, cout, P(pk), P(x2d), cin2, P(pk2), P(bd),
                                    P(sd) if with_style else None, cout + 8 if with_style else 0, P(scd), P(shd), 1,
                                    P(yd), P(zd), 0, P(ovf))
    assert rc == 0, lib.cpx_last_error()
    torch.cuda.synchronize()
    w64, wp64 = (torch.from_numpy(from_split(to_split(a.transpose(0, 2, 3, 1))).astype(np.float64)).permute(0, 3, 1, 2)
                 for a in (w, wp))
    x64, x264 = _ref(x).permute(0, 3, 1, 2), _ref(x2).permute(0, 3, 1, 2)
    t = F.conv2d(x64, w64, padding=1) + F.conv2d(x264, wp64) + torch.from_numpy(bias.astype(np.float64))[None, :, None, None]
    mag = F.conv2d(x64.abs(), w64.abs(), padding=1) + F.conv2d(x264.abs(), wp64.abs())
    u = t + (torch.from_numpy(style[:, :cout].astype(np.float64))[:, :, None, None] if with_style else 0)
    z = torch.relu(torch.from_numpy(scale.astype(np.float64))[None, :, None, None] * u +
                   torch.from_numpy(shift.astype(np.float64))[None, :, None, None])
    tol_t = 1e-6 * (mag + 1.0) + 2.0 ** -21 * t.abs()
    y_got = torch.from_numpy(_host_split(yd)).permute(0, 3, 1, 2).double()
    assert ((y_got - t).abs() <= tol_t).all(), float((y_got - t).abs().max())
    z_got = torch.from_numpy(_host_split(zd)).permute(0, 3, 1, 2).double()
    tol = tol_t * np.abs(scale).max() + 2.0 ** -21 * z.abs()
    assert ((z_got - z).abs() <= tol).all(), float((z_got - z).abs().max())
    assert int(ovf.sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,variant", [(64, 32, 0), (128, 64, 0), (256, 128, 0), (64, 32, 1), (128, 64, 1),
                                              (256, 128, 1)])
def test_x3_conv_in_up(dev, cin, cout, variant):
    """in_up: the input tensor is half the output size and read 2x nearest-upsampled (the up
    path's nn.Upsample folded into the convolution's halo loads) — vs fp64 conv2d of the
    explicitly upsampled tensor; with the residual read upsampled too (res_up)."""
    lib, td = dev.lib, dev.torch_device
    rng = np.random.default_rng(cin + cout + 100 * variant)
    N, H, W = 2, 24, 40
    bm = ct.c_int()
    assert lib.cpx_cpnet_x3_cfg(3, cin, cout, variant, ct.byref(bm)) == 0
    x = rng.standard_normal((N, H // 2, W // 2, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, cin, 3, 3)) * (2.0 / (cin * 9)) ** 0.5).astype(np.float32)
    bias = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    res = rng.standard_normal((N, H // 2, W // 2, cout)).astype(np.float32)
    pk = torch.from_numpy(pack_conv(w, bm.value)).to(td)
    xd, resd = _dev_split(x, td), _dev_split(res, td)
    yd = torch.empty((N, H, W, cout), dtype=torch.int32, device=td)
    bd = torch.from_numpy(bias).to(td)
    ovf = torch.zeros(N, dtype=torch.int32, device=td)
    P = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    rc = lib.cpx_cpnet_x3_conv(dev.h, 3, variant, P(xd), 1, N, H, W, cin, cout, P(pk), P(bd), P(resd), 1,
                               None, 0, None, None, 0, P(yd), None, 0, None, None, 0, None, P(ovf))
    assert rc == 0, lib.cpx_last_error()
    hi, lo = split_f16(w)
    w64 = torch.from_numpy(hi.astype(np.float64) + lo.astype(np.float64) / 2048.0)
    up = lambda t: t.repeat_interleave(2, 2).repeat_interleave(2, 3)  # noqa: E731
    x64 = up(_ref(x).permute(0, 3, 1, 2))
    r64 = up(_ref(res).permute(0, 3, 1, 2))
    t = F.conv2d(x64, w64, padding=1) + torch.from_numpy(bias.astype(np.float64))[None, :, None, None] + r64
    mag = F.conv2d(x64.abs(), w64.abs(), padding=1)
    tol = 1e-6 * (mag + r64.abs() + 1.0) + 2.0 ** -21 * t.abs()
    got = torch.from_numpy(_host_split(yd)).permute(0, 3, 1, 2).double()
    assert ((got - t).abs() <= tol).all(), float((got - t).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1])
def test_x3_head_and_overflow(dev, variant):
    lib, td = dev.lib, dev.torch_device
    rng = np.random.default_rng(7)
    N, H, W, cin, cout, nh = 1, 24, 40, 32, 32, 3
    bm = ct.c_int()
    assert lib.cpx_cpnet_x3_cfg(3, cin, cout, variant, ct.byref(bm)) == 0
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, cin, 3, 3)) * 0.08).astype(np.float32)
    bias = (0.1 * rng.standard_normal(cout)).astype(np.float32)
    hw = rng.standard_normal((nh, 32)).astype(np.float32)
    hb = rng.standard_normal(nh).astype(np.float32)
    scale = np.ones(cout, np.float32)
    shift = np.zeros(cout, np.float32)
    P = lambda t: ct.c_void_p(t.data_ptr())  # noqa: E731
    pk = torch.from_numpy(pack_conv(w, bm.value)).to(td)
    xd = _dev_split(x, td)
    out = torch.empty((N, H, W, nh), dtype=torch.float32, device=td)
    dv = [torch.from_numpy(a).to(td) for a in (bias, scale, shift, hw, hb)]
    ovf = torch.zeros(1, dtype=torch.int32, device=td)
    rc = lib.cpx_cpnet_x3_conv(dev.h, 3, variant, P(xd), 0, N, H, W, cin, cout, P(pk), P(dv[0]), None, 0, None, 0,
                               P(dv[1]), P(dv[2]), 1, None, None, 0, P(dv[3]), P(dv[4]), nh, P(out), P(ovf))
    assert rc == 0
    hi, lo = split_f16(w)
    w64 = torch.from_numpy(hi.astype(np.float64) + lo.astype(np.float64) / 2048.0)
    z = torch.relu(F.conv2d(_ref(x).permute(0, 3, 1, 2), w64, padding=1) +
                   torch.from_numpy(bias.astype(np.float64))[None, :, None, None])
    ref = torch.einsum("nchw,jc->nhwj", z, torch.from_numpy(hw.astype(np.float64))) + torch.from_numpy(hb.astype(np.float64))
    got = out.cpu().double()
    assert (got - ref).abs().max() <= 1e-5 * (ref.abs().max() + 1)
    assert int(ovf.item()) == 0
    # an activation beyond the fp16 range raises the flag of its own image only (the host
    # re-runs just those FOVs): image 1 of 3 carries the large input
    x3 = np.concatenate([x, np.clip(x * 1e5, -60000, 60000), x])
    zd = torch.empty((3, H, W, cout), dtype=torch.int32, device=td)
    xd2 = torch.from_numpy(to_split(x3).reshape(3, H, W, 2 * cin).view(np.int32)).to(td)
    ovf3 = torch.zeros(3, dtype=torch.int32, device=td)
    rc = lib.cpx_cpnet_x3_conv(dev.h, 3, variant, P(xd2), 0, 3, H, W, cin, cout, P(pk), P(dv[0]), None, 0, None, 0,
                               None, None, 0, None, P(zd), 0, None, None, 0, None, P(ovf3))
    assert rc == 0
    assert ovf3.cpu().tolist() == [0, 1, 0]


@pytest.mark.gpu
def test_x3_stem_pool_style(dev):
    from cpx.cpnet import build_cpnet
    from cpx.cpnet_x3 import FusedCPnetX3, _fold_proj
    td = dev.torch_device
    net = build_cpnet(seed=3)
    f = FusedCPnetX3(net, dev)
    rng = np.random.default_rng(5)
    N, H, W = 2, 32, 48
    x = rng.uniform(-0.2, 1.5, (N, H, W, 2)).astype(np.float32)
    p, z = f._stem(torch.from_numpy(x).to(td), f.down[0])
    blk = net.down[0]
    x64 = torch.from_numpy(x.astype(np.float64)).permute(0, 3, 1, 2)
    with torch.no_grad():
        netd = net.double()
        z_ref = netd.down[0].conv[1][:2](netd.down[0].conv[0](x64))  # BN0-ReLU-conv0, BN1-ReLU
        wpf, _ = _fold_proj(blk.proj)  # BatchNorm folded; the bias joins conv1's (b1p)
        p_ref = F.conv2d(x64, wpf.double())
    z_got = torch.from_numpy(_host_split(z)).permute(0, 3, 1, 2).double()
    p_got = torch.from_numpy(_host_split(p)).permute(0, 3, 1, 2).double()
    assert (z_got - z_ref).abs().max() <= 1e-5 * (z_ref.abs().max() + 1)
    assert (p_got - p_ref).abs().max() <= 1e-5 * (p_ref.abs().max() + 1)
    # pool: exact max of the split values, then BatchNorm + ReLU
    y = rng.standard_normal((N, 16, 20, 64)).astype(np.float32)
    yd = _dev_split(y, td)
    bn = f.down[2]["bn"][0]  # BatchNorm on the 64 channels entering the third down block
    xo, zo = f._pool(yd, bn)
    yr = from_split(to_split(y))
    mx = yr.reshape(N, 8, 2, 10, 2, 64).max(axis=(2, 4))
    np.testing.assert_array_equal(_host_split(xo), mx)
    zr = np.maximum(bn[0].cpu().numpy().astype(np.float64) * mx + bn[1].cpu().numpy(), 0)
    assert np.abs(_host_split(zo) - zr).max() <= 1e-6 * (np.abs(zr).max() + 1)
    # style + Linear layers
    d3 = rng.standard_normal((N, 7, 9, 256)).astype(np.float32)
    S = f._style(_dev_split(d3, td)).cpu().numpy().astype(np.float64)
    st = from_split(to_split(d3)).astype(np.float64).mean(axis=(1, 2))
    st = st / np.sqrt((st ** 2).sum(axis=1, keepdims=True))
    ref = st @ f.lin_w.cpu().numpy().astype(np.float64).T + f.lin_b.cpu().numpy()
    assert np.abs(S - ref).max() <= 1e-5 * (np.abs(ref).max() + 1)


@pytest.mark.gpu
def test_x3_forward_vs_cpu_fp32(dev):
    """Whole CPnet: native f16x3 on the GPU vs the fp32 module on the CPU (the reference's
    precision); and two GPU runs bit-identical."""
    import os
    from cpx.cpnet import build_cpnet
    from cpx.cpnet_x3 import FusedCPnetX3
    td = dev.torch_device
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    wpath = os.path.join(repo, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    net = build_cpnet(state_dict_path=wpath if os.path.exists(wpath) else None)
    f = FusedCPnetX3(net, dev)
    rng = np.random.default_rng(11)
    N = 3
    x = np.clip(rng.gamma(0.6, 0.4, (N, 224, 224, 2)), 0, 3).astype(np.float32)
    xd = torch.from_numpy(x).to(td)
    out1 = f(xd).cpu().numpy()
    out2 = f(xd).cpu().numpy()
    np.testing.assert_array_equal(out1, out2)
    torch.set_num_threads(16)
    with torch.no_grad():
        ref = net.float()(torch.from_numpy(x).permute(0, 3, 1, 2)).permute(0, 2, 3, 1).numpy()
    err = np.abs(out1 - ref).max(axis=(0, 1, 2))
    rng_ = np.abs(ref).max(axis=(0, 1, 2))
    print("x3 vs cpu fp32: max abs err per output", err, "range", rng_)
    assert np.all(err <= 1e-5 * rng_ + 1e-6)


@pytest.mark.gpu
def test_x3_folded_projections_vs_separate(dev, monkeypatch):
    """The 1x1 block projections folded into the blocks' second 3x3 convolutions
    (cpx_cpnet_x3_conv_proj, the default) against separate projection passes whose split-rounded
    outputs are added as residuals: the whole forward agrees to fp32 rounding."""
    import os
    from cpx import cpnet_x3
    from cpx.cpnet import build_cpnet
    td = dev.torch_device
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    wpath = os.path.join(repo, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    net = build_cpnet(state_dict_path=wpath if os.path.exists(wpath) else None)
    rng = np.random.default_rng(13)
    x = torch.from_numpy(np.clip(rng.gamma(0.6, 0.4, (3, 224, 224, 2)), 0, 3).astype(np.float32)).to(td)
    folded = cpnet_x3.FusedCPnetX3(net, dev)(x).cpu().numpy()
    monkeypatch.setattr(cpnet_x3, "X3_FOLD", False)
    unfolded = cpnet_x3.FusedCPnetX3(net, dev)(x).cpu().numpy()
    rng_ = np.abs(unfolded).max(axis=(0, 1, 2))
    assert np.all(np.abs(folded - unfolded).max(axis=(0, 1, 2)) <= 1e-5 * rng_ + 1e-6)

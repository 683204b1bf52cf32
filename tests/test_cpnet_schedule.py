"""CPU check of the fused CPnet schedule's algebra (cpx/cpnet_fused.py): the libcpx passes are
replaced by their torch definitions in fp32, so any rewrite error (BatchNorm folding, bias
merging, upsample commuting, pool fusion) shows up against the eager module."""
import torch
import torch.nn.functional as F

from cpx.cpnet import build_cpnet
from cpx.cpnet_fused import FusedCPnet


class _EmuDev:
    torch_device = torch.device("cpu")
    lib = None
    h = None

    def _bind_stream(self):
        pass


def _bc(v):
    return v[None, :, None, None]


def _up(t):
    return t.repeat_interleave(2, 2).repeat_interleave(2, 3)


class _Emu(FusedCPnet):
    def __init__(self, net):
        super().__init__(net, _EmuDev())

        def cvt(o):
            if isinstance(o, torch.Tensor):
                return o.float()
            if isinstance(o, (list, tuple)):
                return type(o)(cvt(v) for v in o)
            if isinstance(o, dict):
                return {k: cvt(v) for k, v in o.items()}
            return o
        self.down = cvt(self.down)
        self.up = cvt(self.up)
        self.w_out, self.b_out = self.w_out.float(), self.b_out.float()
        # exact fp32 weights for the check (the product stores bf16 copies)
        for d, blk in zip(self.down, net.down):
            d["w"] = [blk.conv[t][-1].weight.detach().float() for t in range(4)]
        for u, blk in zip(self.up, net.up):
            u["w"] = [c[-1].weight.detach().float() for c in
                      (blk.conv0, blk.conv1.conv, blk.conv2.conv, blk.conv3.conv)]
        self.w_out = net.output[-1].weight.detach().float()
        self.b_out = net.output[-1].bias.detach().float()

    def _epi(self, conv, bias, res=None, res_up=False, style=None, bn=None, relu=True,
             y=False, z=True, z_up=False):
        t = conv.float() + (_bc(bias) if bias is not None else 0.0)
        if res is not None:
            t = t + (_up(res) if res_up else res)
        yo = t if y else None
        if not z:
            return yo, None
        u = t + (style[:, :, None, None] if style is not None else 0.0)
        if bn is not None:
            u = _bc(bn[0]) * u + _bc(bn[1])
        if relu:
            u = torch.clamp_min(u, 0.0)
        return yo, (_up(u) if z_up else u)

    def _pool(self, x, bn):
        xo = F.max_pool2d(x, 2, 2)
        return xo, torch.clamp_min(_bc(bn[0]) * xo + _bc(bn[1]), 0.0)


def test_fused_schedule_algebra_matches_module():
    net = build_cpnet(seed=4)
    emu = _Emu(net)
    x = torch.rand(2, 2, 64, 48, generator=torch.Generator().manual_seed(0)) * 3.0
    with torch.no_grad():
        ref = net(x)
        got = emu(x.contiguous(memory_format=torch.channels_last))
    # only the folded 1x1 projections carry bf16 weights
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 2e-2 * scale
    assert torch.corrcoef(torch.stack([got.ravel(), ref.ravel()]))[0, 1] > 0.9999

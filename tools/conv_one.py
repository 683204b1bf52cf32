"""Development: time ONE native 3x3 convolution shape (for rocprofv3 counter passes).

python tools/conv_one.py --cin 32 --cout 32 --H 224 --N 144 [--res --y --z --style --zup --resup]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx._lib import check  # noqa: E402
from cpx.cpnet_fused import _p, _pack3x3  # noqa: E402
from cpx.device import Device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=32)
    ap.add_argument("--cout", type=int, default=32)
    ap.add_argument("--H", type=int, default=224)
    ap.add_argument("--N", type=int, default=144)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stamps", action="store_true", help="read the CPX_CONV_STAMP phase sums")
    for f in ("res", "y", "style", "zup", "resup", "noz"):
        ap.add_argument("--" + f, action="store_true")
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    CL = torch.channels_last
    N, H, W, cin, cout = a.N, a.H, a.H, a.cin, a.cout
    x = torch.randn(N, cin, H, W, device=td).to(torch.bfloat16).contiguous(memory_format=CL)
    w = torch.randn(cout, cin, 3, 3) * (2.0 / (9 * cin)) ** 0.5
    pk = _pack3x3(dev.lib, w, td)
    bias = torch.randn(cout, device=td)
    rs = (N, cout, H // 2, W // 2) if a.resup else (N, cout, H, W)
    res = torch.randn(*rs, device=td).to(torch.bfloat16).contiguous(memory_format=CL) if a.res else None
    sty = torch.randn(N, cout, device=td) if a.style else None
    scale, shift = torch.randn(cout, device=td), torch.randn(cout, device=td)
    yo = torch.empty((N, cout, H, W), dtype=torch.bfloat16, device=td, memory_format=CL) if a.y else None
    zs = (N, cout, 2 * H, 2 * W) if a.zup else (N, cout, H, W)
    zo = None if a.noz else torch.empty(zs, dtype=torch.bfloat16, device=td, memory_format=CL)

    def run():
        check(dev.lib.cpx_cpnet_conv3x3(dev.h, _p(x), N, H, W, cin, cout, _p(pk), _p(bias), _p(res),
                                        int(a.resup), _p(sty), _p(scale), _p(shift), 1, _p(yo), _p(zo),
                                        int(a.zup)), "conv3x3")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1e3
    if a.stamps:
        import ctypes as ct
        buf = (ct.c_ulonglong * 16)()
        dev.lib.cpx_conv_prof_read(buf)
        vals = list(buf)[:8]
        tot = sum(vals) or 1
        names = ["issue loads", "wait+LDS store", "barrier", "mfma", "barrier2", "bias/res", "y", "z"]
        print("phase shares (wave 0 of each block): " +
              ", ".join(f"{nm}={v / tot * 100:.1f}%" for nm, v in zip(names, vals)))
    print(f"{cin}->{cout} H={H} N={N}: {us:.1f} us  {2.0 * N * H * W * cin * cout * 9 / us / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()

"""Development timing of every native 3x3 convolution of the CPnet forward, in isolation.

Runs one FusedCPnet forward over N tiles of 224^2 and, inside a wrapper around
cpx_cpnet_conv3x3, replays each call `reps` times between HIP events on the launch stream.
Reports per call: shapes, epilogue flags, us, TFLOP/s and the minimum HBM bytes (input, residual,
outputs once).  CPX_LIB=<path> selects a libcpx variant (tools/build_variants.sh).

python tools/conv_bench.py [--tiles 144] [--reps 10]
"""
import argparse
import ctypes as ct
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-processing-suite_amd"))
import torch  # noqa: E402

from cpx.cpnet import build_cpnet  # noqa: E402
from cpx.cpnet_fused import FusedCPnet  # noqa: E402
from cpx.device import Device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=144)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forward", type=int, default=5, help="timed whole forwards")
    a = ap.parse_args()
    dev = Device(0)
    td = dev.torch_device
    net = build_cpnet(seed=0).to(td)
    f = FusedCPnet(net, dev)
    x = torch.randn(a.tiles, 2, 224, 224, device=td).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    lib = dev.lib
    real = lib.cpx_cpnet_conv3x3
    rows = []

    class Wrap:
        def __call__(self, *args):
            h, xin, N, H, W, cin, cout, pk, bias, res, res_up, sty, sc, sh, relu, y, z, z_up = args
            rc = real(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                real(*args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.reps * 1e3
            def on(v):
                return v is not None and (not isinstance(v, ct.c_void_p) or v.value is not None)
            flops = 2.0 * N * H * W * cin * cout * 9
            px = N * H * W
            byt = px * cin * 2 + px * cout * 2 * (on(y) + on(z) * (4 if z_up else 1))
            if on(res):
                byt += px * cout * 2 // (4 if res_up else 1)
            rows.append((cin, cout, H, int(on(res)), int(on(y)),
                         int(on(z)), int(on(sty)), us, flops / us / 1e6,
                         byt / us / 1e3))
            return rc

    with torch.no_grad():
        f(x)
        torch.cuda.synchronize()
        lib.cpx_cpnet_conv3x3 = Wrap()
        f(x)
        lib.cpx_cpnet_conv3x3 = real
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.forward):
            f(x)
        e1.record()
        torch.cuda.synchronize()
    print(f"lib={os.environ.get('CPX_LIB', 'default')} tiles={a.tiles}")
    print(" cin cout   H res y z sty       us   TFLOP/s   GB/s(min)")
    tot = 0.0
    for r in rows:
        tot += r[7]
        print(f"{r[0]:4d} {r[1]:4d} {r[2]:3d} {r[3]:3d} {r[4]} {r[5]} {r[6]:3d} {r[7]:8.1f} {r[8]:9.1f} {r[9]:9.1f}")
    print(f"sum of native convs: {tot / 1e3:.3f} ms; whole forward: {e0.elapsed_time(e1) / a.forward:.3f} ms")


if __name__ == "__main__":
    main()

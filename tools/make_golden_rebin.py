"""Golden fixtures for the image re-binning row — test tooling.

Runs the REFERENCE function Image_re-binning.py:12-22 `process_image_in_memory` (imported
unmodified from /root/reference with boto3 stubbed; needs Pillow >= 9.1 for
Image.Resampling — the container's python3.10 has Pillow 12.2.0) on 16-bit TIFF planes built
from the integer-only seeded generators of oracle/synth_golden.py, and stores inputs, outputs
and the Pillow version in tests/golden/rebin_cases.npz.  The full-size case (2080^2 -> 1080^2)
stores only its seed and the SHA-256 of the output (the input is regenerated bit-exactly).

    python tools/make_golden_rebin.py
"""
from __future__ import annotations

import hashlib
import importlib.util
import io
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import synth_golden as sg  # noqa: E402

sys.dont_write_bytecode = True


def load_reference():
    sys.modules.setdefault("boto3", types.ModuleType("boto3"))
    spec = importlib.util.spec_from_file_location("rebin_ref", "/root/reference/Image_re-binning.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def ref_resize(m, a: np.ndarray, res: int) -> np.ndarray:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, format="tiff")
    out = m.process_image_in_memory(buf.getvalue(), target_size=(res, res))
    return np.array(Image.open(io.BytesIO(out)))


# (seed, H, W, target): downscale, upscale, identity width, odd sizes, saturated planes
SMALL = [(11, 97, 130, 64), (12, 50, 40, 120), (13, 64, 64, 64), (14, 300, 260, 128),
         (15, 208, 208, 108), (16, 33, 257, 17)]
FULL = (21, 2080, 2080, 1080)


def main():
    import PIL
    m = load_reference()
    out = {"pillow_version": np.array(PIL.__version__)}
    for i, (seed, H, W, res) in enumerate(SMALL):
        a = sg.plane(seed, H, W, n_blobs=max(3, H * W // 2000))
        if i % 2:  # noise-only planes exercise the 16-bit overflow / clip path
            a = (sg._stream(seed, H * W, 3) & 0xFFFF).astype(np.uint16).reshape(H, W)
        out[f"in_{i}"] = a
        out[f"out_{i}"] = ref_resize(m, a, res)
        out[f"res_{i}"] = np.array(res)
        if i == 0:  # the reference's complete output container (LZW TIFF bytes)
            from PIL import Image
            buf = io.BytesIO()
            Image.fromarray(a).save(buf, format="tiff")
            out["in_bytes_0"] = np.frombuffer(buf.getvalue(), np.uint8)
            out["out_bytes_0"] = np.frombuffer(m.process_image_in_memory(buf.getvalue(), target_size=(res, res)), np.uint8)
    seed, H, W, res = FULL
    a = sg.plane(seed, H, W, n_blobs=300)
    o = ref_resize(m, a, res)
    out["full_seed"] = np.array([seed, H, W, res])
    out["full_sha256"] = np.array(hashlib.sha256(o.astype("<u2").tobytes()).hexdigest())
    out["full_out_rows"] = o[::97].copy()
    dst = os.path.join(REPO, "tests", "golden", "rebin_cases.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, "Pillow", PIL.__version__, "cases", len(SMALL))


if __name__ == "__main__":
    main()

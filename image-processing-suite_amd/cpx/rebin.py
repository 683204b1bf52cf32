"""Image re-binning — the MI355X replacement of Image_re-binning.py.

The reference walks an S3 prefix, and for every image decodes it with PIL, resizes it to a
square `resolution` with LANCZOS and re-uploads it as an LZW TIFF under the key with 'Image'
replaced by 'Image_binned' (Image_re-binning.py:12-58).  Here the resize runs on the GPU
(libcpx cpx_rebin_u16, bit-identical to Pillow's resampler for 16-bit planes) for batches of
planes; decoding and the LZW container stay on the host (Pillow, as in the reference), with a
local directory tree standing in for the bucket.

  python -m cpx.rebin --bucket_name ROOT --image_folder path/to/Images --resolution 1080
"""
from __future__ import annotations

import argparse
import concurrent.futures
import io
import logging
import os

import numpy as np

log = logging.getLogger("cpx.rebin")
VALID_EXTENSIONS = (".png", ".jpg", ".jpeg", ".tif", ".tiff")  # Image_re-binning.py:36


def _decode(image_bytes: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(image_bytes)) as img:
        if img.mode not in ("I;16", "I;16L"):
            raise ValueError(f"re-binning on the GPU handles 16-bit planes, got mode {img.mode}")
        return np.array(img)


def _encode(plane: np.ndarray) -> bytes:
    from PIL import Image
    out = io.BytesIO()
    # the reference's container: Image_re-binning.py:20
    Image.fromarray(plane).save(out, format="tiff", compression="tiff_lzw")
    return out.getvalue()


def rebin_planes(dev, planes, out_h: int, out_w: int):
    """uint16 planes [G, H, W] (numpy or device int16 tensor) -> device int16 [G, out_h, out_w]."""
    import torch
    if isinstance(planes, np.ndarray):
        planes = torch.from_numpy(np.ascontiguousarray(planes).view(np.int16)).to(dev.torch_device)
    out = torch.empty((planes.shape[0], out_h, out_w), dtype=torch.int16, device=planes.device)
    dev.rebin(planes, out_h, out_w, out)
    return out


def process_image_in_memory(image_bytes: bytes, target_size=(1080, 1080), dev=None) -> bytes:
    """Image_re-binning.py:12-22: decode, resize to target_size (width, height) with LANCZOS,
    return the LZW TIFF bytes — the resize on the GPU."""
    from .device import Device
    dev = dev or Device(0)
    a = _decode(image_bytes)
    out = rebin_planes(dev, a[None], target_size[1], target_size[0])
    return _encode(out[0].cpu().numpy().view(np.uint16))


def process_images(root: str, image_folder: str, resolution: int, dev=None, batch: int = 32,
                   threads: int = 8) -> int:
    """Image_re-binning.py:25-58 over a local tree: every image under root/image_folder goes to
    the same relative key with 'Image' -> 'Image_binned'.  Returns the number processed."""
    from .device import Device
    dev = dev or Device(0)
    if not image_folder.endswith("/"):
        image_folder += "/"
    keys = []
    base = os.path.join(root, image_folder)
    for dp, _, files in os.walk(base):
        for f in sorted(files):
            if f.lower().endswith(VALID_EXTENSIONS):
                keys.append(os.path.relpath(os.path.join(dp, f), root))
    keys.sort()

    def load(k):
        # Image_re-binning.py:56-58: a file that fails is logged and skipped, the loop continues
        try:
            with open(os.path.join(root, k), "rb") as fh:
                return _decode(fh.read())
        except Exception:  # noqa: BLE001
            log.error("Failed to process '%s'", k, exc_info=True)
            return None

    n = 0
    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        for i in range(0, len(keys), batch):
            chunk = keys[i:i + batch]
            planes = list(ex.map(load, chunk))
            shapes = {p.shape for p in planes if p is not None}
            groups = {s: [j for j, p in enumerate(planes) if p is not None and p.shape == s] for s in shapes}
            for s, idx in groups.items():
                out = rebin_planes(dev, np.stack([planes[j] for j in idx]), resolution, resolution)
                host = out.cpu().numpy().view(np.uint16)
                blobs = list(ex.map(_encode, [host[t] for t in range(len(idx))]))
                for t, j in enumerate(idx):
                    dst = os.path.join(root, chunk[j].replace("Image", "Image_binned"))
                    os.makedirs(os.path.dirname(dst), exist_ok=True)
                    with open(dst, "wb") as fh:
                        fh.write(blobs[t])
                    n += 1
    log.info("processed %d images", n)
    return n


def main(argv=None):
    ap = argparse.ArgumentParser(description="Re-bin the images of a folder (GPU LANCZOS resize).")
    ap.add_argument("--bucket_name", default=".", help="local root standing in for the S3 bucket")
    ap.add_argument("--image_folder", required=True)
    ap.add_argument("--resolution", type=int, default=1080)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    from .device import Device
    process_images(a.bucket_name, a.image_folder, a.resolution, dev=Device(a.device))


if __name__ == "__main__":
    main()

"""Minimal baseline-TIFF reader/writer for the host side of the pipeline.

The reference reads planes with ``tifffile.imread`` (Illumination_QC_mult.py:145,
Cellpose_GPU_s3fs.py:72,81) / ``imageio.imread`` (MaxProjection.py:39) and writes the
projection with ``imageio.imwrite(..., format='tiff')`` (MaxProjection.py:48): an uncompressed,
single-strip, minisblack little-endian TIFF.  Neither tifffile nor imageio is part of this
image, so this module decodes uncompressed strip/tile-free TIFFs directly with numpy (the
microscope / CellProfiler common case) and falls back to Pillow for compressed files; the
writer emits the same tag set the reference's imageio/tifffile writer produces.
"""
from __future__ import annotations

import io
import json
import struct

import numpy as np

_TYPES = {1: ("B", 1), 2: ("s", 1), 3: ("H", 2), 4: ("I", 4), 5: ("II", 8), 6: ("b", 1),
          7: ("B", 1), 8: ("h", 2), 9: ("i", 4), 11: ("f", 4), 12: ("d", 8), 16: ("Q", 8)}


def _read_ifd(buf: bytes, off: int, bo: str) -> dict:
    n = struct.unpack(bo + "H", buf[off:off + 2])[0]
    tags = {}
    for i in range(n):
        e = off + 2 + 12 * i
        tag, typ, cnt = struct.unpack(bo + "HHI", buf[e:e + 8])
        fmt, size = _TYPES.get(typ, ("B", 1))
        total = size * cnt
        data = buf[e + 8:e + 12] if total <= 4 else buf[struct.unpack(bo + "I", buf[e + 8:e + 12])[0]:][:total]
        if typ == 2:
            tags[tag] = data[:cnt].rstrip(b"\0").decode("latin-1")
        elif typ == 5:
            v = struct.unpack(bo + "I" * (2 * cnt), data[:total])
            tags[tag] = tuple(v[k] / v[k + 1] if v[k + 1] else 0.0 for k in range(0, 2 * cnt, 2))
        else:
            tags[tag] = struct.unpack(bo + fmt * cnt, data[:total])
    return tags


def imread(src) -> np.ndarray:
    """Decode the first page of a TIFF (path, bytes or binary file object) to a numpy array."""
    if isinstance(src, (bytes, bytearray, memoryview)):
        buf = bytes(src)
    elif hasattr(src, "read"):
        buf = src.read()
    else:
        with open(src, "rb") as f:
            buf = f.read()
    if buf[:2] not in (b"II", b"MM"):
        raise ValueError("not a TIFF file")
    bo = "<" if buf[:2] == b"II" else ">"
    if struct.unpack(bo + "H", buf[2:4])[0] != 42:
        raise ValueError("BigTIFF/unknown TIFF version not supported")
    tags = _read_ifd(buf, struct.unpack(bo + "I", buf[4:8])[0], bo)
    W, H = tags[256][0], tags[257][0]
    bits = tags.get(258, (1,))[0]
    comp = tags.get(259, (1,))[0]
    spp = tags.get(277, (1,))[0]
    fmt = tags.get(339, (1,))[0]
    if comp != 1 or spp != 1 or 273 not in tags or 322 in tags:
        return _pil_read(buf)
    kind = {1: "u", 2: "i", 3: "f"}.get(fmt, "u")
    dt = np.dtype(f"{bo}{kind}{bits // 8}")
    offs, counts = tags[273], tags.get(279, (W * H * dt.itemsize,))
    raw = b"".join(buf[o:o + c] for o, c in zip(offs, counts))
    arr = np.frombuffer(raw, dtype=dt, count=W * H).reshape(H, W)
    return arr.astype(dt.newbyteorder("="), copy=True)


def read_into(path: str, out: np.ndarray) -> None:
    """Decode the first page of the TIFF at `path` into `out` (a writable C-contiguous 2-D array,
    e.g. a slice of a pinned staging buffer).  Uncompressed strips whose sample type and byte
    order match `out` are read straight from the file into `out` (readinto: no intermediate
    copies, the GIL released during the reads); anything else goes through imread and a copy.
    Raises ValueError on a shape mismatch."""
    with open(path, "rb") as f:
        head = f.read(65536)
        if head[:2] not in (b"II", b"MM"):
            raise ValueError(f"{path}: not a TIFF file")
        bo = "<" if head[:2] == b"II" else ">"
        if struct.unpack(bo + "H", head[2:4])[0] != 42:
            raise ValueError(f"{path}: BigTIFF/unknown TIFF version not supported")
        ifd = struct.unpack(bo + "I", head[4:8])[0]
        tags = None
        if ifd + 2 <= len(head):
            n = struct.unpack(bo + "H", head[ifd:ifd + 2])[0]
            if ifd + 2 + 12 * n + 4 <= len(head):
                try:
                    tags = _read_ifd(head, ifd, bo)
                except struct.error:
                    tags = None
        direct = False
        if tags is not None and 256 in tags and 257 in tags and 273 in tags:
            W, H = tags[256][0], tags[257][0]
            bits = tags.get(258, (1,))[0]
            kind = {1: "u", 2: "i", 3: "f"}.get(tags.get(339, (1,))[0], "u")
            dt = np.dtype(f"{bo}{kind}{bits // 8}")
            direct = (tags.get(259, (1,))[0] == 1 and tags.get(277, (1,))[0] == 1 and 322 not in tags
                      and dt.newbyteorder("=") == out.dtype and dt.isnative and out.flags.c_contiguous
                      and len(tags.get(279, ())) == len(tags[273]))
            if (H, W) != out.shape:
                raise ValueError(f"{path}: shape {(H, W)}, expected {out.shape}")
        if direct:
            mv = memoryview(out.reshape(-1).view(np.uint8))
            pos = 0
            for o, c in zip(tags[273], tags[279]):
                c = min(c, out.nbytes - pos)
                f.seek(o)
                got = f.readinto(mv[pos:pos + c])
                if got != c:
                    raise ValueError(f"{path}: truncated strip")
                pos += c
            if pos != out.nbytes:
                raise ValueError(f"{path}: strips hold {pos} of {out.nbytes} bytes")
            return
    arr = imread(path)
    if arr.shape != out.shape:
        raise ValueError(f"{path}: shape {arr.shape}, expected {out.shape}")
    out[...] = arr


def _pil_read(buf: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(buf)) as im:
        return np.array(im)


def imwrite_bytes(arr: np.ndarray) -> bytes:
    """Uncompressed single-strip minisblack TIFF with the tag set of imageio/tifffile's writer
    (MaxProjection.py:47-48): 256,257,258,259=1,262=1,270 shape JSON,273,277,278,279,
    282/283=1/1,296=1,305='tifffile.py'."""
    arr = np.ascontiguousarray(arr)
    if arr.ndim != 2:
        raise ValueError("2-D planes only")
    H, W = arr.shape
    kind = {"u": 1, "i": 2, "f": 3}[arr.dtype.kind]
    bits = arr.dtype.itemsize * 8
    desc = json.dumps({"shape": [H, W]}).encode() + b"\0"
    soft = b"tifffile.py\0"
    entries = []
    ntag = 14 + (1 if kind != 1 else 0)
    ifd_off = 8
    data_off = ifd_off + 2 + 12 * ntag + 4
    extra = bytearray()

    def put(blob: bytes) -> int:
        nonlocal extra
        o = data_off + len(extra)
        extra += blob
        if len(extra) % 2:
            extra += b"\0"
        return o

    o_desc = put(desc + b"\0" * 16)  # tifffile reserves 16 spare bytes after the shape JSON
    o_xres = put(struct.pack("<II", 1, 1))
    o_yres = put(struct.pack("<II", 1, 1))
    o_soft = put(soft)
    img_off = ((data_off + len(extra) + 15) // 16) * 16
    nbytes = arr.nbytes
    entries = [(256, 4, 1, W), (257, 4, 1, H), (258, 3, 1, bits), (259, 3, 1, 1), (262, 3, 1, 1),
               (270, 2, len(desc), o_desc), (273, 4, 1, img_off), (277, 3, 1, 1), (278, 4, 1, H),
               (279, 4, 1, nbytes), (282, 5, 1, o_xres), (283, 5, 1, o_yres), (296, 3, 1, 1),
               (305, 2, len(soft), o_soft)]
    if kind != 1:
        entries.append((339, 3, 1, kind))
    entries.sort()
    out = bytearray(b"II*\0" + struct.pack("<I", ifd_off))
    out += struct.pack("<H", len(entries))
    for tag, typ, cnt, val in entries:
        if typ == 3 and cnt == 1:
            out += struct.pack("<HHIHH", tag, typ, cnt, val, 0)
        else:
            out += struct.pack("<HHII", tag, typ, cnt, val)
    out += struct.pack("<I", 0)
    out += extra
    out += b"\0" * (img_off - len(out))
    out += arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
    return bytes(out)


def imwrite(path: str, arr: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(imwrite_bytes(arr))

"""cpx.tiffio against the reference's own files (CPU): the max-projection TIFF written by the
reference (tests/golden/maxproj.npz, imageio/tifffile 2021.7.2) is reproduced byte for byte and
the QC fixture planes decode to the arrays the reference read."""
import os

import numpy as np

from cpx import tiffio


def test_writer_matches_reference_bytes(golden_dir):
    d = np.load(os.path.join(golden_dir, "maxproj.npz"))
    assert tiffio.imwrite_bytes(d["expected"]) == d["expected_tiff"].tobytes()


def test_reader_roundtrip(golden_dir):
    d = np.load(os.path.join(golden_dir, "maxproj.npz"))
    b = d["expected_tiff"].tobytes()
    import io
    np.testing.assert_array_equal(tiffio.imread(io.BytesIO(b)), d["expected"])
    for z in range(5):
        p = d[f"plane{z}"]
        np.testing.assert_array_equal(tiffio.imread(io.BytesIO(tiffio.imwrite_bytes(p))), p)


def test_reads_qc_cli_planes(golden_dir):
    folder = os.path.join(golden_dir, "qc_cli", "images")
    names = sorted(os.listdir(folder))
    assert names
    for n in names:
        a = tiffio.imread(os.path.join(folder, n))
        assert a.dtype == np.uint16 and a.shape == (96, 120)


def test_read_into_matches_imread(tmp_path):
    """tiffio.read_into (strips read straight into a staging buffer) == imread, for the
    uncompressed u16 case and the fallback path (other dtype), and a shape mismatch raises."""
    import numpy as np
    import pytest
    from cpx import tiffio
    rng = np.random.default_rng(3)
    a = rng.integers(0, 65536, (300, 257), dtype=np.uint16)
    p = tmp_path / "a.tiff"
    tiffio.imwrite(str(p), a)
    out = np.full((300, 257), 7, np.uint16)
    tiffio.read_into(str(p), out)
    np.testing.assert_array_equal(out, a)
    f = rng.standard_normal((40, 50)).astype(np.float32)
    tiffio.imwrite(str(tmp_path / "f.tiff"), f)
    of = np.zeros((40, 50), np.float32)
    tiffio.read_into(str(tmp_path / "f.tiff"), of)
    np.testing.assert_array_equal(of, f)
    with pytest.raises(ValueError):
        tiffio.read_into(str(p), np.zeros((300, 256), np.uint16))


def test_read_into_fallback_paths(tmp_path):
    """read_into's imread-and-cast fallback: an 8-bit plane, a big-endian 16-bit plane and an
    LZW-compressed 16-bit plane (written by Pillow) land in a uint16 staging buffer exactly as
    imread(...).astype(np.uint16)."""
    import struct
    from PIL import Image
    rng = np.random.default_rng(8)
    a8 = rng.integers(0, 256, (33, 47), dtype=np.uint8)
    tiffio.imwrite(str(tmp_path / "u8.tiff"), a8)
    out = np.full((33, 47), 9, np.uint16)
    tiffio.read_into(str(tmp_path / "u8.tiff"), out)
    np.testing.assert_array_equal(out, tiffio.imread(str(tmp_path / "u8.tiff")).astype(np.uint16))
    np.testing.assert_array_equal(out, a8.astype(np.uint16))
    # big-endian: the little-endian file with its header and sample bytes swapped
    a16 = rng.integers(0, 65536, (21, 30), dtype=np.uint16)
    le = tiffio.imwrite_bytes(a16)
    ifd = struct.unpack("<I", le[4:8])[0]
    n = struct.unpack("<H", le[ifd:ifd + 2])[0]
    be = bytearray(b"MM" + struct.pack(">H", 42) + struct.pack(">I", ifd))
    be += le[8:ifd] + struct.pack(">H", n)
    img_off = None
    for i in range(n):
        e = ifd + 2 + 12 * i
        tag, typ, cnt = struct.unpack("<HHI", le[e:e + 8])
        if typ == 3 and cnt == 1:
            val = struct.unpack("<H", le[e + 8:e + 10])[0]
            be += struct.pack(">HHIHH", tag, typ, cnt, val, 0)
        else:
            val = struct.unpack("<I", le[e + 8:e + 12])[0]
            be += struct.pack(">HHII", tag, typ, cnt, val)
            if tag == 273:
                img_off = val
            if typ == 5:  # rationals live in the data area: swap them there too
                be_data = struct.pack(">II", *struct.unpack("<II", le[val:val + 8]))
                le = le[:val] + be_data + le[val + 8:]
    be += le[ifd + 2 + 12 * n:img_off]
    be += a16.astype(">u2").tobytes()
    (tmp_path / "be.tiff").write_bytes(bytes(be))
    out = np.zeros((21, 30), np.uint16)
    tiffio.read_into(str(tmp_path / "be.tiff"), out)
    np.testing.assert_array_equal(out, a16)
    # LZW-compressed 16-bit (Pillow/libtiff)
    Image.fromarray(a16).save(str(tmp_path / "lzw.tiff"), compression="tiff_lzw")
    out = np.zeros((21, 30), np.uint16)
    tiffio.read_into(str(tmp_path / "lzw.tiff"), out)
    np.testing.assert_array_equal(out, a16)

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

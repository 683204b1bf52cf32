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

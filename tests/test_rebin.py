"""Image re-binning (Image_re-binning.py:12-22).

Golden vectors: tests/golden/rebin_cases.npz, made by tools/make_golden_rebin.py from the
reference function itself (Pillow 12.2.0).  CPU tests pin the restatement oracle/rebin_oracle.py;
GPU tests check libcpx cpx_rebin_u16 bit-exactly against the same vectors.
"""
import hashlib
import io
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import rebin_oracle as ro  # noqa: E402
import synth_golden as sg  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden", "rebin_cases.npz")
N_SMALL = 6


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).astype("<u2").tobytes()).hexdigest()


@pytest.mark.parametrize("i", range(N_SMALL))
def test_oracle_matches_reference_small(gold, i):
    r = int(gold[f"res_{i}"])
    assert np.array_equal(ro.resize_lanczos_u16(gold[f"in_{i}"], r, r), gold[f"out_{i}"])


def test_oracle_matches_reference_full_size(gold):
    seed, H, W, r = (int(v) for v in gold["full_seed"])
    got = ro.resize_lanczos_u16(sg.plane(seed, H, W, n_blobs=300), r, r)
    assert np.array_equal(got[::97], gold["full_out_rows"])
    assert _sha(got) == str(gold["full_sha256"])


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(N_SMALL))
def test_gpu_rebin_bit_exact(dev, gold, i):
    from cpx.rebin import rebin_planes
    a, r = gold[f"in_{i}"], int(gold[f"res_{i}"])
    out = rebin_planes(dev, a[None], r, r).cpu().numpy().view(np.uint16)[0]
    assert np.array_equal(out, gold[f"out_{i}"])


@pytest.mark.gpu
def test_gpu_rebin_full_size_batch(dev, gold):
    """2080^2 -> 1080^2 for a batch of planes (the golden one twice, plus a different plane)."""
    from cpx.rebin import rebin_planes
    seed, H, W, r = (int(v) for v in gold["full_seed"])
    a = sg.plane(seed, H, W, n_blobs=300)
    b = sg.plane(seed + 1, H, W, n_blobs=100)
    out = rebin_planes(dev, np.stack([a, b, a]), r, r).cpu().numpy().view(np.uint16)
    assert _sha(out[0]) == str(gold["full_sha256"]) and _sha(out[2]) == str(gold["full_sha256"])
    assert np.array_equal(out[1][::5, ::5], ro.resize_lanczos_u16(b, r, r)[::5, ::5])


@pytest.mark.gpu
def test_process_image_in_memory_bytes_identical(dev, gold):
    """The whole reference function: TIFF bytes in -> LZW TIFF bytes out, byte-identical."""
    from cpx.rebin import process_image_in_memory
    r = int(gold["res_0"])
    out = process_image_in_memory(gold["in_bytes_0"].tobytes(), target_size=(r, r), dev=dev)
    assert out == gold["out_bytes_0"].tobytes()


@pytest.mark.gpu
def test_rebin_cli_tree(dev, gold, tmp_path):
    """Image_re-binning.py:25-58 over a local tree: keys with 'Image' -> 'Image_binned'."""
    from PIL import Image
    from cpx.rebin import process_images
    src = tmp_path / "exp" / "Images" / "r01c01"
    src.mkdir(parents=True)
    for i in (0, 2):
        Image.fromarray(gold[f"in_{i}"]).save(str(src / f"plane{i}.tiff"), format="tiff")
    (src / "notes.txt").write_text("skip me")
    n = process_images(str(tmp_path), "exp/Images", 64, dev=dev)
    assert n == 2
    for i in (0, 2):
        out = np.array(Image.open(str(tmp_path / "exp" / "Image_binneds" / "r01c01" / f"plane{i}.tiff")))
        assert np.array_equal(out, ro.resize_lanczos_u16(gold[f"in_{i}"], 64, 64))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,oh,ow", [(400, 360, 40, 36),     # ksize > 32: two-pass kernels
                                      (130, 97, 70, 33),      # fused, non-square, odd
                                      (61, 300, 61, 75),      # horizontal only
                                      (300, 61, 75, 61),      # vertical only
                                      (45, 600, 170, 510),    # fused, up x / down y... mixed
                                      (1100, 700, 530, 1000)])  # fused, several tiles both axes
def test_gpu_rebin_paths_vs_oracle(dev, H, W, oh, ow):
    """Every kernel path (fused tile kernel, two-pass fallbacks) against the oracle."""
    from cpx.rebin import rebin_planes
    rng = np.random.default_rng(H * 7 + W)
    a = np.stack([rng.integers(0, 65536, (H, W), dtype=np.uint16),
                  sg.plane(5, H, W, n_blobs=20)])
    out = rebin_planes(dev, a, oh, ow).cpu().numpy().view(np.uint16)
    for g in range(2):
        assert np.array_equal(out[g], ro.resize_lanczos_u16(a[g], ow, oh)), g

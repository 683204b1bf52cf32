"""CPU: the Cells marker-watershed oracle (oracle/ws_oracle.py, ws_oracle_c.c) against
scikit-image 0.18.3's own outputs (tests/golden/watershed_cases.npz, tools/make_golden_ws.py),
and the parallel characterisation the HIP kernel computes (`watershed_minimax`) against both."""
import numpy as np
import pytest

import cpx_oracle as orc
import ws_oracle as wo


@pytest.fixture(scope="module")
def golden(golden_dir):
    import os
    return np.load(os.path.join(golden_dir, "watershed_cases.npz"))


@pytest.mark.parametrize("impl", ["c", "py"])
def test_generic_flood_matches_skimage(golden, impl):
    for n in golden["names_generic"]:
        mask = golden[f"{n}_mask"] if golden[f"{n}_has_mask"] else None
        got = wo.watershed(golden[f"{n}_image"], golden[f"{n}_markers"], mask, impl=impl)
        np.testing.assert_array_equal(got, golden[f"{n}_out"], err_msg=str(n))


def test_cells_watershed_matches_skimage(golden):
    d = int(golden["distance"])
    for n in golden["names_cells"]:
        nuc, corr = golden[f"{n}_nuclei"], golden[f"{n}_corr"]
        cells, cyto = wo.cells_watershed(nuc, corr, d)
        np.testing.assert_array_equal(cells, golden[f"{n}_cells"], err_msg=str(n))
        np.testing.assert_array_equal(cyto, np.where(nuc == 0, cells, 0))
        # the watershed is not the Voronoi expansion: boundaries between touching cells move
        assert (cells != orc.expand_labels(nuc, d)).any()


def test_minimax_form_equals_heap_flood(golden):
    d = int(golden["distance"])
    for n in golden["names_cells"]:
        nuc, corr = golden[f"{n}_nuclei"], golden[f"{n}_corr"]
        foot = orc.expand_labels(nuc, d) > 0
        got = wo.watershed_minimax(wo.elevation_key(corr), nuc, foot)
        np.testing.assert_array_equal(got, golden[f"{n}_cells"], err_msg=str(n))


def test_minimax_form_random_cases():
    rng = np.random.default_rng(3)
    for case in range(20):
        H, W = rng.integers(5, 60, 2)
        corr = rng.integers(0, 5, (H, W)).astype(np.float32) * 1000  # heavy 16-bit ties
        nuc = np.zeros((H, W), np.int32)
        for lab in range(1, rng.integers(1, 8)):
            y, x = rng.integers(0, H), rng.integers(0, W)
            nuc[y:y + rng.integers(1, 4), x:x + rng.integers(1, 4)] = lab
        mask = rng.random((H, W)) < 0.85
        key = wo.elevation_key(corr)
        ref = wo.watershed(key.astype(np.float64), nuc, mask, impl="py")
        np.testing.assert_array_equal(wo.watershed(key.astype(np.float64), nuc, mask, impl="c"), ref)
        np.testing.assert_array_equal(wo.watershed_minimax(key, nuc, mask), ref, err_msg=f"case {case}")


def test_quantise_edges():
    v = np.array([np.nan, np.inf, -np.inf, -1.0, 0.0, 0.99, 1.0, 65534.99, 65535.0, 1e9], np.float32)
    np.testing.assert_array_equal(wo.quantise(v), [65535, 65535, 0, 0, 0, 0, 1, 65534, 65535, 65535])
    with pytest.raises(ValueError):
        wo.elevation_key(np.zeros((4096, 4096), np.float32))

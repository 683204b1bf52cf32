"""End-to-end plate run (cpx.plate): LoadData + TIFFs -> <out>/<plate>/<time>/ four CSV tables,
consistent with the batch pipeline and the per-FOV QC session on the same planes."""
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def test_plate_run_tables(tmp_path, dev):
    import torch
    from cpx import plate, tiffio
    from cpx.csvout import OBJECT_TABLES, feature_names
    from cpx.synth import synth_fovs, synth_illum
    n, C, H, W = 3, 2, 384, 416
    chans = ["DNA", "AGP"]
    raw = synth_fovs(n, C, H, W, dev.torch_device, seed=5).cpu().numpy().view(np.uint16)
    imgdir = tmp_path / "images"
    imgdir.mkdir()
    rows = []
    for f in range(n):
        row = {"Metadata_Plate": "P07", "Metadata_Well": f"B{f + 1:02d}", "Metadata_Site": 1,
               "Metadata_Timepoint": 48, "Metadata_Compound": "cmpd", "Metadata_ConcLevel": 1}
        for c, ch in enumerate(chans):
            name = f"r02c{f + 1:02d}f01p01-ch{c + 1}.tiff"
            tiffio.imwrite(str(imgdir / name), raw[f * C + c])
            row[f"FileName_{ch}"] = name
        rows.append(row)
    ld = tmp_path / "load_data.csv"
    pd.DataFrame(rows).to_csv(ld, index=False)
    ill = tmp_path / "illum"
    ill.mkdir()
    np.save(ill / "DNA_illum.npy", synth_illum(1, H, W, seed=3)[0].astype(np.float32))
    d = plate.run(["--load-data", str(ld), "--data-path", str(imgdir), "--illum-path", str(ill),
                   "--channels", *chans, "--out", str(tmp_path / "out"), "--batch", "2", "--threads", "4"])
    assert d == str(tmp_path / "out" / "P07" / "48")
    img = pd.read_csv(os.path.join(d, "Image.csv"), float_precision="round_trip")
    assert img["ImageNumber"].tolist() == [1, 2, 3]
    assert img["Metadata_Well"].tolist() == ["B01", "B02", "B03"]
    for s in OBJECT_TABLES:
        o = pd.read_csv(os.path.join(d, f"{s}.csv"))
        assert list(o.columns[3:]) == feature_names(chans)
        counts = o.groupby("ImageNumber").size().reindex([1, 2, 3], fill_value=0).tolist()
        assert counts == img[f"Count_{s}"].tolist(), s
        assert (o["AreaShape_Area"] > 0).all()
    assert img["Count_Nuclei"].sum() > 0
    # QC columns == the per-FOV session on the same planes and flat-fields
    from cpx import qc
    s = qc.session()
    s.set_illum(0, np.load(ill / "DNA_illum.npy"))
    s.set_illum(1, None)
    for f in range(n):
        s.submit([raw[f * C], raw[f * C + 1]], C=2)
        slope, pct, _ = s.qc()
        np.testing.assert_allclose(img.loc[f, ["ImageQuality_PowerLogLogSlope_DNA",
                                               "ImageQuality_PowerLogLogSlope_AGP"]].to_numpy(float),
                                   slope, rtol=1e-12)
        np.testing.assert_array_equal(img.loc[f, ["ImageQuality_PercentMaximal_DNA",
                                                  "ImageQuality_PercentMaximal_AGP"]].to_numpy(float), pct)

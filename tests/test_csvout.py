"""Table layout of cpx.csvout (CPU): the four CSVs Pycyto_pertime.py:46-75 reads."""
import numpy as np
import pandas as pd

from cpx.csvout import OBJECT_TABLES, PlateTables, feature_names


def test_feature_names_layout():
    names = feature_names(["DNA", "AGP"])
    assert len(names) == 15 + 2 * 29
    assert names[0] == "AreaShape_Area" and names[15] == "Intensity_IntegratedIntensity_DNA"
    assert names[20] == "Texture_Contrast_DNA_3_00_256"
    assert names[-1] == "Texture_Correlation_AGP_3_03_256"
    assert len(set(names)) == len(names)


def test_plate_tables_roundtrip(tmp_path):
    chans = ["DNA", "AGP"]
    t = PlateTables(chans)
    F = len(feature_names(chans))
    rng = np.random.default_rng(0)
    # images added out of order (batches finish in any order): output sorted by ImageNumber
    for img, n in ((2, 3), (1, 2)):
        t.add_image(img, {"Metadata_Plate": "P01", "Metadata_Well": f"A0{img}", "Metadata_Site": 1,
                          "Metadata_Timepoint": 24, "FileName_DNA": "x.tiff"},
                    [-1.5, -2.0], [0.01, 0.02], {s: n for s in OBJECT_TABLES})
        for s in OBJECT_TABLES:
            t.add_objects(s, img, np.arange(n, 0, -1), rng.normal(size=(n, F)))
    d = t.write(str(tmp_path), "P01", 24)
    img = pd.read_csv(f"{d}/Image.csv")
    assert img["ImageNumber"].tolist() == [1, 2]
    assert "FileName_DNA" not in img.columns
    assert {"Metadata_Plate", "Metadata_Well", "ImageQuality_PowerLogLogSlope_DNA",
            "ImageQuality_PercentMaximal_AGP", "Count_Nuclei", "Count_Cytoplasm"} <= set(img.columns)
    for s in OBJECT_TABLES:
        o = pd.read_csv(f"{d}/{s}.csv")
        assert list(o.columns[:3]) == ["ImageNumber", "ObjectNumber", "Number_Object_Number"]
        assert list(o.columns[3:]) == feature_names(chans)
        assert o[["ImageNumber", "ObjectNumber"]].values.tolist() == [[1, 1], [1, 2], [2, 1], [2, 2], [2, 3]]
        # the merge Pycyto_pertime.py:53-58 performs
        m = o.merge(img[["ImageNumber", "Metadata_Plate", "Metadata_Well"]], on="ImageNumber", how="left")
        assert m["Metadata_Well"].tolist() == ["A01", "A01", "A02", "A02", "A02"]

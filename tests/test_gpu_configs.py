"""BASELINE configs[2] at test scale: one plate x 4 timepoints, 4 FOVs per well, the wells
sharded over two ranks (cpx.launch, both ranks on the one test GPU) -> <out>/<plate>/<time>/
{Image,Nuclei,Cells,Cytoplasm}.csv byte-identical to one process, then the per-time profiles
(cpx.profiles = Pycyto_pertime.py:29-172) over the four timepoints of the sharded output.

Reference: Feature_extraction_opt.py:63-76,147-178 (one job per (plate, time)), Cellpose_GPU_s3fs.py
:269-300 (one consumer per GPU), Pycyto_pertime.py:29-172 (per-time profiles of those tables)."""
import filecmp
import os

import numpy as np
import pandas as pd
import pytest

from cpx import plate
from cpx.csvout import OBJECT_TABLES

TIMES = [6, 12, 24, 48]
WELLS = [f"B{w:02d}" for w in range(1, 9)]
SITES = 4
CHANS = ["DNA", "AGP"]


def _compound(wi):
    """every 4th well DMSO (the normalisation controls), the rest cycle through three compounds"""
    return ("DMSO", 0) if wi % 4 == 0 else (["CmpA", "CmpB", "CmpC"][wi % 3], 1 + wi % 2)


@pytest.mark.gpu
def test_config2_plate_times_two_ranks_then_profiles(tmp_path, dev):
    from cpx import launch, profiles, tiffio
    from cpx.synth import synth_fovs
    C, H, W = len(CHANS), 384, 416
    imgdir = tmp_path / "images"
    imgdir.mkdir()
    lds = []
    for t in TIMES:
        n = len(WELLS) * SITES
        raw = synth_fovs(n, C, H, W, dev.torch_device, seed=100 + t).cpu().numpy().view(np.uint16)
        rows = []
        for wi, well in enumerate(WELLS):
            cmpd, conc = _compound(wi)
            for s in range(SITES):
                f = wi * SITES + s
                row = {"Metadata_Plate": "P01", "Metadata_Well": well, "Metadata_Site": s + 1,
                       "Metadata_Timepoint": t, "Metadata_Compound": cmpd, "Metadata_ConcLevel": conc}
                for c, ch in enumerate(CHANS):
                    name = f"t{t}_f{f}_c{c}.tiff"
                    tiffio.imwrite(str(imgdir / name), raw[f * C + c])
                    row[f"FileName_{ch}"] = name
                rows.append(row)
        ld = tmp_path / f"ld_t{t}.csv"
        pd.DataFrame(rows).to_csv(ld, index=False)
        lds.append(str(ld))
    common = ["--load-data", *lds, "--data-path", str(imgdir), "--channels", *CHANS,
              "--batch", "8", "--threads", "4", "--pipes", "1"]
    one = plate.run(common + ["--out", str(tmp_path / "one"), "--world", "1", "--rank", "0"])
    two = launch.main(["--gpus", "2", "--devices", "0,0", "--", *common, "--out", str(tmp_path / "two")])
    assert [os.path.relpath(d, tmp_path / "one") for d in one] == [f"P01/{t}" for t in TIMES]
    assert [os.path.relpath(d, tmp_path / "two") for d in two] == [f"P01/{t}" for t in TIMES]
    for d1, d2 in zip(one, two):
        for name in ("Image", *OBJECT_TABLES, "site_status"):
            assert filecmp.cmp(os.path.join(d1, f"{name}.csv"), os.path.join(d2, f"{name}.csv"),
                               shallow=False), (d1, name)
        img = pd.read_csv(os.path.join(d2, "Image.csv"))
        assert len(img) == len(WELLS) * SITES
        assert (pd.read_csv(os.path.join(d2, "Nuclei.csv")).groupby("ImageNumber").size() > 0).all()
    # per-time profiles of the sharded plate (Pycyto_pertime.py over the four timepoints)
    written = profiles.concatenate_csv(str(tmp_path / "two"), [str(t) for t in TIMES], "P01",
                                       str(tmp_path / "prof"), "P01_profiles",
                                       local_dir=str(tmp_path / "tmp"))
    assert len(written) == 3 * len(TIMES)
    for t in TIMES:
        base = tmp_path / "prof" / "P01_profiles" / str(t)
        sel = pd.read_csv(base / "CP_features_selected.csv")
        assert len(sel) == len(WELLS) and sel.columns[0] == "Metadata_Plate"
        avg = pd.read_csv(base / "CPfeatures_average_cosine_similarity.csv")
        assert set(avg.Metadata_compound_code) == {"DMSO", "CmpA", "CmpB", "CmpC"}

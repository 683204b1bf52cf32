"""a5 host drop-in (cpx.maxproj) vs MaxProjection.py's contract: path rewrite, CSV sniffing,
plate / chunk / group formation (CPU), and the GPU projection + TIFF bytes vs the reference
golden, the CLI end to end on a local S3 stand-in, and a configs[4]-sized z-stack (GPU)."""
import io
import json
import os

import numpy as np
import pandas as pd
import pytest

from cpx import maxproj, tiffio


def _meta(golden_dir):
    with open(os.path.join(golden_dir, "maxproj.json")) as f:
        return json.load(f)


def test_modify_imagepath_matches_reference(golden_dir):
    m = _meta(golden_dir)
    for src, exp in m["modify_imagepath"].items():
        assert maxproj.modify_imagepath(src) == exp
    assert maxproj.modify_imagepath(m["keys"][0]) == m["out_key"]


def _plate_df(plates=("P1", "P2"), C=2, Z=3, sites=2, extra=1):
    rows = []
    for pl in plates:
        for s in range(sites):
            for z in range(Z):
                for c in range(C):
                    rows.append(dict(PlateID=pl, Image_PathName=f"{pl}/Images",
                                     Image_FileName=f"s{s}p{z + 1}c{c + 1}.tiff", FieldID=s, PlaneID=z + 1,
                                     ChannelID=c + 1))
        for e in range(extra):  # an incomplete trailing chunk
            rows.append(dict(PlateID=pl, Image_PathName=f"{pl}/Images", Image_FileName=f"x{e}.tiff",
                             FieldID=99, PlaneID=1, ChannelID=1))
    return pd.DataFrame(rows)


def test_chunk_groups_plane_major_and_incomplete_skipped(caplog):
    df = _plate_df()
    out = list(maxproj.chunk_groups(df, 2, 3))
    assert [(p, i) for p, i, _ in out] == [("P1", 0), ("P1", 6), ("P2", 0), ("P2", 6)]
    _, _, groups = out[1]
    assert groups[0] == [f"P1/Images/s1p{z}c1.tiff" for z in (1, 2, 3)]
    assert groups[1] == [f"P1/Images/s1p{z}c2.tiff" for z in (1, 2, 3)]
    assert sum("Skipping incomplete chunk" in r.message for r in caplog.records) == 2


def test_read_csv_sniffs_semicolons(tmp_path):
    s3 = maxproj.LocalS3(str(tmp_path))
    df = _plate_df(plates=("P1",), sites=1, extra=0)
    buf = io.BytesIO(df.to_csv(index=False, sep=";").encode())
    s3.upload_fileobj(buf, "meta", "sets/plate.csv")
    got = maxproj.read_csv_from_s3("meta", "sets/plate.csv", s3)
    pd.testing.assert_frame_equal(got, df)


@pytest.mark.gpu
def test_max_projection_matches_reference_golden(dev, golden_dir, tmp_path):
    d = np.load(os.path.join(golden_dir, "maxproj.npz"))
    m = _meta(golden_dir)
    s3 = maxproj.LocalS3(str(tmp_path))
    for z, k in enumerate(m["keys"]):
        s3.upload_fileobj(io.BytesIO(tiffio.imwrite_bytes(d[f"plane{z}"])), "bkt", k)
    maxproj.max_projection(m["keys"], "bkt", s3)
    data = s3.get_object(Bucket="bkt", Key=m["out_key"])["Body"].read()
    assert data == d["expected_tiff"].tobytes()


@pytest.mark.gpu
def test_max_projection_shape_mismatch_raises(dev, tmp_path):
    s3 = maxproj.LocalS3(str(tmp_path))
    keys = ["a/Images/1.tiff", "a/Images/2.tiff"]
    s3.upload_fileobj(io.BytesIO(tiffio.imwrite_bytes(np.zeros((4, 5), np.uint16))), "b", keys[0])
    s3.upload_fileobj(io.BytesIO(tiffio.imwrite_bytes(np.zeros((5, 4), np.uint16))), "b", keys[1])
    with pytest.raises(ValueError, match="Image shape mismatch in group"):
        maxproj.max_projection(keys, "b", s3)


@pytest.mark.gpu
def test_cli_end_to_end_local_s3(dev, tmp_path, caplog):
    C, Z, H, W = 2, 3, 64, 80
    df = _plate_df(C=C, Z=Z)
    root = str(tmp_path)
    s3 = maxproj.LocalS3(root)
    rng = np.random.default_rng(0)
    planes = {}
    for _, r in df.iterrows():
        k = f"{r.Image_PathName}/{r.Image_FileName}"
        shape = (H, W + 2) if r.Image_FileName == "s1p2c2.tiff" and r.PlateID == "P2" else (H, W)
        a = rng.integers(0, 65536, shape, dtype=np.uint16)
        planes[k] = a
        s3.upload_fileobj(io.BytesIO(tiffio.imwrite_bytes(a)), "img", k)
    s3.upload_fileobj(io.BytesIO(df.to_csv(index=False).encode()), "meta", "set.csv")
    n = maxproj.main(["--bucket_data_set", "meta", "--data_set", "set.csv", "--channels", str(C),
                      "--planes", str(Z), "--bucket_images", "img", "--local-root", root])
    assert n == 7  # 4 chunks x 2 groups, one group with a shape mismatch
    assert any("Image shape mismatch" in r.message for r in caplog.records)
    for pl, i, groups in maxproj.chunk_groups(df, C, Z):
        for g in groups:
            out_key = maxproj.modify_imagepath(g[0])
            imgs = [planes[k] for k in g]
            if len({a.shape for a in imgs}) > 1:
                assert not os.path.exists(os.path.join(root, "img", *out_key.split("/")))
                continue
            got = s3.get_object(Bucket="img", Key=out_key)["Body"].read()
            assert got == tiffio.imwrite_bytes(np.maximum.reduce(imgs))


@pytest.mark.gpu
def test_zstack_configs4_size(dev):
    """configs[4] geometry: 2048^2 x 5 channels x 7 planes (plane-major) -> 5 projections."""
    from cpx.maxproj import session
    C, Z, H, W = 5, 7, 2048, 2048
    rng = np.random.default_rng(4)
    planes = [rng.integers(0, 65536, (H, W), dtype=np.uint16) for _ in range(C * Z)]
    s = session()
    for c in range(C):
        s.set_illum(c, None)
    s.submit(planes, C=C, Z=Z)
    for c in range(C):
        np.testing.assert_array_equal(s.read_plane(c), np.maximum.reduce([planes[z * C + c] for z in range(Z)]))

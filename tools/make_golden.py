"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code — test tooling.

Run in the survey container's python3.9 (numpy 1.26, scipy 1.7.1, skimage 0.18.3, tifffile,
imageio), which can import the reference scripts from /root/reference:

    /opt/conda/bin/python3.9 tools/make_golden.py            # QC / max-projection / skimage
    python tools/make_golden.py --cellpose-helpers            # scale_to_8bit (needs torch+PIL)

What is imported from the reference (unmodified, read-only):
  Illumination_QC_mult.py  rps / calculate_saturation_cp_exact / calculate_qc_metrics /
                           process_site / main (CLI run on a tiny LoadData set)
  MaxProjection.py         modify_imagepath / max_projection (boto3 stubbed, in-memory S3)
  Cellpose_GPU_s3fs.py     scale_to_8bit (tifffile stubbed)
plus scikit-image 0.18.3 regionprops / greycomatrix / greycoprops for the object table and the
feature definitions.  Only inputs and outputs are written (no reference source is copied).
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import tempfile
import types
import warnings

import numpy as np

warnings.filterwarnings("ignore")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))
import synth_golden as sg  # noqa: E402

sys.dont_write_bytecode = True


def _import_ref(name):
    if REF not in sys.path:
        sys.path.insert(0, REF)
    return __import__(name)


# ------------------------------------------------------------------------------------------
def gen_qc():
    qc = _import_ref("Illumination_QC_mult")
    cases = {}
    # small planes: several sizes / flat-field dtypes / edge cases
    specs = [
        ("s256_f32", 256, 256, "f32", 11), ("s520_f32", 520, 520, "f32", 12),
        ("s130x104_f64", 130, 104, "f64", 13), ("s208x260_none", 208, 260, "none", 14),
        ("s16_f32", 16, 16, "f32", 15), ("s64_zero", 64, 64, "zero", 16),
        ("s64_nan", 64, 64, "nan", 17), ("s256_sat", 256, 256, "sat", 18),
        ("s96_const", 96, 96, "const", 19),
    ]
    arrays = {}
    meta = {}
    for name, H, W, kind, seed in specs:
        raw = sg.plane(seed, H, W, n_blobs=12)
        ill = None
        if kind in ("f32", "sat", "nan"):
            ill = sg.illum(seed, H, W, np.float32)
        elif kind == "f64":
            ill = sg.illum(seed, H, W, np.float64)
        if kind == "zero":
            raw = np.zeros((H, W), np.uint16)
        if kind == "const":
            raw = np.full((H, W), 1234, np.uint16)
        if kind == "sat":
            raw[::7, ::5] = 65535
        if kind == "nan":
            raw[3, 3] = 0
            ill = ill.copy()
            ill[3, 3] = 0.0  # 0/0 -> NaN
        img = raw.astype(float)
        if ill is not None and img.shape == ill.shape:
            img = img / ill
        with np.errstate(all="ignore"):
            res = qc.calculate_qc_metrics(img, "CH")
            radii, magsum, powersum = qc.rps(img)
        arrays[f"{name}_raw"] = raw
        if ill is not None:
            arrays[f"{name}_illum"] = ill
        arrays[f"{name}_powersum"] = np.asarray(powersum, dtype=np.float64)
        meta[name] = dict(H=H, W=W, kind=kind, seed=seed,
                          slope=float(res["ImageQuality_PowerLogLogSlope_CH"]),
                          pct_max=float(res["ImageQuality_PercentMaximal_CH"]))
    # full-size FOV (seeded, regenerated bit-exactly by oracle/synth_golden.full_case)
    raw, ill = sg.full_case(seed=7, H=2080, W=2080, C=5, n_blobs=300)
    full = []
    for c in range(5):
        img = raw[c].astype(float) / ill[c]
        res = qc.calculate_qc_metrics(img, f"C{c}")
        _, _, ps = qc.rps(img)
        arrays[f"full_c{c}_powersum"] = np.asarray(ps, dtype=np.float64)
        full.append(dict(slope=float(res[f"ImageQuality_PowerLogLogSlope_C{c}"]),
                         pct_max=float(res[f"ImageQuality_PercentMaximal_C{c}"])))
    meta["full"] = dict(seed=7, H=2080, W=2080, C=5, n_blobs=300, channels=full)
    np.savez_compressed(os.path.join(OUT, "qc_cases.npz"), **arrays)
    with open(os.path.join(OUT, "qc_cases.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("qc cases:", list(meta))


def gen_qc_cli():
    """Run the reference CLI main() on a tiny LoadData set with TIFF planes."""
    import tifffile
    import pandas as pd
    qc = _import_ref("Illumination_QC_mult")
    d = os.path.join(OUT, "qc_cli")
    os.makedirs(os.path.join(d, "images"), exist_ok=True)
    os.makedirs(os.path.join(d, "illum"), exist_ok=True)
    chans = ["DNA", "AGP", "Mito"]
    rows = []
    H, W = 96, 120
    for site in range(4):
        row = {"Metadata_Plate": "P01", "Metadata_Well": f"A{site + 1:02d}", "Metadata_Site": 1,
               "Metadata_Timepoint": 24, "ImageQuality_Old_DNA": 1.0}
        for ci, ch in enumerate(chans):
            fn = f"r01c{site + 1:02d}f01p01-ch{ci + 1}.tiff"
            if not (site == 2 and ch == "Mito"):  # one missing file -> "File Not Found"
                tifffile.imwrite(os.path.join(d, "images", fn), sg.plane(100 + site * 10 + ci, H, W, n_blobs=6))
            row[f"FileName_{ch}"] = fn
        rows.append(row)
    pd.DataFrame(rows).to_csv(os.path.join(d, "load_data.csv"), index=False)
    # illum: DNA as {c}_illum.npy (f32), AGP as Illum{c}.npy (f64), Mito absent (warning, raw used)
    np.save(os.path.join(d, "illum", "DNA_illum.npy"), sg.illum(200, H, W, np.float32))
    np.save(os.path.join(d, "illum", "IllumAGP.npy"), sg.illum(201, H, W, np.float64))
    out = os.path.join(d, "expected_qc.csv")
    argv = sys.argv
    sys.argv = ["Illumination_QC_mult.py", "--load-data", os.path.join(d, "load_data.csv"),
                "--data-path", os.path.join(d, "images"), "--illum-path", os.path.join(d, "illum"),
                "--channels", *chans, "--output", out, "--threads", "2"]
    try:
        qc.main()
    finally:
        sys.argv = argv
    print("qc cli expected:", out)


def gen_maxproj():
    import imageio
    sys.modules.setdefault("boto3", types.ModuleType("boto3"))
    mp = _import_ref("MaxProjection")

    class FakeS3:
        def __init__(self):
            self.objects = {}

        def get_object(self, Bucket, Key):
            return {"Body": io.BytesIO(self.objects[(Bucket, Key)])}

        def upload_fileobj(self, fileobj, bucket, key):
            self.objects[(bucket, key)] = fileobj.read()

    s3 = FakeS3()
    arrays = {}
    keys = []
    Z, H, W = 5, 48, 64
    for z in range(Z):
        a = sg.plane(300 + z, H, W, n_blobs=4, saturate=False)
        buf = io.BytesIO()
        imageio.imwrite(buf, a, format="tiff")
        k = f"plate1/Images/r01c01f01p{z + 1:02d}-ch1sk1fk1fl1.tiff"
        s3.objects[("bkt", k)] = buf.getvalue()
        keys.append(k)
        arrays[f"plane{z}"] = a
    mp.max_projection(keys, "bkt", s3)
    out_key = mp.modify_imagepath(keys[0])
    data = s3.objects[("bkt", out_key)]
    arrays["expected"] = imageio.imread(io.BytesIO(data))
    arrays["expected_tiff"] = np.frombuffer(data, dtype=np.uint8)
    paths = {p: mp.modify_imagepath(p) for p in
             ["a/Images/b.tiff", "Images/x.tif", "a/b/c.tiff", "a/Images/Images/d.tiff", "a/ImagesX/e.tiff"]}
    np.savez_compressed(os.path.join(OUT, "maxproj.npz"), **arrays)
    with open(os.path.join(OUT, "maxproj.json"), "w") as f:
        json.dump({"keys": keys, "out_key": out_key, "modify_imagepath": paths}, f, indent=1)
    print("maxproj:", out_key)


def gen_objects_features():
    from skimage.measure import regionprops
    from skimage.feature import greycomatrix, greycoprops
    arrays = {}
    meta = {}
    # (a) object table on a 700x640 label image with box 200 (reference constant BOX_SIZE)
    lab = sg.labels(21, 700, 640, n=40, rmin=6, rmax=60)
    arrays["objects_labels"] = lab
    rows = []
    for p in regionprops(lab):
        yc, xc = map(int, p.centroid)
        rows.append([p.label, p.area, *p.bbox, p.centroid[0], p.centroid[1], yc, xc])
    arrays["objects_table"] = np.array(rows, dtype=np.float64)
    # (b) features on a 320x288 FOV with 3 channels
    H, W, C = 320, 288, 3
    lab2 = sg.labels(22, H, W, n=24, rmin=3, rmax=30)
    planes = np.stack([sg.plane(400 + c, H, W, n_blobs=10).astype(np.float32) /
                       sg.illum(500 + c, H, W, np.float32) for c in range(C)]).astype(np.float32)
    arrays["feat_labels"] = lab2
    arrays["feat_planes"] = planes
    angles = [0, np.pi / 4, np.pi / 2, 3 * np.pi / 4]
    frows = []
    for p in regionprops(lab2):
        sl = p.slice
        row = [p.area, p.perimeter, p.centroid[0], p.centroid[1], p.bbox_area, p.extent,
               p.equivalent_diameter, p.major_axis_length, p.minor_axis_length, p.eccentricity,
               p.orientation, *p.bbox]
        for c in range(C):
            pr = regionprops(lab2, intensity_image=planes[c])[[q.label for q in regionprops(lab2)].index(p.label)]
            vals = planes[c][sl][p.image]
            row += [float(vals.astype(np.float64).sum()), float(pr.mean_intensity),
                    float(np.std(vals.astype(np.float64))), float(pr.min_intensity), float(pr.max_intensity)]
            crop = planes[c][sl] * (lab2[sl] == p.label)
            mn, mx = np.min(crop), np.max(crop)
            q8 = np.zeros(crop.shape, np.uint8) if mx == mn else (
                255.0 * (crop.astype(np.float32) - mn) / (mx - mn)).astype(np.uint8)
            P = greycomatrix(q8, [3], angles, levels=256)
            for a in range(4):
                Pa = P[:, :, :, a:a + 1]
                row += [float(greycoprops(Pa, prop)[0, 0]) for prop in
                        ["contrast", "dissimilarity", "homogeneity", "ASM", "energy", "correlation"]]
        frows.append(row)
    arrays["feat_expected"] = np.array(frows, dtype=np.float64)
    # (c) secondary objects: skimage expand_labels on touching / gapped nuclei (ties included)
    from skimage.segmentation import expand_labels
    lab3 = sg.labels(23, 257, 301, n=30, rmin=3, rmax=20)
    lab3[100:104, 50:54] = 77  # two small squares at even distance -> equidistant pixels
    lab3[100:104, 64:68] = 78
    arrays["expand_labels_in"] = lab3
    for dist in (1, 5, 15):
        arrays[f"expand_labels_d{dist}"] = expand_labels(lab3, dist)
    meta["features"] = dict(H=H, W=W, C=C, n_objects=len(frows))
    np.savez_compressed(os.path.join(OUT, "objects_features.npz"), **arrays)
    with open(os.path.join(OUT, "objects_features.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("objects/features:", meta)


def gen_cellpose_helpers():
    sys.modules.setdefault("tifffile", types.ModuleType("tifffile"))
    cp = _import_ref("Cellpose_GPU_s3fs")
    arrays = {}
    rng_cases = []
    for k in range(6):
        a = sg.plane(600 + k, 40, 50, n_blobs=3).astype(np.float32) / np.float32(1.0 + 0.1 * k)
        if k == 3:
            a[:] = 7.0  # max == min -> zeros
        if k == 4:
            a[::3] = 0.0
        rng_cases.append(a)
        arrays[f"in{k}"] = a
        arrays[f"out{k}"] = cp.scale_to_8bit(a)
    consts = dict(BOX_SIZE=cp.BOX_SIZE, FEATURE_LENGTH=cp.FEATURE_LENGTH, CELLPOSE_MODEL=cp.CELLPOSE_MODEL,
                  MODEL_NAME=cp.MODEL_NAME, INFERENCE_BATCH_SIZE=cp.INFERENCE_BATCH_SIZE)
    np.savez_compressed(os.path.join(OUT, "scale8.npz"), **arrays)
    with open(os.path.join(OUT, "cellpose_consts.json"), "w") as f:
        json.dump(consts, f, indent=1)
    print("cellpose helpers:", consts)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cellpose-helpers", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    if a.cellpose_helpers:
        gen_cellpose_helpers()
    else:
        todo = a.only.split(",") if a.only else ["qc", "qc_cli", "maxproj", "objects"]
        if "qc" in todo:
            gen_qc()
        if "qc_cli" in todo:
            gen_qc_cli()
        if "maxproj" in todo:
            gen_maxproj()
        if "objects" in todo:
            gen_objects_features()

"""Per-plate well normalisation on the GPU: the drop-in for Normalize_CP_ami.py (SURVEY 8(f)
rank 2, after-path half).

`normalize_plates(...)` / `python -m cpx.normalize` follow Normalize_CP_ami.py:29-138 on the
`<base>/<plate>[/<time>]/{Image,Nuclei,Cells,Cytoplasm}.csv` tables (local directories stand in
for the buckets): ImageQC_* failing images (optionally dropped), Metadata_Well/Site attached from
Image, column clean-up and table prefixes, site-count scaling of integer features, per-well
aggregation, outer merge, plate-map annotation and DMSO-fitted MAD-robustize.  Host pandas does
the table plumbing exactly as the reference; the reductions run in libcpx:

  reference call (file:line)                                   libcpx
  `df[ints].multiply(scaling_factor)` + `groupby(Well).agg(mean)` (:105-113)
                                                               cpx_group_kahan_accumulate (scale fused)
  `groupby(Well).agg("median")` (:113)                         cpx_group_median (scale fused)
  pycytominer normalize(method="mad_robustize") (:124-129)      cpx_robust_mad + cpx_mad_transform

pycytominer's `annotate` is restated (inner merge of the Metadata_-prefixed plate map on
Metadata_Well, metadata columns first); pycytominer is absent and unpinned by the reference.
"""
from __future__ import annotations

import argparse
import logging
import os
from functools import reduce

import numpy as np

from .profiles import ProfileEngine, read_table

TABLE_PREFIX = {"Image": "Image_", "Nuclei": "DNA_", "Cells": "Cell_", "Cytoplasm": "Cyto_"}
DROP_SUBSTRINGS = ["ExecutionTime", "ModuleError", "URL"]
log = logging.getLogger("cpx.normalize")


def failing_images(image_df):
    """Normalize_CP_ami.py:67 — ImageNumbers with any ImageQC_* flag set."""
    return image_df.loc[image_df.filter(like="ImageQC_").any(axis=1), "ImageNumber"]


def well_tables(eng: ProfileEngine, tables: dict, qc_drop: bool, agg: str = "mean"):
    """Normalize_CP_ami.py:66-116 on read tables -> merged per-well frame."""
    import pandas as pd
    tables = dict(tables)
    image_df = tables["Image"]
    failing = failing_images(image_df)
    for name, df in tables.items():
        if "Metadata_Well" not in df.columns:
            df = df.merge(image_df[["ImageNumber", "Metadata_Well", "Metadata_Site"]], on="ImageNumber", how="left")
            tables[name] = df
        if qc_drop:
            log.info("Removing QC failed images")
            tables[name] = df[~df["ImageNumber"].isin(failing)]
    for name, prefix in TABLE_PREFIX.items():
        df = tables[name]
        keep_meta = {"Metadata_Well", "Metadata_Site"} if qc_drop else {"Metadata_Well"}
        df = df.drop(columns=[c for c in df.columns if c == "ImageNumber"
                              or (c.startswith("Metadata") and c not in keep_meta)
                              or any(sub in c for sub in DROP_SUBSTRINGS)])
        df = df.rename(columns=lambda x: prefix + x if not x.startswith("Metadata_") else x)
        row_scale, scaled = None, ()
        if qc_drop:
            # sites per well -> max_sites / sites, applied to the integer features inside the
            # GPU reduction (rows of wells without a site count drop out, as the inner merge)
            site_counts = df.groupby("Metadata_Well")["Metadata_Site"].nunique()
            factor = site_counts.max() / site_counts
            row_scale = df["Metadata_Well"].map(factor).to_numpy(dtype=np.float64)
            drop_rows = np.isnan(row_scale)
            if drop_rows.any():
                df, row_scale = df[~drop_rows], row_scale[~drop_rows]
            scaled = [c for c in df.select_dtypes(include="integer").columns if not c.startswith("Metadata")]
            df = df.drop(columns=["Metadata_Site"])
        tables[name] = eng.group_agg(df.reset_index(drop=True), ["Metadata_Well"], agg, row_scale, scaled)
    return reduce(lambda l, r: pd.merge(l, r, on="Metadata_Well", how="outer"), tables.values())


def annotate(profiles, platemap):
    """pycytominer annotate(profiles, platemap, join_on=[["Metadata_Well"], ["Metadata_Well"]])."""
    pm = platemap.copy()
    pm.columns = [c if c.startswith("Metadata_") else f"Metadata_{c}" for c in pm.columns]
    out = pm.merge(profiles, on="Metadata_Well", how="inner")
    meta = [c for c in out.columns if c.startswith("Metadata_")]
    return out.loc[:, meta + [c for c in out.columns if c not in meta]]


def normalize_time(eng: ProfileEngine, tables: dict, platemap, time: str, dmso: str = "DMSO",
                   qc_drop: bool = False, agg: str = "mean"):
    """Normalize_CP_ami.py:47-131 for one plate/time -> the Normalized_features frame."""
    import pandas as pd
    pm = platemap[["Metadata_Compound", "Metadata_ConcLevel", "Metadata_Well", "Metadata_Plate"]].copy()
    pm["Metadata_Compound"] = pm["Metadata_Compound"].apply(lambda x: str(x).upper())
    df = annotate(well_tables(eng, tables, qc_drop, agg), pm)
    df["Metadata_Timepoint"] = time
    feats = df.columns[~df.columns.str.contains("Metadata")].to_list()
    meta = [c for c in df.columns if c.startswith("Metadata_")]
    fit = ((df["Metadata_Compound"] == dmso) & (df["Metadata_Timepoint"] == time)).to_numpy()
    Z = eng.mad_sigmoid(df.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan),
                        np.nonzero(fit)[0], sigmoid=False) if feats else np.zeros((len(df), 0))
    out = df.loc[:, meta].merge(pd.DataFrame(Z, columns=feats, index=df.index),
                                left_index=True, right_index=True)
    f2 = out.columns[~out.columns.str.contains("Metadata")].to_list()
    out[f2] = out[f2].astype(float)
    return out


def normalize_plates(bucket_name: str, plates, times, base_folder_path: str, output_bucket: str,
                     DMSO: str = "DMSO", output_prefix: str = "", well_agg_func: str = "mean",
                     no_time_subFolder: bool = False, qc_drop: bool = False, dev=None):
    """Normalize_CP_ami.py:29-138 `concatenate_csv_from_s3` over local directories."""
    if well_agg_func not in ("mean", "median"):
        raise NotImplementedError(f"--well_agg_func {well_agg_func!r}: libcpx implements mean and median")
    eng = ProfileEngine(dev)
    written = []
    for plate in plates:
        log.info("Processing plate ID: %s", plate)
        pm = read_table(os.path.join(bucket_name, f"{base_folder_path}/Plate_{plate.lstrip('binned/')}_PlateMap.csv"))
        for time in times:
            log.info("Processing timepoint: %s", time)
            d = os.path.join(bucket_name, base_folder_path, plate) if no_time_subFolder else \
                os.path.join(bucket_name, base_folder_path, plate, str(time))
            tables = {n: read_table(os.path.join(d, f"{n}.csv")) for n in TABLE_PREFIX}
            out = normalize_time(eng, tables, pm, str(time), DMSO, qc_drop, well_agg_func)
            dst = os.path.join(output_bucket, output_prefix, plate)
            os.makedirs(dst, exist_ok=True)
            p = os.path.join(dst, f"Normalized_features_{time}.csv")
            out.to_csv(p, index=False)
            log.info("Saved to %s", p)
            written.append(p)
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description="Normalize each timepoint of a project folder against DMSO (GPU).")
    ap.add_argument("--bucket_name", type=str, required=True, help="local root standing in for the input bucket")
    ap.add_argument("--base_folder", type=str, required=True)
    ap.add_argument("--plates", nargs="+", required=True)
    ap.add_argument("--times", nargs="+")
    ap.add_argument("--DMSO", type=str, default="DMSO")
    ap.add_argument("--output_bucket", type=str, required=True, help="local root standing in for the output bucket")
    ap.add_argument("--output_prefix", type=str, required=True)
    ap.add_argument("--well_agg_func", type=str, default="mean")
    ap.add_argument("--no_time_subFolder", action="store_true")
    ap.add_argument("--qc_drop", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(message)s", level=logging.INFO)
    return normalize_plates(a.bucket_name, a.plates, a.times, a.base_folder, a.output_bucket, a.DMSO,
                            a.output_prefix, a.well_agg_func, a.no_time_subFolder, a.qc_drop)


if __name__ == "__main__":
    main()

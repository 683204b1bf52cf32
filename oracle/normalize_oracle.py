"""CPU restatement (test infrastructure only) of Normalize_CP_ami.py:29-127
`concatenate_csv_from_s3` (second half): per plate and time,
  * read the plate map `<base>/Plate_<plate.lstrip('binned/')>_PlateMap.csv` (Compound upper-cased,
    :41-44) and `<base>/<plate>[/<time>]/{Image,Nuclei,Cells,Cytoplasm}.csv` (:47-64);
  * images flagged by any ImageQC_* column fail (:67); tables without Metadata_Well get
    Well/Site from Image (:68-76); with qc_drop the failing images' rows are removed (:77-79);
  * per table: drop ImageNumber, other Metadata, ExecutionTime/ModuleError/URL columns, prefix
    the rest (Image_, DNA_, Cell_, Cyto_); with qc_drop, integer features are scaled by
    max_sites / sites_in_well (:86-111); aggregate per Metadata_Well with `well_agg_func`
    (:113); outer-merge the four tables on Metadata_Well (:116);
  * pycytominer `annotate` with the plate map on Metadata_Well (:119) and `normalize(
    method="mad_robustize")` fitted on `Metadata_Compound == DMSO and Metadata_Timepoint ==
    time` (:124-129); features cast to float and written to
    `<prefix>/<plate>/Normalized_features_<time>.csv` (:131-138).
pycytominer is absent and unpinned by the reference (requirements.txt): annotate is restated as
the inner merge of the plate map (columns Metadata_-prefixed) with the profiles on
Metadata_Well, metadata columns first; RobustMAD as in profiles_oracle (pinned to pandas/scipy).
"""
from __future__ import annotations

import os
from functools import reduce

import numpy as np

import profiles_oracle as po

TABLE_PREFIX = {"Image": "Image_", "Nuclei": "DNA_", "Cells": "Cell_", "Cytoplasm": "Cyto_"}
DROP_SUBSTRINGS = ["ExecutionTime", "ModuleError", "URL"]


def well_tables(tables: dict, qc_drop: bool, agg: str = "mean"):
    """:66-116 on already-read tables -> merged per-well frame."""
    import pandas as pd
    tables = dict(tables)
    image_df = tables["Image"]
    failing = image_df.loc[image_df.filter(like="ImageQC_").any(axis=1), "ImageNumber"]
    for name, df in tables.items():
        if "Metadata_Well" not in df.columns:
            df = df.merge(image_df[["ImageNumber", "Metadata_Well", "Metadata_Site"]], on="ImageNumber", how="left")
            tables[name] = df
        if qc_drop:
            tables[name] = df[~df["ImageNumber"].isin(failing)]
    for name, prefix in TABLE_PREFIX.items():
        df = tables[name]
        keep_meta = {"Metadata_Well", "Metadata_Site"} if qc_drop else {"Metadata_Well"}
        df = df.drop(columns=[c for c in df.columns if c == "ImageNumber"
                              or (c.startswith("Metadata") and c not in keep_meta)
                              or any(sub in c for sub in DROP_SUBSTRINGS)])
        df = df.rename(columns=lambda x: prefix + x if not x.startswith("Metadata_") else x)
        if qc_drop:
            site_counts = df.groupby("Metadata_Well")["Metadata_Site"].nunique()
            scaling = (site_counts.max() / site_counts).rename("scaling_factor")
            df = df.merge(scaling, on="Metadata_Well")
            ints = [c for c in df.select_dtypes(include="integer").columns if not c.startswith("Metadata")]
            df[ints] = df[ints].multiply(df["scaling_factor"], axis=0)
            df = df.drop(columns=["scaling_factor", "Metadata_Site"])
        gb = df.groupby("Metadata_Well", as_index=False)
        # pandas 1.5.3 drops non-numeric columns in agg("mean"/"median")
        df = gb.mean(numeric_only=True) if agg == "mean" else gb.median(numeric_only=True)
        tables[name] = df
    return reduce(lambda l, r: pd.merge(l, r, on="Metadata_Well", how="outer"), tables.values())


def annotate(profiles, platemap):
    """pycytominer annotate(join_on=[["Metadata_Well"], ["Metadata_Well"]]) restated."""
    pm = platemap.copy()
    pm.columns = [c if c.startswith("Metadata_") else f"Metadata_{c}" for c in pm.columns]
    out = pm.merge(profiles, on="Metadata_Well", how="inner")
    meta = [c for c in out.columns if c.startswith("Metadata_")]
    return out.loc[:, meta + [c for c in out.columns if c not in meta]]


def normalize_time(tables: dict, platemap, time: str, dmso: str = "DMSO", qc_drop: bool = False,
                   agg: str = "mean"):
    """One plate/time -> the Normalized_features frame."""
    import pandas as pd
    pm = platemap[["Metadata_Compound", "Metadata_ConcLevel", "Metadata_Well", "Metadata_Plate"]].copy()
    pm["Metadata_Compound"] = pm["Metadata_Compound"].apply(lambda x: str(x).upper())
    df = annotate(well_tables(tables, qc_drop, agg), pm)
    df["Metadata_Timepoint"] = time
    feats = df.columns[~df.columns.str.contains("Metadata")].to_list()
    meta = [c for c in df.columns if c.startswith("Metadata_")]
    fit = df.query(f"Metadata_Compound == '{dmso}' and Metadata_Timepoint == '{time}'")
    med, mad = po.robust_mad_fit(fit.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan))
    X = df.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan)
    Z = (X - med) / (mad + po.MAD_EPS)
    out = df.loc[:, meta].merge(pd.DataFrame(Z, columns=feats, index=df.index),
                                left_index=True, right_index=True)
    f2 = out.columns[~out.columns.str.contains("Metadata")].to_list()
    out[f2] = out[f2].astype(float)
    return out


def platemap_key(base_folder_path: str, plate: str) -> str:
    return f"{base_folder_path}/Plate_{plate.lstrip('binned/')}_PlateMap.csv"


def read_plate_time(root, base_folder_path, plate, time, no_time_subfolder=False):
    d = os.path.join(root, base_folder_path, plate) if no_time_subfolder else \
        os.path.join(root, base_folder_path, plate, str(time))
    return {n: po.read_table(os.path.join(d, f"{n}.csv")) for n in TABLE_PREFIX}

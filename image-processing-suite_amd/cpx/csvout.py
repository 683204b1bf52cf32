"""Per-plate/time measurement tables in the layout Pycyto_pertime.py reads.

Pycyto_pertime.py:46-49 reads `<base>/<plate>/<time>/{Image,Nuclei,Cells,Cytoplasm}.csv` (the
CellProfiler output synced by Feature_extraction_opt.py:177) and merges the object tables with
Image on ImageNumber (:51-58), then aggregates numeric columns per well (:61-75).  This module
writes those four tables from the GPU pipeline's results:
  Image.csv      ImageNumber, the LoadData Metadata_* columns, ImageQuality_PowerLogLogSlope_<ch>,
                 ImageQuality_PercentMaximal_<ch>, Count_Nuclei, Count_Cells, Count_Cytoplasm
  <Object>.csv   ImageNumber, ObjectNumber, Number_Object_Number, then the feature columns of
                 `feature_names(channels)` (AreaShape_*, Intensity_*_<ch>, Texture_*_<ch>_3_<dir>_256)
ImageNumber is the 1-based LoadData row; ObjectNumber is the object's label, which the
segmentation makes consecutive (1..K per image) and which Cells and Cytoplasm share with their
nucleus.  Rows are sorted by (ImageNumber, ObjectNumber), so the output does not depend on the
number of GPUs or on batch order.
"""
from __future__ import annotations

import os

import numpy as np

SHAPE_NAMES = ["AreaShape_Area", "AreaShape_Perimeter", "AreaShape_Center_Y", "AreaShape_Center_X",
               "AreaShape_BoundingBoxArea", "AreaShape_Extent", "AreaShape_EquivalentDiameter",
               "AreaShape_MajorAxisLength", "AreaShape_MinorAxisLength", "AreaShape_Eccentricity",
               "AreaShape_Orientation", "AreaShape_BoundingBoxMinimum_Y", "AreaShape_BoundingBoxMinimum_X",
               "AreaShape_BoundingBoxMaximum_Y", "AreaShape_BoundingBoxMaximum_X"]
INTENSITY_NAMES = ["IntegratedIntensity", "MeanIntensity", "StdIntensity", "MinIntensity", "MaxIntensity"]
TEXTURE_NAMES = ["Contrast", "Dissimilarity", "Homogeneity", "AngularSecondMoment", "Energy", "Correlation"]
TEXTURE_SCALE = 3
OBJECT_TABLES = ("Nuclei", "Cells", "Cytoplasm")


def feature_names(channels):
    """Column names of a cpx_features row (layout of include/cpx.h: CPX_N_SHAPE shape columns,
    then per channel 5 intensity + 4 directions x 6 texture columns)."""
    names = list(SHAPE_NAMES)
    for ch in channels:
        names += [f"Intensity_{n}_{ch}" for n in INTENSITY_NAMES]
        for d in range(4):
            names += [f"Texture_{p}_{ch}_{TEXTURE_SCALE}_{d:02d}_256" for p in TEXTURE_NAMES]
    return names


class PlateTables:
    """Accumulates per-FOV results of one plate/time and writes the four CSVs."""

    def __init__(self, channels):
        self.channels = list(channels)
        self.cols = feature_names(self.channels)
        self.images = []                       # dicts
        self.objects = {t: [] for t in OBJECT_TABLES}  # (ImageNumber, labels[n], feats[n, F])

    def add_image(self, image_number: int, metadata: dict, qc_slope, qc_pct, counts: dict):
        row = {"ImageNumber": int(image_number)}
        row.update({k: v for k, v in metadata.items() if k.startswith("Metadata_")})
        for ch, s, p in zip(self.channels, qc_slope, qc_pct):
            row[f"ImageQuality_PowerLogLogSlope_{ch}"] = float(s)
            row[f"ImageQuality_PercentMaximal_{ch}"] = float(p)
        for t in OBJECT_TABLES:
            row[f"Count_{t}"] = int(counts.get(t, 0))
        self.images.append(row)

    def add_objects(self, table: str, image_number: int, labels, feats):
        labels = np.asarray(labels, dtype=np.int64)
        feats = np.asarray(feats, dtype=np.float64)
        if feats.shape != (len(labels), len(self.cols)):
            raise ValueError(f"{table}: feature block {feats.shape} for {len(labels)} objects x "
                             f"{len(self.cols)} columns")
        self.objects[table].append((int(image_number), labels, feats))

    def frames(self):
        import pandas as pd
        out = {"Image": pd.DataFrame(self.images).sort_values("ImageNumber", kind="stable")
               .reset_index(drop=True) if self.images else pd.DataFrame(columns=["ImageNumber"])}
        for t in OBJECT_TABLES:
            blocks = []
            for img, labels, feats in self.objects[t]:
                df = pd.DataFrame(feats, columns=self.cols)
                df.insert(0, "Number_Object_Number", labels)
                df.insert(0, "ObjectNumber", labels)
                df.insert(0, "ImageNumber", img)
                blocks.append(df)
            if blocks:
                df = pd.concat(blocks, ignore_index=True)
                df = df.sort_values(["ImageNumber", "ObjectNumber"], kind="stable").reset_index(drop=True)
            else:
                df = pd.DataFrame(columns=["ImageNumber", "ObjectNumber", "Number_Object_Number"] + self.cols)
            out[t] = df
        return out

    def write(self, base: str, plate: str, time) -> str:
        d = os.path.join(base, str(plate), str(time))
        os.makedirs(d, exist_ok=True)
        for name, df in self.frames().items():
            df.to_csv(os.path.join(d, f"{name}.csv"), index=False)
        return d

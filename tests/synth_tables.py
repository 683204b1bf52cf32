"""Synthetic per-time measurement tables in the layout `cpx.csvout` writes (inputs of the
profile step, Pycyto_pertime.py:46-49), for tests and tools/profiles_bench.py.

A plate of `n_wells` wells x `sites` FOVs: Image.csv carries the LoadData metadata the
reference reads (Plate, Site, Well, Timepoint, Compound, ConcLevel) plus QC and count columns;
Nuclei/Cells/Cytoplasm carry ImageNumber, ObjectNumber and `n_feat` float features per object
(feature_names layout when n_feat is None).  Every 4th well is DMSO; the others cycle through
compounds x concentration levels with replicate wells, and each compound shifts a few features
so normalisation and feature selection have structure to act on.  A few NaNs, exact ties and
constant columns exercise the NaN / variance paths.
"""
from __future__ import annotations

import numpy as np


def plate_tables(n_wells: int = 24, sites: int = 2, objects: int = 20, n_feat: int | None = 24,
                 seed: int = 0, channels=("DNA", "ER", "RNA", "AGP", "Mito"), plate: str = "Plate_1",
                 time: str = "T1", nan_frac: float = 0.002):
    import pandas as pd
    from cpx.csvout import feature_names
    rng = np.random.default_rng(seed)
    cols = feature_names(channels) if n_feat is None else [f"Feature_{i:03d}" for i in range(n_feat)]
    F = len(cols)
    compounds = ["CmpA", "CmpB", "CmpC"]
    wells = [f"{chr(ord('A') + w // 24)}{w % 24 + 1:02d}" for w in range(n_wells)]
    images, objs = [], {t: [] for t in ("Nuclei", "Cells", "Cytoplasm")}
    effect = {c: rng.normal(0, 1.0, F) * (rng.random(F) < 0.3) for c in compounds}
    img_no = 0
    for wi, well in enumerate(wells):
        if wi % 4 == 0:
            cmpd, conc = "DMSO", 0
        else:
            k = wi - wi // 4 - 1
            cmpd, conc = compounds[k % 3], 1 + (k // 3) % 2
        for s in range(sites):
            img_no += 1
            n = int(rng.integers(max(1, objects // 2), objects * 3 // 2 + 1))
            images.append({"ImageNumber": img_no, "Metadata_Plate": plate, "Metadata_Site": s + 1,
                           "Metadata_Well": well, "Metadata_Timepoint": time,
                           "Metadata_Compound": cmpd, "Metadata_ConcLevel": conc,
                           "ImageQuality_PowerLogLogSlope_DNA": float(rng.normal(-2.0, 0.1)),
                           "ImageQuality_PercentMaximal_DNA": float(rng.random() * 1e-3),
                           "Count_Nuclei": n, "Count_Cells": n, "Count_Cytoplasm": n})
            for t_i, t in enumerate(objs):
                base = rng.lognormal(0.0, 0.5, (n, F)) * (10.0 ** (np.arange(F) % 5 - 1))
                base += effect.get(cmpd, 0.0) * (1 + t_i)
                base[:, 0] = np.round(base[:, 0])         # integer-valued column (ties)
                base[:, 1] = 7.0                          # constant column
                base[rng.random((n, F)) < nan_frac] = np.nan
                df = pd.DataFrame(base, columns=cols)
                df.insert(0, "Number_Object_Number", np.arange(1, n + 1))
                df.insert(0, "ObjectNumber", np.arange(1, n + 1))
                df.insert(0, "ImageNumber", img_no)
                objs[t].append(df)
    out = {"Image": pd.DataFrame(images)}
    for t, blocks in objs.items():
        df = pd.concat(blocks, ignore_index=True)
        # column-contiguous blocks, the layout pandas.read_csv produces
        out[t] = pd.DataFrame({c: np.ascontiguousarray(df[c].to_numpy()) for c in df.columns})
    return out


def write_tree(root: str, base_folder: str, time: str, tables) -> str:
    import os
    d = os.path.join(root, base_folder, str(time))
    os.makedirs(d, exist_ok=True)
    for name, df in tables.items():
        df.to_csv(os.path.join(d, f"{name}.csv"), index=False)
    return d

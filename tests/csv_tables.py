"""Shared by the configs[0] CPU test and the GPU CSV-parity test: one FOV's result tables in the
layout Pycyto_pertime.py reads, written through cpx.csvout.PlateTables."""
import numpy as np

from cpx.csvout import PlateTables

CHANNELS = ("DNA", "ER", "RNA", "AGP", "Mito")


def cpu_tables(out: dict, image_number: int = 1, metadata=None):
    """oracle/cpu_pipeline.run_fov output -> PlateTables."""
    t = PlateTables(CHANNELS)
    slopes = [q[f"ImageQuality_PowerLogLogSlope_{i}"] for i, q in enumerate(out["qc"])]
    pcts = [q[f"ImageQuality_PercentMaximal_{i}"] for i, q in enumerate(out["qc"])]
    labs = {"Nuclei": out["nuclei"], "Cells": out["cells"], "Cytoplasm": out["cyto"]}
    counts = {s: int(len(np.unique(l[l > 0]))) for s, l in labs.items()}
    t.add_image(image_number, metadata or {"Metadata_Well": "A01"}, slopes, pcts, counts)
    for s, l in labs.items():
        t.add_objects(s, image_number, np.unique(l[l > 0]), out["feats"][s])
    return t


def gpu_tables(res, b: int = 0, image_number: int = 1, metadata=None):
    """FovResults (one FOV of a fetched batch) -> PlateTables."""
    t = PlateTables(CHANNELS)
    C = len(CHANNELS)
    qc = res.qc[b * C:(b + 1) * C]
    counts = {s: int(res.hdr[s]["n_objects"][b]) for s in ("Nuclei", "Cells", "Cytoplasm")}
    t.add_image(image_number, metadata or {"Metadata_Well": "A01"}, qc["slope"], qc["pct_max"], counts)
    for s in ("Nuclei", "Cells", "Cytoplasm"):
        t.add_objects(s, image_number, res.objects[s][b]["label"], res.feats[s][b])
    return t

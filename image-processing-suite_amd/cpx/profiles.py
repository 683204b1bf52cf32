"""Per-time plate profiles on the GPU: the drop-in for Pycyto_pertime.py.

`concatenate_csv(...)` / `python -m cpx.profiles` follow Pycyto_pertime.py:29-172 step by step
on the `<base>/<time>/{Image,Nuclei,Cells,Cytoplasm}.csv` tables that `cpx.csvout` writes (a
local directory stands in for the S3 buckets).  Host pandas does the table plumbing the
reference does (CSV I/O, metadata merges, column bookkeeping); every numeric reduction runs in
libcpx (include/cpx.h, k_profiles.hip) with the arithmetic of the library call it replaces:

  reference call (file:line)                                  libcpx
  `groupby(keys, as_index=False).mean()` (:69-72)             cpx_group_kahan_accumulate/_finalize
  pycytominer normalize(mad_robustize) fit (:83-88)           cpx_robust_mad
  RobustMAD transform + double_sigmoid + abs (:13-16, 89-91)  cpx_mad_transform
  feature_select stats (:93-104)                              cpx_column_stats, cpx_nancorr
  cosine_similarity within treatment groups (:115-140)        cpx_cosine_groups

`groupby(...).mean()` is taken with the reference's pandas 1.5.3 behaviour (non-numeric
columns outside the keys are dropped), which is `numeric_only=True` in current pandas.
"""
from __future__ import annotations

import argparse
import csv
import io
import os
from functools import reduce

import numpy as np

from . import _lib

KEYS = ["Metadata_Plate", "Metadata_Well", "Metadata_Timepoint", "Metadata_Compound"]
IMAGE_META = ["ImageNumber", "Metadata_Plate", "Metadata_Site", "Metadata_Well",
              "Metadata_Timepoint", "Metadata_Compound", "Metadata_ConcLevel"]
K_SIG = 3              # Pycyto_pertime.py:13
ALPHA = 2.3538         # Pycyto_pertime.py:14
MAD_SCALE = 1 / 1.4826  # pycytominer RobustMAD -> scipy median_abs_deviation(scale=1/1.4826)
MAD_EPS = 1e-18        # pycytominer normalize(mad_robustize_epsilon=1e-18)
FEATURE_SELECT_OPS = ["variance_threshold", "drop_na_columns", "correlation_threshold", "drop_outliers"]


def _group_codes(gb) -> np.ndarray:
    """Row -> group index in sorted-key order; -1 for rows whose keys hold NaN (pandas drops
    them; ngroup() reports NaN for them)."""
    c = gb.ngroup().to_numpy(dtype=np.float64)
    return np.where(np.isnan(c), -1, c).astype(np.int64)


class ProfileEngine:
    """GPU numerics of the profile step on one device (cpx.device.Device)."""

    def __init__(self, dev=None):
        import torch
        from .device import Device
        self.dev = dev if dev is not None else Device(0)
        self.torch = torch
        self.td = self.dev.torch_device

    def _t(self, a, dtype=None):
        return self.torch.from_numpy(np.ascontiguousarray(a, dtype=dtype)).to(self.td)

    # -- Pycyto_pertime.py:69-72 -----------------------------------------------------------
    def group_mean(self, df, keys=KEYS):
        """`df.groupby(keys, as_index=False).mean()` (sorted keys, NaN keys dropped, numeric
        columns only) with pandas' Kahan group mean on the GPU."""
        return self.group_agg(df, keys, "mean")

    def _upload_rows(self, df, cols):
        """fp64 [n, K] row-major device copy of df[cols].  pandas keeps each column contiguous
        inside its dtype block, so columns are uploaded one by one (views, no host re-layout:
        DataFrame.to_numpy's interleave of mixed blocks costs seconds at 10^6 rows) into a
        column-major device buffer that is then transposed in HBM."""
        torch = self.torch
        cm = torch.empty((len(cols), len(df)), dtype=torch.float64, device=self.td)
        for i, c in enumerate(cols):
            v = df[c].to_numpy(dtype=np.float64, na_value=np.nan)
            cm[i].copy_(torch.from_numpy(np.ascontiguousarray(v)))
        return cm.t().contiguous()

    def _kahan_means(self, df, cols, codes, G, func="mean", row_scale=None, scaled_cols=()) -> np.ndarray:
        """Per-group means (pandas Kahan) or medians of df[cols] for row group codes in [0, G)
        (-1: row dropped); `row_scale` [n] multiplies the columns named in `scaled_cols`."""
        torch = self.torch
        keep = codes >= 0
        rows = np.nonzero(keep)[0]
        order = rows[np.argsort(codes[keep], kind="stable")].astype(np.int32)
        counts = np.bincount(codes[keep], minlength=G)
        offs = np.zeros(G + 1, dtype=np.int32)
        np.cumsum(counts, out=offs[1:])
        K = len(cols)
        vals = self._upload_rows(df, cols)
        rs = cs = None
        if row_scale is not None and len(scaled_cols):
            rs = self._t(np.asarray(row_scale, dtype=np.float64))
            sc = set(scaled_cols)
            cs = self._t(np.array([c in sc for c in cols], dtype=np.uint8))
        out = torch.empty((G, K), dtype=torch.float64, device=self.td)
        if func == "mean":
            sumx = torch.zeros((G, K), dtype=torch.float64, device=self.td)
            comp = torch.zeros_like(sumx)
            nobs = torch.zeros((G, K), dtype=torch.int64, device=self.td)
            self.dev.group_kahan(vals, self._t(order), self._t(offs), sumx, comp, nobs, rs, cs)
            self.dev.group_finalize(sumx, nobs, out)
        elif func == "median":
            self.dev.group_median(vals, self._t(order), self._t(offs), int(counts.max(initial=0)), out, rs, cs)
        else:
            raise NotImplementedError(f"well aggregation {func!r}: libcpx implements 'mean' and 'median'")
        return out.cpu().numpy()

    def group_agg(self, df, keys, func="mean", row_scale=None, scaled_cols=()):
        """`df.groupby(keys, as_index=False).agg(func)` for func in {"mean", "median"} (pandas
        1.5.3: non-numeric columns dropped), optionally with per-row scaling of some columns
        fused into the reduction (the values pandas would have multiplied first)."""
        import pandas as pd
        gb = df.groupby(keys, sort=True)
        codes = _group_codes(gb)
        key_df = gb.size().reset_index()[keys]
        G = len(key_df)
        cols = [c for c in df.columns if c not in keys and
                (pd.api.types.is_numeric_dtype(df[c]) or pd.api.types.is_bool_dtype(df[c]))]
        if G == 0 or not cols:
            return pd.concat([key_df, pd.DataFrame(index=key_df.index, columns=cols, dtype=float)], axis=1)
        vals = self._kahan_means(df, cols, codes, G, func, row_scale, scaled_cols)
        return pd.concat([key_df, pd.DataFrame(vals, columns=cols, index=key_df.index)], axis=1)

    def object_means(self, obj, image, keys=KEYS):
        """`obj.merge(image[IMAGE_META], on="ImageNumber", how="left").drop(ImageNumber, Site,
        ConcLevel).groupby(keys, as_index=False).mean()` without materialising the merge: every
        object row takes the well group of its image.  Callers check `object_means_applies`."""
        import pandas as pd
        igb = image.groupby(keys, sort=True)
        icode = _group_codes(igb)
        ikeys = igb.size().reset_index()[keys]
        lut = pd.Series(icode, index=image["ImageNumber"].to_numpy())
        codes = lut.reindex(obj["ImageNumber"].to_numpy()).to_numpy()
        used = np.unique(codes[codes >= 0])
        remap = np.full(len(ikeys), -1, dtype=np.int64)
        remap[used] = np.arange(len(used))
        codes = np.where(codes >= 0, remap[np.maximum(codes, 0)], -1)
        key_df = ikeys.iloc[used].reset_index(drop=True)
        cols = [c for c in obj.columns if c != "ImageNumber" and
                (pd.api.types.is_numeric_dtype(obj[c]) or pd.api.types.is_bool_dtype(obj[c]))]
        if len(used) == 0 or not cols:
            return pd.concat([key_df, pd.DataFrame(index=key_df.index, columns=cols, dtype=float)], axis=1)
        means = self._kahan_means(obj, cols, codes, len(used))
        return pd.concat([key_df, pd.DataFrame(means, columns=cols, index=key_df.index)], axis=1)


    # -- Pycyto_pertime.py:83-91 -----------------------------------------------------------
    def mad_sigmoid(self, X: np.ndarray, fit_rows: np.ndarray, sigmoid: bool = True) -> np.ndarray:
        """normalize(mad_robustize) fitted on X[fit_rows], then (sigmoid=True) |double_sigmoid|;
        X [N, K]."""
        torch = self.torch
        N, K = X.shape
        if K == 0:
            return np.zeros((N, 0))
        col = self._t(np.asarray(X, dtype=np.float64).T)
        med = torch.empty(K, dtype=torch.float64, device=self.td)
        mad = torch.empty_like(med)
        self.dev.robust_mad(col, self._t(np.asarray(fit_rows, dtype=np.int32)), MAD_SCALE, med, mad)
        out = torch.empty_like(col)
        self.dev.mad_transform(col, med, mad, MAD_EPS, out, double_sigmoid=sigmoid, alpha=ALPHA)
        return out.cpu().numpy().T.copy()

    # -- Pycyto_pertime.py:93-104 (pycytominer feature_select) ------------------------------
    def column_stats(self, X: np.ndarray):
        torch = self.torch
        N, K = X.shape
        col = self._t(np.asarray(X, dtype=np.float64).T)
        st = torch.empty(48 * K, dtype=torch.uint8, device=self.td)
        self.dev.column_stats(col, st)
        raw = st.cpu().numpy()
        arr = (_lib.ColumnStat * K).from_buffer_copy(raw.tobytes())
        return [(s.na_count, s.nunique, s.top_count, s.second_count, s.max, s.min) for s in arr]

    def corr(self, X: np.ndarray) -> np.ndarray:
        torch = self.torch
        N, K = X.shape
        col = self._t(np.asarray(X, dtype=np.float64).T)
        out = torch.empty((K, K), dtype=torch.float64, device=self.td)
        self.dev.nancorr(col, out)
        return out.cpu().numpy()

    def excluded_features(self, df, features, freq_cut=0.05, unique_cut=0.01, na_cutoff=0.05,
                          corr_threshold=0.9, outlier_cutoff=500):
        """pycytominer feature_select(operation=FEATURE_SELECT_OPS) with its default cut-offs:
        the union of the four operations' exclusions, each computed on all rows."""
        import pandas as pd
        X = df.loc[:, features].to_numpy(dtype=np.float64, na_value=np.nan)
        n = X.shape[0]
        out = set()
        if not features:
            return out
        for name, (na, nuniq, top, sec, mx, mn) in zip(features, self.column_stats(X)):
            if top == 0 or sec == 0 or sec / top < freq_cut:      # variance_threshold (freq)
                out.add(name)
            if nuniq / n < unique_cut:                            # variance_threshold (unique)
                out.add(name)
            if na / n > na_cutoff:                                # drop_na_columns
                out.add(name)
            if abs(mx) > outlier_cutoff or abs(mn) > outlier_cutoff:  # drop_outliers
                out.add(name)
        corr = self.corr(X)                                       # correlation_threshold
        order = pd.DataFrame(corr, index=features, columns=features).abs().sum().sort_values().index
        tri = np.tril(np.ones(corr.shape, dtype=bool), k=-1)
        for a, b in zip(*np.nonzero(tri & (corr > corr_threshold))):
            pa, pb = features[a], features[b]
            out.add(pa if order.get_loc(pa) > order.get_loc(pb) else pb)
        return out

    # -- Pycyto_pertime.py:115-140 ---------------------------------------------------------
    def group_cosine(self, groups):
        """groups: list of [n_i, F] arrays -> list of upper-triangle similarity vectors."""
        torch = self.torch
        if not groups:
            return []
        F = groups[0].shape[1]
        sizes = np.array([g.shape[0] for g in groups], dtype=np.int64)
        offs = np.zeros(len(groups) + 1, dtype=np.int32)
        np.cumsum(sizes, out=offs[1:])
        npair = sizes * (sizes - 1) // 2
        poffs = np.zeros(len(groups) + 1, dtype=np.int64)
        np.cumsum(npair, out=poffs[1:])
        if F == 0:
            return [np.zeros(int(p)) for p in npair]
        x = self._t(np.concatenate(groups, axis=0), np.float64)
        norms = torch.empty(x.shape[0], dtype=torch.float64, device=self.td)
        out = torch.empty(int(poffs[-1]), dtype=torch.float64, device=self.td)
        self.dev.cosine_groups(x, self._t(offs), self._t(poffs), norms, out)
        o = out.cpu().numpy()
        return [o[poffs[i]:poffs[i + 1]] for i in range(len(groups))]


def object_means_applies(image, *objs) -> bool:
    """The merge-free per-well mean is exact when the object tables carry no Image metadata of
    their own and every object's ImageNumber names exactly one Image row."""
    if not image["ImageNumber"].is_unique:
        return False
    meta = set(IMAGE_META) - {"ImageNumber"}
    ids = image["ImageNumber"].to_numpy()
    for o in objs:
        if meta & set(o.columns) or not np.isin(o["ImageNumber"].to_numpy(), ids).all():
            return False
    return True


def double_sigmoid_host(x):
    """Pycyto_pertime.py:13-16 (reporting helper; the pipeline uses cpx_mad_transform)."""
    return (x / ALPHA) ** K_SIG / np.sqrt(1 + (x / ALPHA) ** (2 * K_SIG))


def read_table(path: str):
    """Pycyto_pertime.py:19-27: the delimiter (';' or ',') is sniffed from the first 1 KiB.
    Divergence: where the sniffer cannot decide (narrow tables, whose first 1 KiB holds several
    lines and a cut one — CellProfiler's wide tables never hit this, the reference would raise
    csv.Error) the table is read with ','."""
    import pandas as pd
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    try:
        sep = csv.Sniffer().sniff(text[:1024], delimiters=";,").delimiter
    except csv.Error:
        sep = ","
    return pd.read_csv(io.StringIO(text), sep=sep)


def well_profiles(eng: ProfileEngine, image, nuclei, cells, cytoplasm):
    """Pycyto_pertime.py:51-76: metadata attach, column drops, per-well means, Image_ prefix,
    outer merge of cells, nuclei, Image, cytoplasm on the four keys."""
    import pandas as pd
    keep = {"Metadata_Plate", "Metadata_Timepoint", "Metadata_Well", "Metadata_Site",
            "Metadata_Compound", "Metadata_ConcLevel"}
    if "Metadata_Site" not in nuclei.columns and object_means_applies(image, nuclei, cells, cytoplasm):
        # same frames as the merge -> drop -> groupby below, without copying the object tables
        nuclei, cells, cytoplasm = (eng.object_means(t, image) for t in (nuclei, cells, cytoplasm))
        image = image.drop(["ImageNumber"], axis=1)
        image = image.drop(columns=[c for c in image.columns
                                    if image[c].dtype == "object" and not c.startswith("Metadata")])
        image = eng.group_mean(image).rename(columns=lambda x: "Image_" + x if x not in keep else x)
        return reduce(lambda l, r: pd.merge(l, r, on=KEYS, how="outer"), [cells, nuclei, image, cytoplasm])
    if "Metadata_Site" not in nuclei.columns:
        meta = image[IMAGE_META]
        nuclei = nuclei.merge(meta, on="ImageNumber", how="left")
        cells = cells.merge(meta, on="ImageNumber", how="left")
        cytoplasm = cytoplasm.merge(meta, on="ImageNumber", how="left")
    drop = ["ImageNumber", "Metadata_Site", "Metadata_ConcLevel"]
    nuclei, cells, cytoplasm = (t.drop(drop, axis=1) for t in (nuclei, cells, cytoplasm))
    image = image.drop(["ImageNumber"], axis=1)
    image = image.drop(columns=[c for c in image.columns
                                if image[c].dtype == "object" and not c.startswith("Metadata")])
    nuclei, cells, cytoplasm, image = (eng.group_mean(t) for t in (nuclei, cells, cytoplasm, image))
    image = image.rename(columns=lambda x: "Image_" + x if x not in keep else x)
    return reduce(lambda l, r: pd.merge(l, r, on=KEYS, how="outer"), [cells, nuclei, image, cytoplasm])


def profile_time(eng: ProfileEngine, image, nuclei, cells, cytoplasm, plate: str, time: str,
                 tmp_csv: str):
    """Pycyto_pertime.py:51-156 for one time point -> (selected, averaged similarities,
    similarities) frames."""
    import pandas as pd
    df = well_profiles(eng, image, nuclei, cells, cytoplasm)
    df["Metadata_Timepoint"] = time
    df.Metadata_Plate = plate
    feats = df.columns[~df.columns.str.contains("Metadata")].to_list()
    meta = [c for c in df.columns if c.startswith("Metadata_")]   # pycytominer infer_cp_features
    fit_mask = ((df["Metadata_Compound"] == "DMSO") & (df["Metadata_Timepoint"] == time)).to_numpy()
    Z = eng.mad_sigmoid(df.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan),
                        np.nonzero(fit_mask)[0])
    norm = df.loc[:, meta].merge(pd.DataFrame(Z, columns=feats, index=df.index),
                                 left_index=True, right_index=True)
    feats = norm.columns[~norm.columns.str.contains("Metadata")].tolist()
    drop = eng.excluded_features(norm, feats)
    norm.drop(list(drop), axis="columns").to_csv(tmp_csv, index=False)
    selected = pd.read_csv(tmp_csv)
    avg, sims = treatment_similarities(eng, selected)
    return selected, avg, sims


def treatment_similarities(eng: ProfileEngine, selected):
    """Pycyto_pertime.py:115-156: cosine similarity of the replicate wells of every
    (Compound, Timepoint, ConcLevel) combination, upper triangle and its mean."""
    import pandas as pd
    cp = selected.drop(columns=["Metadata_Plate", "Metadata_Well", "Metadata_Site"])
    combos = cp[["Metadata_Compound", "Metadata_Timepoint", "Metadata_ConcLevel"]].drop_duplicates().values
    groups, frames = [], []
    for code, tp, conc in combos:
        group = cp[(cp["Metadata_Compound"] == code) & (cp["Metadata_Timepoint"] == tp) &
                   (cp["Metadata_ConcLevel"] == conc)]
        if len(group) == 0:   # sklearn rejects an empty sample (NaN ConcLevel never matches)
            raise ValueError(f"Found array with 0 sample(s) for group {(code, tp, conc)}")
        f = group.drop(columns=["Metadata_Compound", "Metadata_Timepoint", "Metadata_ConcLevel"]).fillna(0)
        groups.append(f.to_numpy(dtype=np.float64))
        frames.append(group)
    sims_all = eng.group_cosine(groups)
    avg, sims = [], []
    for (code, tp, conc), group, vals in zip(combos, frames, sims_all):
        avg.append({"Metadata_compound_code": code, "Metadata_Timepoint": tp,
                    "Metadata_compound_concentration": conc,
                    "average_cosine_similarity": np.mean(vals) if len(vals) > 0 else np.nan})
        sims.append({"Metadata_Compound": code, "Metadata_Timepoint": tp, "Metadata_Condition": conc,
                     "Replicates": group.index, "cosine_similarities": vals})
    return pd.DataFrame(avg), pd.DataFrame(sims)


def concatenate_csv(bucket_name: str, times, base_folder_path: str, output_bucket: str,
                    output_prefix: str, local_dir: str = "temp_data", dev=None):
    """Pycyto_pertime.py:29-172 `concatenate_csv_from_s3` over local directories: reads
    `<bucket_name>/<base_folder_path>/<time>/*.csv`, writes `<output_bucket>/<output_prefix>/
    <time>/{CP_features_selected, CPfeatures_average_cosine_similarity,
    CPfeatures_cosine_similarities}.csv`."""
    eng = ProfileEngine(dev)
    os.makedirs(local_dir, exist_ok=True)
    written = []
    for time in times:
        print(time)
        src = os.path.join(bucket_name, base_folder_path, str(time))
        tables = {n: read_table(os.path.join(src, f"{n}.csv")) for n in ("Image", "Nuclei", "Cells", "Cytoplasm")}
        selected, avg, sims = profile_time(eng, tables["Image"], tables["Nuclei"], tables["Cells"],
                                           tables["Cytoplasm"], base_folder_path.split("/")[-1], time,
                                           os.path.join(local_dir, "normalized_cpfeature_select.csv"))
        dst = os.path.join(output_bucket, output_prefix, str(time))
        os.makedirs(dst, exist_ok=True)
        for name, frame in (("CP_features_selected", selected),
                            ("CPfeatures_average_cosine_similarity", avg),
                            ("CPfeatures_cosine_similarities", sims)):
            p = os.path.join(dst, f"{name}.csv")
            frame.to_csv(p, index=False)
            print(f"Saved to {p}")
            written.append(p)
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description="Per-time CP profiles (Pycyto_pertime.py) on the GPU.")
    ap.add_argument("--bucket_name", required=True, help="local root standing in for the input bucket")
    ap.add_argument("--base_folder", required=True)
    ap.add_argument("--times", nargs="+", required=True)
    ap.add_argument("--output_bucket", required=True, help="local root standing in for the output bucket")
    ap.add_argument("--output_prefix", required=True)
    ap.add_argument("--local_dir", default="temp_data")
    a = ap.parse_args(argv)
    print(f"Processing Plate {a.base_folder}...")
    concatenate_csv(a.bucket_name, a.times, a.base_folder, a.output_bucket, a.output_prefix, a.local_dir)


if __name__ == "__main__":
    main()

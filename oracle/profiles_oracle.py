"""CPU restatement (test infrastructure only) of the reference's per-time profile step,
Pycyto_pertime.py:29-172 `concatenate_csv_from_s3`:

  1. read `<base>/<time>/{Image,Nuclei,Cells,Cytoplasm}.csv` (delimiter sniffed, :19-27, :46-49);
  2. attach the Image metadata to the object tables when Metadata_Site is missing (:51-58);
  3. drop ImageNumber/Metadata_Site/Metadata_ConcLevel from the object tables and the object
     (string) columns of Image (:61-65), average every table per (Plate, Well, Timepoint,
     Compound) (:69-72), prefix Image columns with `Image_` (:74), outer-merge
     cells, nuclei, Image, cytoplasm on the four keys (:75) — pandas suffixes the duplicated
     cells/nuclei columns `_x`/`_y`, cytoplasm keeps plain names;
  4. pycytominer `normalize(method="mad_robustize")` fitted on the DMSO rows of this time
     (:83-88), `double_sigmoid` (:13-16) and abs (:89-91);
  5. pycytominer `feature_select` with variance_threshold, drop_na_columns,
     correlation_threshold, drop_outliers (:93-104), written to CSV and read back (:106);
  6. cosine similarity within each (Compound, Timepoint, ConcLevel) group, mean of the upper
     triangle (:115-156).

Numeric kernels restated here (the GPU kernels of k_profiles.hip do the same arithmetic):
  * `group_kahan_mean`: pandas groupby mean (pandas/_libs/groupby.pyx `group_mean`): per group
    and column, Kahan-compensated sum over the group's rows in row order, NaN skipped, a NaN
    compensation (from +-inf) reset to 0, mean = sum / count, NaN for count 0.  Pinned to
    pandas 2.3.3 here (the reference pins pandas 1.5.3, whose group_mean is the same).
  * `nancorr`: pandas DataFrame.corr(method="pearson") = pandas/_libs/algos.pyx `nancorr`:
    for each column pair, Welford updates over the rows where both values are finite,
    r = covxy / sqrt(ssqdmx * ssqdmy), NaN when the divisor is 0 or no rows.  Pinned to pandas.
  * `robust_mad_fit`: pycytominer RobustMAD.fit: median = pandas median (NaN skipped; even n:
    (a + b) / 2 of the two middle values, numpy's median), mad = scipy
    `median_abs_deviation(X, nan_policy="omit", scale=1/1.4826)` = median(|x - median|) /
    (1/1.4826).  Pinned to pandas/scipy; the pycytominer wrapper itself (absent from this
    image, unpinned in the reference's requirements.txt) is restated from its published
    source — parity of the composition is unpinned.
  * transform: (x - median) / (mad + 1e-18); double_sigmoid(x) = (x/alpha)**3 /
    sqrt(1 + (x/alpha)**6), alpha = 2.3538; abs.
  * feature_select operations (pycytominer defaults): variance_threshold (freq_cut 0.05:
    drop when second-most-common count / most-common count < 0.05 or fewer than two distinct
    values; unique_cut 0.01: drop when nunique / n < 0.01), drop_na_columns (NaN fraction >
    0.05), correlation_threshold (0.9, pearson: for each lower-triangle pair with r > 0.9 drop
    the member ranked later by the column's sum of |r|), drop_outliers (max|x| or |min x| > 500).
  * cosine similarity: sklearn `cosine_similarity` (rows scaled by their L2 norm, zero norms
    left as is, then Gram matrix).
"""
from __future__ import annotations

import csv
import io
import math
from functools import reduce

import numpy as np

KEYS = ["Metadata_Plate", "Metadata_Well", "Metadata_Timepoint", "Metadata_Compound"]
IMAGE_META = ["ImageNumber", "Metadata_Plate", "Metadata_Site", "Metadata_Well",
              "Metadata_Timepoint", "Metadata_Compound", "Metadata_ConcLevel"]
K_SIG = 3
ALPHA = 2.3538
MAD_SCALE = 1 / 1.4826
MAD_EPS = 1e-18


# ---------------------------------------------------------------------------- numeric kernels
def group_kahan_mean(values: np.ndarray, group: np.ndarray, n_groups: int) -> np.ndarray:
    """pandas group_mean: values [n, K] float64, group [n] in [0, n_groups) -> [n_groups, K]."""
    values = np.asarray(values, dtype=np.float64)
    n, K = values.shape
    sumx = np.zeros((n_groups, K))
    comp = np.zeros((n_groups, K))
    nobs = np.zeros((n_groups, K), dtype=np.int64)
    for i in range(n):
        g = group[i]
        if g < 0:
            continue
        v = values[i]
        ok = ~np.isnan(v)
        y = v - comp[g]
        t = sumx[g] + y
        c = (t - sumx[g]) - y
        c = np.where(np.isnan(c), 0.0, c)
        comp[g] = np.where(ok, c, comp[g])
        sumx[g] = np.where(ok, t, sumx[g])
        nobs[g] += ok
    with np.errstate(invalid="ignore", divide="ignore"):
        out = sumx / nobs
    out[nobs == 0] = np.nan
    return out


def nancorr(mat: np.ndarray) -> np.ndarray:
    """pandas nancorr (pearson, minp 1): [N, K] -> [K, K]."""
    mat = np.asarray(mat, dtype=np.float64)
    N, K = mat.shape
    fin = np.isfinite(mat)
    out = np.empty((K, K))
    for xi in range(K):
        for yi in range(xi + 1):
            both = fin[:, xi] & fin[:, yi]
            vx_all, vy_all = mat[both, xi], mat[both, yi]
            nobs = 0
            meanx = meany = ssqdmx = ssqdmy = covxy = 0.0
            for vx, vy in zip(vx_all.tolist(), vy_all.tolist()):
                nobs += 1
                dx = vx - meanx
                dy = vy - meany
                meanx += 1.0 / nobs * dx
                meany += 1.0 / nobs * dy
                ssqdmx += (vx - meanx) * dx
                ssqdmy += (vy - meany) * dy
                covxy += (vx - meanx) * dy
            if nobs < 1:
                r = math.nan
            else:
                div = math.sqrt(ssqdmx * ssqdmy)
                r = covxy / div if div != 0 else math.nan
            out[xi, yi] = out[yi, xi] = r
    return out


def median_1d(x: np.ndarray) -> float:
    """numpy median of the non-NaN values (NaN when none)."""
    x = np.sort(x[~np.isnan(x)])
    n = len(x)
    if n == 0:
        return math.nan
    if n % 2:
        return float(x[n // 2])
    return float((x[n // 2 - 1] + x[n // 2]) / 2.0)


def robust_mad_fit(X_fit: np.ndarray):
    """RobustMAD.fit on the fit rows [n, K] -> (median[K], mad[K])."""
    X_fit = np.asarray(X_fit, dtype=np.float64)
    K = X_fit.shape[1]
    med = np.empty(K)
    mad = np.empty(K)
    for j in range(K):
        col = X_fit[:, j]
        col = col[~np.isnan(col)]
        m = median_1d(col)
        med[j] = m
        mad[j] = median_1d(np.abs(col - m)) / MAD_SCALE if len(col) else math.nan
    return med, mad


def double_sigmoid(x):
    """Pycyto_pertime.py:13-16."""
    return (x / ALPHA) ** K_SIG / np.sqrt(1 + (x / ALPHA) ** (2 * K_SIG))


def mad_sigmoid_abs(X: np.ndarray, med: np.ndarray, mad: np.ndarray) -> np.ndarray:
    """Pycyto_pertime.py:83-91: RobustMAD.transform, double_sigmoid, abs."""
    Z = (np.asarray(X, dtype=np.float64) - med) / (mad + MAD_EPS)
    return np.abs(double_sigmoid(Z))


def column_stats(X: np.ndarray):
    """Per column: (na_count, nunique, top count, second count, max, min) over non-NaN values."""
    X = np.asarray(X, dtype=np.float64)
    rows = []
    for j in range(X.shape[1]):
        col = X[:, j]
        v = col[~np.isnan(col)]
        if len(v):
            _, cnt = np.unique(v, return_counts=True)
            cnt = np.sort(cnt)[::-1]
            top = int(cnt[0])
            sec = int(cnt[1]) if len(cnt) > 1 else 0
            rows.append((int(np.isnan(col).sum()), len(cnt), top, sec, float(v.max()), float(v.min())))
        else:
            rows.append((len(col), 0, 0, 0, math.nan, math.nan))
    return rows


def cosine_similarity(X: np.ndarray) -> np.ndarray:
    X = np.asarray(X, dtype=np.float64)
    nrm = np.sqrt(np.einsum("ij,ij->i", X, X))
    nrm[nrm == 0] = 1.0
    Xn = X / nrm[:, None]
    return Xn @ Xn.T


# ------------------------------------------------------------- pycytominer feature_select ops
def excluded_features(df, features, stats=None, corr=None, freq_cut=0.05, unique_cut=0.01,
                      na_cutoff=0.05, corr_threshold=0.9, outlier_cutoff=500):
    """feature_select(operation=[variance_threshold, drop_na_columns, correlation_threshold,
    drop_outliers]) exclusions; `stats` (column_stats rows) and `corr` ([K, K]) may come from the
    GPU, otherwise they are computed here."""
    import pandas as pd
    X = df.loc[:, features].to_numpy(dtype=np.float64, na_value=np.nan)
    n = X.shape[0]
    if stats is None:
        stats = column_stats(X)
    if corr is None:   # pandas' own nancorr (C); nancorr() above restates it (pinned in tests)
        corr = pd.DataFrame(X).corr().to_numpy()
    out = set()
    for name, (na, nuniq, top, sec, mx, mn) in zip(features, stats):
        if top == 0 or sec == 0 or sec / top < freq_cut:   # calculate_frequency -> NaN
            out.add(name)
        if nuniq / n < unique_cut:
            out.add(name)
        if na / n > na_cutoff:                               # get_na_columns
            out.add(name)
        if abs(mx) > outlier_cutoff or abs(mn) > outlier_cutoff:   # drop_outlier_features
            out.add(name)
    # correlation_threshold: rank columns by the sum of |r| (pandas sum, quicksort order)
    cor_df = pd.DataFrame(corr, index=features, columns=features)
    order = cor_df.abs().sum().sort_values().index
    tri = np.tril(np.ones(corr.shape, dtype=bool), k=-1)
    ia, ib = np.nonzero(tri & (corr > corr_threshold))
    for a, b in zip(ia.tolist(), ib.tolist()):   # pair_a = row (later), pair_b = column
        pa, pb = features[a], features[b]
        out.add(pa if order.get_loc(pa) > order.get_loc(pb) else pb)
    return out


# ----------------------------------------------------------------------- table plumbing (host)
def read_table(path: str):
    """Pycyto_pertime.py:19-27: sniff ';' or ',' on the first 1024 characters."""
    import pandas as pd
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    dialect = csv.Sniffer().sniff(text[:1024], delimiters=";,")
    return pd.read_csv(io.StringIO(text), sep=dialect.delimiter)


def well_tables(image, nuclei, cells, cytoplasm, mean_fn=None):
    """Pycyto_pertime.py:51-76 -> the merged per-well frame.  `mean_fn(frame) -> frame` replaces
    `groupby(KEYS, as_index=False).mean()` (the GPU path passes its kernel here)."""
    if mean_fn is None:
        def mean_fn(d):
            # pandas 1.5.3 (the reference's pin) silently drops non-numeric columns here
            return d.groupby(KEYS, as_index=False).mean(numeric_only=True)
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
    nuclei, cells, cytoplasm, image = (mean_fn(t) for t in (nuclei, cells, cytoplasm, image))
    keep = {"Metadata_Plate", "Metadata_Timepoint", "Metadata_Well", "Metadata_Site",
            "Metadata_Compound", "Metadata_ConcLevel"}
    image = image.rename(columns=lambda x: "Image_" + x if x not in keep else x)
    import pandas as pd
    return reduce(lambda l, r: pd.merge(l, r, on=KEYS, how="outer"), [cells, nuclei, image, cytoplasm])


def pycyto_pertime(image, nuclei, cells, cytoplasm, plate: str, time: str, tmp_csv: str):
    """Steps 2-6 on one time point -> (selected frame, averaged similarities, similarities)."""
    import pandas as pd
    df = well_tables(image, nuclei, cells, cytoplasm)
    df["Metadata_Timepoint"] = time
    df.Metadata_Plate = plate
    feats = df.columns[~df.columns.str.contains("Metadata")].to_list()
    meta = [c for c in df.columns if c.startswith("Metadata_")]
    fit = df.query(f"Metadata_Compound == 'DMSO' and Metadata_Timepoint == '{time}'")
    med, mad = robust_mad_fit(fit.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan))
    Z = mad_sigmoid_abs(df.loc[:, feats].to_numpy(dtype=np.float64, na_value=np.nan), med, mad)
    norm = df.loc[:, meta].merge(pd.DataFrame(Z, columns=feats, index=df.index),
                                 left_index=True, right_index=True)
    feats = norm.columns[~norm.columns.str.contains("Metadata")].tolist()
    drop = excluded_features(norm, feats)
    norm.drop(list(drop), axis="columns").to_csv(tmp_csv, index=False)
    selected = pd.read_csv(tmp_csv)
    avg, sims = group_similarities(selected)
    return selected, avg, sims


def group_similarities(selected, cos_fn=None):
    """Pycyto_pertime.py:115-156."""
    import pandas as pd
    cos_fn = cos_fn or cosine_similarity
    cp = selected.drop(columns=["Metadata_Plate", "Metadata_Well", "Metadata_Site"])
    avg, sims = [], []
    for code, tp, conc in cp[["Metadata_Compound", "Metadata_Timepoint",
                              "Metadata_ConcLevel"]].drop_duplicates().values:
        group = cp[(cp["Metadata_Compound"] == code) & (cp["Metadata_Timepoint"] == tp) &
                   (cp["Metadata_ConcLevel"] == conc)]
        f = group.drop(columns=["Metadata_Compound", "Metadata_Timepoint", "Metadata_ConcLevel"]).fillna(0)
        s = cos_fn(f.to_numpy(dtype=np.float64))
        vals = s[np.triu_indices_from(s, k=1)]
        avg.append({"Metadata_compound_code": code, "Metadata_Timepoint": tp,
                    "Metadata_compound_concentration": conc,
                    "average_cosine_similarity": np.mean(vals) if len(vals) > 0 else np.nan})
        sims.append({"Metadata_Compound": code, "Metadata_Timepoint": tp, "Metadata_Condition": conc,
                     "Replicates": group.index, "cosine_similarities": vals})
    return pd.DataFrame(avg), pd.DataFrame(sims)

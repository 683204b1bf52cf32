"""Per-cell embeddings — the MI355X counterpart of Cellpose_GPU_s3fs.py.

Same contract as the reference script:
  * flags (:478-489) --bucket_input --data_base_path --num_consumers --max_workers
    --load_data_key --csv_image_key --channels --out_data_path --single_cell --save_coords
    --xgb_model_path --filter_dead_cells (+ --local-root: a directory standing in for S3 — the
    LoadData CSV is <local-root>/<bucket_input>/<load_data_key>, outputs go under
    <local-root>/<out_data_path>);
  * --csv_image_key: LoadData rows with ImageQC_* flags are dropped and the planes divided by
    <csv_image_key>/<ch>_illum.npy (:252-255, :53-74);
  * per site: segmentation (Cellpose nuclei, diameter 100), regionprops in label order, integer
    centroids, cells whose 200 x 200 box leaves the image dropped, masked crops, per crop and
    channel scale_to_8bit -> RGB -> EfficientNetV2-L pooler_output (1280) under fp16 autocast
    (:140-206); a site that cannot be read, or has no (kept) cell, is {'status': 'empty',
    'n_cells': 0} (:123-136, :150-152, :172-174);
  * outputs (:326-471): <out>_counts.csv (LoadData + Cell_Count [+ Dead_Cells]),
    <out>_coords.parquet (--save_coords: Cell_ID "{well}_{site}_cell{i}", Y_Center, X_Center,
    Is_Dead), <out>_well_aggregated.parquet (per Metadata_Well: mean_features = per-channel
    mean embedding, Cell_Count, first Metadata_Timepoint / Metadata_Plate), and with
    --single_cell <out>_single_cell.parquet (one row per cell: LoadData columns, Cell_Index,
    single_cell_features = the C x 1280 vector).
Design: the GPU path of cpx.pipeline (illumination, segmentation, object table, a7 crops with
the a9 scale_to_8bit fused) runs on batches of FOVs resident in HBM; libcpx
cpx_embed_preprocess does the processor's bicubic resize / normalisation (Pillow-exact 8-bit
arithmetic) straight from the crops; the EfficientNetV2-L forward runs on libcpx's fp16 MFMA
kernels (cpx.effnet_hip: k_effnet.hip), the counterpart of the reference's fp16-autocast model.  assemble() writes the reference's output
tables (host) from the per-site results, with the same float32 summation order.
Weights: timm/tf_efficientnetv2_l.in21k is a remote download, so --effnet-weights takes a local state_dict, else a seeded initialisation
(embedding values parity-unpinned).
"""
from __future__ import annotations

import argparse
import logging
import os

import numpy as np

from . import effnet
from .effnet_hip import EffNetHip

log = logging.getLogger("cpx.embed")
BOX_SIZE = 200                 # Cellpose_GPU_s3fs.py:30
INFERENCE_BATCH_SIZE = 1000    # :31 (images per forward; halved on out-of-memory)


class Embedder:
    """EfficientNetV2-L on one device: crops8 [B][ML][C][S][S] uint8 -> per FOV [n, C, 1280]."""

    def __init__(self, dev, weights: str | None = None, seed: int = 0, batch_images: int = 256,
                 size: int = effnet.INPUT_SIZE):
        import torch
        self.dev, self.torch = dev, torch
        self.size = size
        self.batch = batch_images
        # the module (host) holds the architecture and weights; the forward runs natively
        self.net = EffNetHip(effnet.build_effnet(seed=seed, state_dict_path=weights), dev)

    def pixel_values(self, crops8, index, S):
        """Preprocessed fp16 [len(index), 3, D, D] for the crop images at `index` (int64 image
        offsets into crops8)."""
        from ._lib import check
        from .device import _ptr
        torch = self.torch
        idx = torch.as_tensor(np.asarray(index, np.int64), device=self.dev.torch_device)
        out = torch.empty((len(index), 3, self.size, self.size), dtype=torch.float16, device=self.dev.torch_device)
        self.dev._bind_stream()
        check(self.dev.lib.cpx_embed_preprocess(self.dev.h, _ptr(crops8), _ptr(idx), len(index), S, self.size,
                                                float(effnet.MEAN[0]), float(effnet.STD[0]), _ptr(out)),
              "cpx_embed_preprocess")
        return out

    def forward(self, x):
        """fp16 [n, 3, D, D] pixel values (device) -> fp32 [n, 1280]."""
        return self.net(x.half().contiguous())

    def embed(self, crops8, n_kept, C: int):
        """crops8: device uint8 [B][ML][C][S][S] (slot = cell_idx); n_kept: cells per FOV."""
        torch = self.torch
        B, ML, _, S, _ = crops8.shape
        index = [((b * ML + k) * C + c) for b in range(B) for k in range(int(n_kept[b])) for c in range(C)]
        out = []
        for b in range(B):  # per site, as the reference's consumer (Cellpose_GPU_s3fs.py:184-206)
            idx = index[sum(int(n_kept[k]) for k in range(b)) * C:][: int(n_kept[b]) * C]
            feats = []
            i = 0
            while i < len(idx):
                j = min(i + self.batch, len(idx))
                try:
                    x = self.pixel_values(crops8, idx[i:j], S)
                    feats.append(self.forward(x).cpu().numpy())
                    i = j
                except torch.cuda.OutOfMemoryError:  # Cellpose_GPU_s3fs.py:196-202
                    torch.cuda.empty_cache()
                    # the halved batch size is kept for later sites; at 1 the site is given up
                    self.batch = max(1, self.batch // 2)
                    if self.batch == 1:
                        feats = None
                        break
            if feats is None:  # the reference's empty result for this site
                out.append(None)
                continue
            allf = np.concatenate(feats) if feats else np.zeros((0, effnet.FEATURE_LENGTH), np.float32)
            out.append(allf.reshape(int(n_kept[b]), C, effnet.FEATURE_LENGTH))
        return out


OUTPUT_SUFFIXES = {  # Cellpose_GPU_s3fs.py:326-471: what is written next to --out_data_path
    "counts": "_counts.csv",
    "coords": "_coords.parquet",
    "wells": "_well_aggregated.parquet",
    "wells_filtered": "_filtered_well_aggregated.parquet",
    "single_cell": "_single_cell.parquet",
}


def _site_arrays(results, index, C, L):
    """Per LoadData row (in row order): features [n, C, L] float32, coords [(y, x)], dead [n]."""
    feats, coords, dead = [], [], []
    for idx in index:
        r = results[idx]
        ok = r["status"] != "empty"
        feats.append(np.asarray(r["features"], np.float32) if ok else np.zeros((0, C, L), np.float32))
        coords.append([tuple(c) for c in r["coords"]] if ok else [])
        dead.append(np.asarray(r["is_dead"], bool) if ok else np.zeros(0, bool))
    return feats, coords, dead


def _site_sums(feats, dead, drop_dead):
    """Per site: the float32 embedding sum over its (alive) cells — numpy's axis-0 reduction, i.e.
    cells added in order — and the number of cells that entered it."""
    sums, counts = [], []
    for f, d in zip(feats, dead):
        keep = f[~d] if drop_dead else f
        counts.append(len(keep))
        sums.append(keep.sum(axis=0) if len(keep) else np.zeros(f.shape[1:], np.float32))
    return sums, counts


def _well_table(ld, sums, C, L):
    """One row per Metadata_Well (sorted, as groupby): Cell_Count (sum), first Metadata_Timepoint /
    Metadata_Plate when present, mean_features = float32 well sum / float32 count as nested lists
    (zeros when the well has no cell)."""
    import pandas as pd
    wells = ld["Metadata_Well"].to_numpy()
    keys = sorted(set(wells.tolist()))
    extra = [c for c in ("Metadata_Timepoint", "Metadata_Plate") if c in ld.columns]
    rows = []
    for w in keys:
        pos = np.flatnonzero(wells == w)
        tot = sums[pos[0]].copy()
        for p in pos[1:]:  # sites added in row order
            tot += sums[p]
        n = int(ld["Cell_Count"].to_numpy()[pos].sum())
        row = {"Metadata_Well": w, "Cell_Count": n}
        for c in extra:
            v = ld[c].iloc[pos]
            v = v[v.notna()]
            row[c] = v.iloc[0] if len(v) else np.nan
        row["mean_features"] = (tot / np.float32(n)).tolist() if n > 0 else np.zeros((C, L)).tolist()
        rows.append(row)
    return pd.DataFrame(rows, columns=["Metadata_Well", "Cell_Count", *extra, "mean_features"])


def assemble(load_data, results, channels, out_data_path, save_coords=False, single_cell=False,
             xgb=False, filter_dead_cells=False):
    """Writes the embedding outputs of Cellpose_GPU_s3fs.py:326-471 from the per-site results
    {row index: {'status', 'features' [n, C, 1280] float32, 'coords' [(y, x)], 'is_dead' [n]}}:
      counts       LoadData + Cell_Count (alive cells when dead cells are filtered) [+ Dead_Cells]
      coords       (--save_coords, when any cell) Cell_ID "{well}_{site}_cell{i}", Y/X_Center, Is_Dead
      wells        per well: Cell_Count, first timepoint / plate, mean_features (C x 1280)
      single_cell  (--single_cell) one row per cell of every non-empty site: the LoadData row
                   (original index kept), Cell_Index, single_cell_features (C * 1280)
                   [+ is_dead_cell]; no non-empty site -> the counts table itself
    Dead_Cells is the per-site dead count (0 for empty sites).  Returns the paths written."""
    import pandas as pd
    C, L = len(channels), effnet.FEATURE_LENGTH
    ld = load_data.copy()
    feats, coords, dead = _site_arrays(results, list(ld.index), C, L)
    sums, counts = _site_sums(feats, dead, xgb and filter_dead_cells)
    ld["Cell_Count"] = counts
    if xgb:
        ld["Dead_Cells"] = [int(d.sum()) for d in dead]
    path = {k: out_data_path.replace(".parquet", v) for k, v in OUTPUT_SUFFIXES.items()}
    os.makedirs(os.path.dirname(os.path.abspath(path["counts"])), exist_ok=True)
    ld.to_csv(path["counts"], index=False)
    written = [path["counts"]]
    if save_coords:
        has_site = "Metadata_Site" in ld.columns
        recs = [{"Cell_ID": f"{ld.at[idx, 'Metadata_Well']}_{ld.at[idx, 'Metadata_Site'] if has_site else str(idx)}_cell{i}",
                 "Y_Center": y, "X_Center": x, "Is_Dead": bool(d[i]) if len(d) else False}
                for idx, cs, d in zip(ld.index, coords, dead) for i, (y, x) in enumerate(cs)]
        if recs:
            pd.DataFrame(recs).to_parquet(path["coords"], engine="pyarrow")
            written.append(path["coords"])
    wpath = path["wells_filtered" if filter_dead_cells else "wells"]
    _well_table(ld, sums, C, L).to_parquet(wpath, engine="pyarrow")
    written.append(wpath)
    if single_cell:
        nz = [i for i, f in enumerate(feats) if len(f)]
        if not nz:
            ld.to_parquet(path["single_cell"], engine="pyarrow")
        else:
            reps = np.array([len(feats[i]) for i in nz])
            sc = ld.iloc[np.repeat(nz, reps)].drop(columns=["Cell_Count"]).copy()
            sc["Cell_Index"] = np.concatenate([np.arange(r) for r in reps])
            sc["single_cell_features"] = list(np.concatenate([feats[i] for i in nz]).reshape(int(reps.sum()), C * L))
            if xgb:
                sc["is_dead_cell"] = np.concatenate([dead[i] for i in nz])
            sc.to_parquet(path["single_cell"], engine="pyarrow", row_group_size=100000)
        written.append(path["single_cell"])
    return written


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="Cell segmentation, crops and EfficientNetV2-L embeddings on the GPU.")
    ap.add_argument("--bucket_input", type=str, required=True)
    ap.add_argument("--data_base_path", type=str, required=True)
    ap.add_argument("--num_consumers", type=int, default=2, help="pipelines (batches in flight) on the GPU")
    ap.add_argument("--max_workers", type=int, default=24, help="TIFF decode threads")
    ap.add_argument("--load_data_key", type=str, required=True)
    ap.add_argument("--csv_image_key", type=str, required=False)
    ap.add_argument("--channels", nargs="+", type=str, required=True)
    ap.add_argument("--out_data_path", type=str, required=True)
    ap.add_argument("--single_cell", action="store_true")
    ap.add_argument("--save_coords", action="store_true")
    ap.add_argument("--xgb_model_path", type=str, default=None)
    ap.add_argument("--filter_dead_cells", action="store_true")
    ap.add_argument("--local-root", default="", help="directory standing in for S3 (bucket/key paths)")
    ap.add_argument("--batch", type=int, default=8, help="FOVs per GPU batch")
    ap.add_argument("--effnet-weights", default=None, help="local EfficientNetV2-L state_dict")
    ap.add_argument("--cpnet-weights", default=None)
    ap.add_argument("--device", type=int, default=0)
    return ap.parse_args(argv)


def run(argv=None):
    import concurrent.futures
    import pandas as pd
    import torch
    from . import tiffio
    from .device import Device, as_numpy
    from .pipeline import FovPipeline, PipelineConfig
    from .plate import qc_filter
    a = parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    root = a.local_root
    load_data = pd.read_csv(os.path.join(root, a.bucket_input, a.load_data_key))
    if a.csv_image_key:
        load_data = qc_filter(load_data, pd.read_csv(os.path.join(a.csv_image_key, "Image.csv")))
    else:
        log.info("No csv_image_key provided — skipping image QC filtering.")
    bst = None
    if a.xgb_model_path:
        import xgboost as xgb  # the reference's optional dead-cell classifier (absent here: fails loudly)
        bst = xgb.Booster()
        bst.load_model(a.xgb_model_path)
    chans = list(a.channels)
    C = len(chans)
    tasks = [(idx, [f"{a.data_base_path}/{row[f'FileName_{c}']}" for c in chans]) for idx, row in load_data.iterrows()]
    illum = None
    if a.csv_image_key:
        illum = [np.load(f"{a.csv_image_key}/{c}_illum.npy") for c in chans]
    first = next(tiffio.imread(p[0]) for _, p in tasks if os.path.exists(p[0]))
    H, W = first.shape
    cw = a.cpnet_weights or os.path.join(os.path.dirname(__file__), "weights", "cpnet_nuclei_synth.pt")
    cfg = PipelineConfig(H=H, W=W, C=C, batch=a.batch, channels=tuple(chans), crops=True, crops_f32=False, box=BOX_SIZE,
                         weights=cw if os.path.exists(cw) else None)
    dev = Device(a.device)
    pipe = FovPipeline(dev, cfg, None if illum is None else np.stack([x.astype(np.float32) for x in illum]))
    emb = Embedder(dev, a.effnet_weights)
    results = {}

    def read(paths):
        try:
            planes = [tiffio.imread(p) for p in paths]
            if any(p.shape != (H, W) for p in planes):
                raise ValueError("plane shape")
            return np.stack(planes).astype(np.uint16)
        except Exception as e:  # noqa: BLE001 (producer sends (site_id, None))
            log.error(f"failed on site: {e}")
            return None

    B = cfg.batch
    with concurrent.futures.ThreadPoolExecutor(max(1, a.max_workers)) as ex:
        for i in range(0, len(tasks), B):
            chunk = tasks[i:i + B]
            fovs = list(ex.map(read, [p for _, p in chunk]))
            host = np.zeros((B * C, H, W), np.uint16)
            for k, f in enumerate(fovs):
                if f is not None:
                    host[k * C:(k + 1) * C] = f
            slot = pipe.run(torch.from_numpy(host.view(np.int16)).to(dev.torch_device))
            res = pipe.fetch(slot)
            kept = [0 if fovs[k] is None else int(res.hdr["Nuclei"][k]["n_kept"]) for k in range(len(chunk))]
            kept += [0] * (B - len(chunk))
            own = res.crops8 or {}  # FOVs re-run on their own carry their own crops
            feats = emb.embed(pipe.crops8, [0 if k in own else n for k, n in enumerate(kept)], C)
            for k, c8 in own.items():
                feats[k] = emb.embed(c8, [kept[k]], C)[0] if kept[k] else None
            for k, (idx, _) in enumerate(chunk):
                if fovs[k] is None or kept[k] == 0 or feats[k] is None:
                    results[idx] = {"status": "empty", "n_cells": 0}
                    continue
                o = res.objects["Nuclei"][k]
                o = o[o["kept"] != 0]
                o = o[np.argsort(o["cell_idx"])]
                f = feats[k]
                is_dead = np.zeros(len(f), dtype=bool)
                if bst is not None:
                    import xgboost as xgb
                    is_dead = bst.predict(xgb.DMatrix(f.reshape(len(f), -1))) > 0.5
                results[idx] = {"status": "success", "features": f, "n_cells": len(f),
                                "coords": list(zip(o["yc"].tolist(), o["xc"].tolist())), "is_dead": is_dead}
            log.info("sites %d-%d of %d embedded", i + 1, i + len(chunk), len(tasks))
    out_path = os.path.join(root, a.out_data_path) if root else a.out_data_path
    return assemble(load_data, results, chans, out_path, a.save_coords, a.single_cell,
                    bst is not None, a.filter_dead_cells)


if __name__ == "__main__":
    run()

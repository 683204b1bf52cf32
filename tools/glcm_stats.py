"""Development analysis (CPU only): statistics of the GLCM items of one bench FOV, to size the
per-wave GLCM work unit (k_texture.hip).  Runs the CPU restatement (oracle/cpu_pipeline) up to
the Cells / Cytoplasm labels, then for every (object set, object, channel) item and angle reports
the pair slots T, the non-background pairs, the distinct keys and how far |i - j| reaches.

    python tools/glcm_stats.py [--well 7] [--out stats.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "image-processing-suite_amd"), os.path.join(REPO, "oracle")]

import cpx_oracle as orc  # noqa: E402
import seg_oracle as so  # noqa: E402
import scipy.ndimage as ndi  # noqa: E402

OFFS = [(0, 3), (2, 2), (3, 0), (2, -2)]  # graycomatrix distance 3 at 0, 45, 90, 135 degrees


def pairs(q8, dr, dc):
    h, w = q8.shape
    r1 = h - dr
    c0, c1 = (0, w - dc) if dc >= 0 else (-dc, w)
    if r1 <= 0 or c1 <= c0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    a = q8[:r1, c0:c1].astype(np.int64).ravel()
    b = q8[dr:dr + r1, c0 + dc:c1 + dc].astype(np.int64).ravel()
    return a, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--well", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from cpx import shard
    from cpx.cpnet import build_cpnet
    from cpx.synth import synth_fovs, synth_illum
    import ws_oracle
    H = W = 2080
    C = 5
    illum = synth_illum(C, H, W, seed=1)
    raw = synth_fovs(1, C, H, W, torch.device("cpu"), seed=shard.fov_seed(shard.plate_fovs(n_wells=384)[a.well]))
    raw = raw.numpy().view(np.uint16).reshape(C, H, W)
    w = os.path.join(REPO, "image-processing-suite_amd", "cpx", "weights", "cpnet_nuclei_synth.pt")
    net = build_cpnet(seed=0, model="nuclei", state_dict_path=w)
    corr = np.stack([orc.illum_correct_producer(raw[c], illum[c]) for c in range(C)])
    Ly, Lx = so.net_size(H, W, "nuclei", 100.0)
    tiles, g = so.make_net_input(corr, Ly, Lx)
    with torch.no_grad():
        y = net(torch.from_numpy(tiles)).numpy()
    nuclei = so.compute_masks(so.average_tiles(y, g), H, W)
    cells, cyto = ws_oracle.cells_watershed(nuclei, corr[3], 15)
    rows = []
    for name, lab in (("Nuclei", nuclei), ("Cells", cells), ("Cytoplasm", cyto)):
        for i, sl in enumerate(ndi.find_objects(lab)):
            if sl is None:
                continue
            bh, bw = sl[0].stop - sl[0].start, sl[1].stop - sl[1].start
            for c in range(C):
                q8 = orc.texture_input(corr[c], lab, sl, i + 1)
                for ang, (dr, dc) in enumerate(OFFS):
                    pa, pb = pairs(q8, dr, dc)
                    nb = (pa != 0) | (pb != 0)
                    keys = pa[nb] * 256 + pb[nb]
                    both = (pa != 0) & (pb != 0)
                    d = np.abs(pa[both] - pb[both])
                    u, cnt = np.unique(keys, return_counts=True)
                    rows.append(dict(set=name, px=bh * bw, bh=bh, bw=bw, ch=c, ang=ang, T=len(pa),
                                     nonbg=int(nb.sum()), both=int(both.sum()),
                                     zero_side=int(nb.sum() - both.sum()), distinct=len(u),
                                     maxc=int(cnt.max()) if len(cnt) else 0,
                                     d16=int((d >= 16).sum()), d32=int((d >= 32).sum()),
                                     d64=int((d >= 64).sum()), dmax=int(d.max()) if len(d) else 0,
                                     vals=int(len(np.unique(q8)))))
    import pandas as pd
    df = pd.DataFrame(rows)
    print(df.groupby("set")[["px", "T", "nonbg", "both", "distinct", "maxc", "d16", "d32", "d64", "dmax",
                             "vals"]].describe(percentiles=[0.5, 0.9, 0.99]).T.to_string())
    tot = df[["T", "nonbg", "both", "zero_side", "distinct", "d16", "d32", "d64"]].sum()
    print(tot.to_string())
    print("items (x4 angles):", len(df) // 4, "px > 4096:", int((df.px > 4096).sum() // 4),
          "px > 16384:", int((df.px > 16384).sum() // 4))
    if a.out:
        df.to_json(a.out, orient="records")


if __name__ == "__main__":
    main()

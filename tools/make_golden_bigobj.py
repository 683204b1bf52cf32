"""Golden per-object features for objects at the feature kernels' fast-path limits
(tests/golden/features_boundary.npz), from scikit-image 0.18.3 — run with the survey
container's python3.9:  /opt/conda/bin/python3.9 tools/make_golden_bigobj.py

Labels: oracle/synth_golden.boundary_objects() (texture bbox just under / over 65535 px, a
2100 x 30 strip beyond the 4096-word membership mask, a 400 x 317 blob, 28 small objects);
planes: synth_golden.plane / illum (integer-only seeded generators, regenerated bit-exactly by
the tests), so the fixture holds only the expected feature rows.  Row layout = the one of
tools/make_golden.py gen_objects_features (AreaShape, then per channel Intensity + 4 x 6
greycoprops)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import synth_golden as sg  # noqa: E402

H, W, C = 2200, 720, 2


def planes():
    return np.stack([sg.plane(700 + c, H, W, n_blobs=40).astype(np.float32) /
                     sg.illum(750 + c, H, W, np.float32) for c in range(C)]).astype(np.float32)


def main():
    from skimage.feature import greycomatrix, greycoprops
    from skimage.measure import regionprops
    lab = sg.boundary_objects(H, W)
    pl = planes()
    angles = [0, np.pi / 4, np.pi / 2, 3 * np.pi / 4]
    per_ch = [regionprops(lab, intensity_image=pl[c]) for c in range(C)]
    rows = []
    for i, p in enumerate(regionprops(lab)):
        sl = p.slice
        row = [p.area, p.perimeter, p.centroid[0], p.centroid[1], p.bbox_area, p.extent,
               p.equivalent_diameter, p.major_axis_length, p.minor_axis_length, p.eccentricity,
               p.orientation, *p.bbox]
        for c in range(C):
            pr = per_ch[c][i]
            assert pr.label == p.label
            vals = pl[c][sl][p.image]
            row += [float(vals.astype(np.float64).sum()), float(pr.mean_intensity),
                    float(np.std(vals.astype(np.float64))), float(pr.min_intensity), float(pr.max_intensity)]
            crop = pl[c][sl] * (lab[sl] == p.label)
            mn, mx = np.min(crop), np.max(crop)
            q8 = np.zeros(crop.shape, np.uint8) if mx == mn else (
                255.0 * (crop.astype(np.float32) - mn) / (mx - mn)).astype(np.uint8)
            P = greycomatrix(q8, [3], angles, levels=256)
            for a in range(4):
                Pa = P[:, :, :, a:a + 1]
                row += [float(greycoprops(Pa, prop)[0, 0]) for prop in
                        ["contrast", "dissimilarity", "homogeneity", "ASM", "energy", "correlation"]]
        rows.append(row)
    out = os.path.join(REPO, "tests", "golden", "features_boundary.npz")
    np.savez_compressed(out, expected=np.array(rows, dtype=np.float64), H=H, W=W, C=C,
                        labels_sum=np.int64(lab.astype(np.int64).sum()))
    print(out, len(rows), "objects")


if __name__ == "__main__":
    main()

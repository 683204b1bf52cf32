"""CPU restatement of the reference per-FOV hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for libcpx.  It restates, in plain numpy/scipy, the arithmetic
of the reference scripts (Saguaro-Biosciences/image-processing-suite; each function cites the
file:line it follows) and of the third-party definitions the reference depends on (scikit-image
0.18.3 regionprops / greycomatrix / greycoprops, the version the survey container holds).

Pinning: every function here is checked against golden vectors in tests/golden/, which were
produced by importing the reference's own Illumination_QC_mult.py / MaxProjection.py /
Cellpose_GPU_s3fs.py helpers and scikit-image 0.18.3 (tools/make_golden.py, run under the
survey container's python3.9).  Segmentation (Cellpose) is third-party, unpinned and absent:
its restatement (seg_* functions) is "parity unpinned" against real Cellpose and is pinned only
HIP-vs-this-oracle on identical inputs.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product package (image-processing-suite_amd/cpx) never does.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage as ndi

# ----------------------------------------------------------------------------------------------
# a1: flat-field correction
# ----------------------------------------------------------------------------------------------


def illum_correct_qc(raw: np.ndarray, illum: np.ndarray | None) -> np.ndarray:
    """Illumination_QC_mult.py:145-153: astype(float) then / illum if the shapes match."""
    img = raw.astype(float)
    if illum is not None and img.shape == illum.shape:
        img = img / illum
    return img


def illum_correct_producer(raw: np.ndarray, illum: np.ndarray) -> np.ndarray:
    """Cellpose_GPU_s3fs.py:72: tifffile.imread(path) / channel_correction[n] (numpy promotion:
    uint16 / float32 -> float32)."""
    return raw / illum


# ----------------------------------------------------------------------------------------------
# a2-a4: QC metrics
# ----------------------------------------------------------------------------------------------


def rps(img: np.ndarray):
    """Illumination_QC_mult.py:31-70 (centrosome radial_power_spectrum restated there)."""
    assert img.ndim == 2
    radii2 = (np.arange(img.shape[0]).reshape((img.shape[0], 1)) ** 2) + (np.arange(img.shape[1]) ** 2)
    radii2 = np.minimum(radii2, np.flipud(radii2))
    radii2 = np.minimum(radii2, np.fliplr(radii2))
    maxwidth = min(img.shape[0], img.shape[1]) / 8.0
    if np.ptp(img) > 0:
        img = img / np.median(np.abs(img - np.mean(img)))
    mag = np.abs(np.fft.fft2(img - np.mean(img)))
    power = mag ** 2
    radii = np.floor(np.sqrt(radii2)).astype(int) + 1
    labels = np.arange(2, np.floor(maxwidth)).astype(int).tolist()
    if len(labels) > 0:
        # scipy.ndimage.sum(x, radii, labels) == per-label sum
        r = radii.ravel()
        nb = max(labels) + 1
        keep = r < nb
        magsum = np.bincount(r[keep], weights=mag.ravel()[keep], minlength=nb)[labels]
        powersum = np.bincount(r[keep], weights=power.ravel()[keep], minlength=nb)[labels]
        return np.array(labels), np.array(magsum), np.array(powersum)
    return [2], [0], [0]


def linregress_slope(x: np.ndarray, y: np.ndarray) -> float:
    """scipy.stats.linregress slope: ssxym / ssxm from np.cov(x, y, bias=1)."""
    ssxm, ssxym, _, _ = np.cov(x, y, bias=1).flat
    return float(ssxym / ssxm)


def calculate_saturation_cp_exact(image: np.ndarray, mask=None) -> float:
    """Illumination_QC_mult.py:73-95."""
    pixel_data = image[mask] if mask is not None else image
    pixel_count = pixel_data.size
    if pixel_count == 0:
        return 0.0
    max_val = np.max(pixel_data)
    number_pixels_maximal = np.sum(pixel_data == max_val)
    return 100.0 * float(number_pixels_maximal) / float(pixel_count)


def calculate_qc_metrics(image: np.ndarray, channel_name: str) -> dict:
    """Illumination_QC_mult.py:98-125 (column names and NaN/0.0 conventions kept)."""
    results = {}
    try:
        with np.errstate(all="ignore"):
            radii, magsum, powersum = rps(image)
            # the [2],[0],[0] list fallback makes `powersum > 0` raise TypeError -> NaN (ref :115)
            valid = powersum > 0
            if np.sum(valid) > 2:
                results[f"ImageQuality_PowerLogLogSlope_{channel_name}"] = linregress_slope(
                    np.log(radii[valid]), np.log(powersum[valid]))
            else:
                results[f"ImageQuality_PowerLogLogSlope_{channel_name}"] = 0.0
    except Exception:
        results[f"ImageQuality_PowerLogLogSlope_{channel_name}"] = np.nan
    try:
        results[f"ImageQuality_PercentMaximal_{channel_name}"] = calculate_saturation_cp_exact(image)
    except Exception:
        results[f"ImageQuality_PercentMaximal_{channel_name}"] = np.nan
    return results


# ----------------------------------------------------------------------------------------------
# a5: max projection
# ----------------------------------------------------------------------------------------------


def max_projection(planes: list[np.ndarray]) -> np.ndarray:
    """MaxProjection.py:42-45: shape check then np.maximum.reduce."""
    if not all(p.shape == planes[0].shape for p in planes):
        raise ValueError("Image shape mismatch in group")
    return np.maximum.reduce(planes)


def modify_imagepath(filepath: str) -> str:
    """MaxProjection.py:16-22."""
    parts = filepath.split("/")
    if "Images" not in parts:
        return filepath
    parts[parts.index("Images")] = "ImagesStacked"
    return "/".join(parts)


# ----------------------------------------------------------------------------------------------
# a7 / a9: object table, crops, 8-bit scaling
# ----------------------------------------------------------------------------------------------


def scale_to_8bit(image_16bit: np.ndarray) -> np.ndarray:
    """Cellpose_GPU_s3fs.py:34-43."""
    min_val, max_val = np.min(image_16bit), np.max(image_16bit)
    if max_val == min_val:
        return np.zeros(image_16bit.shape, dtype=np.uint8)
    scaled = 255.0 * (image_16bit.astype(np.float32) - min_val) / (max_val - min_val)
    return scaled.astype(np.uint8)


def object_table(masks: np.ndarray, box: int = 200) -> list[dict]:
    """regionprops(masks) order + Cellpose_GPU_s3fs.py:159-170 integer centroid / edge filter.

    Objects come in ascending label order (skimage uses ndi.find_objects; absent labels are
    skipped).  centroid = float64 mean of the pixel coordinates (skimage _regionprops.py
    `centroid` = coords.mean(axis=0)).  kept objects get cell_idx 0,1,... (:391-393)."""
    h, w = masks.shape
    half = box // 2
    out = []
    slices = ndi.find_objects(masks)
    kept_idx = 0
    for i, sl in enumerate(slices):
        if sl is None:
            continue
        label = i + 1
        img = masks[sl] == label
        rr, cc = np.nonzero(img)
        coords = np.vstack([rr + sl[0].start, cc + sl[1].start]).T
        centroid = coords.mean(axis=0)
        yc, xc = map(int, centroid)
        kept = not ((yc - half < 0) or (yc + half > h) or (xc - half < 0) or (xc + half > w))
        out.append(dict(label=label, area=int(img.sum()),
                        bbox=(sl[0].start, sl[1].start, sl[0].stop, sl[1].stop),
                        centroid=(float(centroid[0]), float(centroid[1])), yc=yc, xc=xc,
                        kept=kept, cell_idx=kept_idx if kept else -1))
        if kept:
            kept_idx += 1
    return out


def crops(image_hwc: np.ndarray, masks: np.ndarray, table: list[dict], box: int = 200):
    """Cellpose_GPU_s3fs.py:164-170: masked box x box x C crops of kept objects, in order."""
    half = box // 2
    res = []
    for o in table:
        if not o["kept"]:
            continue
        yc, xc = o["yc"], o["xc"]
        y1, y2, x1, x2 = yc - half, yc + half, xc - half, xc + half
        binary_mask = (masks[y1:y2, x1:x2] == o["label"])[:, :, np.newaxis]
        res.append(image_hwc[y1:y2, x1:x2, :] * binary_mask)
    return res


# ----------------------------------------------------------------------------------------------
# a8: features (skimage 0.18.3 definitions, CellProfiler-style names)
# ----------------------------------------------------------------------------------------------

SHAPE_NAMES = ["AreaShape_Area", "AreaShape_Perimeter", "AreaShape_Center_Y", "AreaShape_Center_X",
               "AreaShape_BoundingBoxArea", "AreaShape_Extent", "AreaShape_EquivalentDiameter",
               "AreaShape_MajorAxisLength", "AreaShape_MinorAxisLength", "AreaShape_Eccentricity",
               "AreaShape_Orientation", "AreaShape_BoundingBoxMinimum_Y", "AreaShape_BoundingBoxMinimum_X",
               "AreaShape_BoundingBoxMaximum_Y", "AreaShape_BoundingBoxMaximum_X"]
INTENSITY_NAMES = ["IntegratedIntensity", "MeanIntensity", "StdIntensity", "MinIntensity",
                   "MaxIntensity"]
TEXTURE_PROPS = ["Contrast", "Dissimilarity", "Homogeneity", "AngularSecondMoment", "Energy",
                 "Correlation"]
GLCM_ANGLES = [0.0, np.pi / 4, np.pi / 2, 3 * np.pi / 4]
GLCM_DISTANCE = 3


def feature_names(channels: list[str]) -> list[str]:
    names = list(SHAPE_NAMES)
    for ch in channels:
        names += [f"Intensity_{n}_{ch}" for n in INTENSITY_NAMES]
        for a in range(4):
            names += [f"Texture_{p}_{ch}_{GLCM_DISTANCE}_{a:02d}_256" for p in TEXTURE_PROPS]
    return names


_STREL_4 = np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], dtype=np.uint8)


def perimeter(image: np.ndarray) -> float:
    """skimage 0.18.3 measure/_regionprops_utils.py perimeter(image, neighbourhood=4)."""
    image = image.astype(np.uint8)
    eroded = ndi.binary_erosion(image, _STREL_4, border_value=0)
    border = image - eroded
    weights = np.zeros(50, dtype=np.double)
    weights[[5, 7, 15, 17, 25, 27]] = 1
    weights[[21, 33]] = math.sqrt(2)
    weights[[13, 23]] = (1 + math.sqrt(2)) / 2
    pimg = ndi.convolve(border, np.array([[10, 2, 10], [2, 1, 2], [10, 2, 10]]), mode="constant", cval=0)
    hist = np.bincount(pimg.ravel(), minlength=50)
    return float(hist @ weights)


def _moments_central(image: np.ndarray, center, order=3):
    """skimage 0.18.3 measure/_moments.py moments_central (float64 dot-product form)."""
    calc = image.astype(np.float64)
    for dim, dim_length in enumerate(image.shape):
        delta = np.arange(dim_length, dtype=np.float64) - center[dim]
        powers_of_delta = delta[:, np.newaxis] ** np.arange(order + 1, dtype=np.float64)
        calc = np.rollaxis(calc, dim, image.ndim)
        calc = np.dot(calc, powers_of_delta)
        calc = np.rollaxis(calc, -1, dim)
    return calc


def shape_row(img: np.ndarray, sl) -> list[float]:
    """regionprops properties of one object (img = masks[bbox] == label)."""
    area = float(img.sum())
    rr, cc = np.nonzero(img)
    coords = np.vstack([rr + sl[0].start, cc + sl[1].start]).T
    centroid = coords.mean(axis=0)
    # moments (skimage: moments(image.astype(uint8), 3) -> local_centroid -> moments_central)
    u8 = img.astype(np.uint8)
    m = _moments_central(u8, (0.0, 0.0), 3)
    local_centroid = (m[1, 0] / m[0, 0], m[0, 1] / m[0, 0])
    mu = _moments_central(u8, local_centroid, 3)
    mu0 = mu[0, 0]
    T = np.zeros((2, 2))
    T[0, 0] = mu[0, 2] / mu0
    T[1, 1] = mu[2, 0] / mu0
    T[0, 1] = T[1, 0] = -mu[1, 1] / mu0
    ev = np.linalg.eigvalsh(T)
    ev = np.clip(ev, 0, None)
    l1, l2 = sorted(ev, reverse=True)
    a, b, _, c = T.flat
    if a - c == 0:
        orient = -math.pi / 4.0 if b < 0 else math.pi / 4.0
    else:
        orient = 0.5 * math.atan2(-2 * b, c - a)
    bba = float(img.size)
    return [area, perimeter(img), float(centroid[0]), float(centroid[1]), bba, area / bba,
            (4 * area / math.pi) ** 0.5, 4 * math.sqrt(l1), 4 * math.sqrt(l2),
            0.0 if l1 == 0 else math.sqrt(1 - l2 / l1), orient,
            float(sl[0].start), float(sl[1].start), float(sl[0].stop), float(sl[1].stop)]


def glcm(image: np.ndarray, distance: int, angle: float, levels: int = 256) -> np.ndarray:
    """skimage 0.18.3 greycomatrix (symmetric=False, normed=False) for one (distance, angle):
    P[i, j] counts image[r, c] = i, image[r + round(sin a * d), c + round(cos a * d)] = j."""
    dr = int(round(math.sin(angle) * distance))
    dc = int(round(math.cos(angle) * distance))
    h, w = image.shape
    r0, r1 = max(0, -dr), min(h, h - dr)
    c0, c1 = max(0, -dc), min(w, w - dc)
    if r1 <= r0 or c1 <= c0:
        return np.zeros((levels, levels), dtype=np.int64)
    a = image[r0:r1, c0:c1].astype(np.int64)
    b = image[r0 + dr:r1 + dr, c0 + dc:c1 + dc].astype(np.int64)
    return np.bincount((a * levels + b).ravel(), minlength=levels * levels).reshape(levels, levels)


def greycoprops(P: np.ndarray) -> list[float]:
    """skimage 0.18.3 feature/texture.py greycoprops for one 2-D GLCM:
    [contrast, dissimilarity, homogeneity, ASM, energy, correlation]."""
    P = P.astype(np.float64)
    s = P.sum()
    if s == 0:
        s = 1.0
    P = P / s
    n = P.shape[0]
    I, J = np.ogrid[0:n, 0:n]
    con = float(np.sum(P * (I - J) ** 2))
    dis = float(np.sum(P * np.abs(I - J)))
    hom = float(np.sum(P * (1.0 / (1.0 + (I - J) ** 2))))
    asm = float(np.sum(P ** 2))
    ene = math.sqrt(asm)
    Ii = np.arange(n).reshape(n, 1)
    Jj = np.arange(n).reshape(1, n)
    di = Ii - np.sum(Ii * P)
    dj = Jj - np.sum(Jj * P)
    std_i = math.sqrt(np.sum(P * di ** 2))
    std_j = math.sqrt(np.sum(P * dj ** 2))
    cov = float(np.sum(P * (di * dj)))
    cor = 1.0 if (std_i < 1e-15 or std_j < 1e-15) else cov / (std_i * std_j)
    return [con, dis, hom, asm, ene, cor]


def intensity_row(vals32: np.ndarray) -> list[float]:
    """Intensity_* of one object: integrated (fp64 sum), mean (skimage mean_intensity),
    std (population, fp64), min, max."""
    v64 = vals32.astype(np.float64)
    return [float(v64.sum()), float(np.mean(vals32)), float(np.std(v64)), float(vals32.min()),
            float(vals32.max())]


def texture_input(plane32: np.ndarray, masks: np.ndarray, sl, label: int) -> np.ndarray:
    """Masked bbox crop quantised by scale_to_8bit (Cellpose_GPU_s3fs.py:34-43, :169)."""
    crop = plane32[sl] * (masks[sl] == label)
    return scale_to_8bit(crop)


def expand_labels(label_image: np.ndarray, distance: int) -> np.ndarray:
    """skimage 0.18.3 segmentation.expand_labels (scipy exact EDT feature transform)."""
    distances, nearest = ndi.distance_transform_edt(label_image == 0, return_indices=True)
    out = np.zeros_like(label_image)
    dil = distances <= distance
    out[dil] = label_image[tuple(idx[dil] for idx in nearest)]
    return out


def secondary_objects(nuclei: np.ndarray, distance: int):
    """Cells = expand_labels(nuclei, distance); Cytoplasm = Cells where Nuclei == 0."""
    cells = expand_labels(nuclei, distance)
    cyto = np.where(nuclei == 0, cells, 0).astype(cells.dtype)
    return cells, cyto


def features(masks: np.ndarray, planes32: np.ndarray) -> np.ndarray:
    """Per-object feature matrix [n_objects, 15 + C*29] in ascending label order.
    planes32: [C, H, W] float32 corrected planes."""
    C = planes32.shape[0]
    rows = []
    for i, sl in enumerate(ndi.find_objects(masks)):
        if sl is None:
            continue
        label = i + 1
        img = masks[sl] == label
        row = shape_row(img, sl)
        for ch in range(C):
            vals = planes32[ch][sl][img]
            row += intensity_row(vals)
            q8 = texture_input(planes32[ch], masks, sl, label)
            for a in GLCM_ANGLES:
                row += greycoprops(glcm(q8, GLCM_DISTANCE, a))
        rows.append(row)
    return np.array(rows, dtype=np.float64).reshape(len(rows), 15 + C * 29)

"""GPU image QC host: per-site QC worker and CLI with the reference's contract, math on MI355X.

Contract kept from the reference (Illumination_QC_mult.py):
  * flags --load-data --data-path --illum-path --channels --output --threads (:17-25);
  * per channel ImageQuality_PowerLogLogSlope_<ch> and ImageQuality_PercentMaximal_<ch>;
    slope 0.0 when at most two rings carry power, NaN on the exception path; a missing plane
    gives QC_Error_<ch> = "File Not Found", another failure the exception text (:98-162);
  * flat-field per channel from <ch>_illum.npy, else Illum<ch>.npy, else none; an illum of
    another shape than the plane is ignored (:148-153, :180-199);
  * stale ImageQuality_* / QC_Error columns dropped, new ones appended per row (:171-225).
Design: host threads only decode TIFFs.  The CLI (`main`) batches sites: `--batch` decoded
sites whose planes are all present, 2-D uint16 of one shape go to the GPU in ONE call
(cpx_illum_correct + cpx_qc_rps over batch x C planes: flat-field, PercentMaximal, fp64
pruned-FFT ring spectrum + slope); sites that are not (a missing or unreadable plane, another
dtype or shape, a flat-field of another shape) take the per-site path `process_site`, which is
also the drop-in worker for callers that drive their own pool.  One libcpx context per process;
GPU calls are serialised by the session lock.

    python -m cpx.qc --load-data LoadData.csv --data-path IMAGES --illum-path ILLUM \
                     --channels DNA AGP Mito --output QC_Results.csv --threads 24 [--batch 16]
"""
from __future__ import annotations

import argparse
import concurrent.futures
import ctypes as ct
import logging
import os

import numpy as np

from . import _lib
from . import tiffio

log = logging.getLogger("cpx.qc")
_SESSION = None


def session():
    """The process-wide GPU session (created on first use)."""
    global _SESSION
    if _SESSION is None:
        from .fov import FovSession
        _SESSION = FovSession(int(os.environ.get("CPX_DEVICE", "0")))
    return _SESSION


def parse_args(argv=None):
    """Command line of the GPU QC tool (flag names and meaning as the reference CLI)."""
    ap = argparse.ArgumentParser(prog="python -m cpx.qc",
                                 description="image QC (PowerLogLogSlope, PercentMaximal) on the GPU")
    ap.add_argument("--load-data", required=True, help="LoadData CSV (FileName_<channel> columns)")
    ap.add_argument("--data-path", required=True, help="folder the FileName_* entries are relative to")
    ap.add_argument("--illum-path", default=None, help="folder with per-channel flat-field .npy files")
    ap.add_argument("--channels", nargs="+", required=True, help="channel names, in column order")
    ap.add_argument("--output", default="QC_Results.csv", help="CSV written with the QC columns appended")
    ap.add_argument("--threads", type=int, default=24, help="host threads decoding TIFF planes")
    ap.add_argument("--batch", type=int, default=16, help="sites per GPU call (1 = one call per site)")
    return ap.parse_args(argv)


def _metrics(ch_name, slope, pct, status):
    res = {}
    res[f'ImageQuality_PowerLogLogSlope_{ch_name}'] = float('nan') if status == _lib.CPX_QC_NAN else (
        0.0 if status == _lib.CPX_QC_FLAT else float(slope))
    res[f'ImageQuality_PercentMaximal_{ch_name}'] = float(pct)
    return res


def calculate_qc_metrics(image, channel_name):
    """Both QC measures of one float image (already flat-field corrected on the host)."""
    s = session()
    torch = s.torch
    img = np.ascontiguousarray(image, dtype=np.float64)
    if img.ndim != 2:
        return {f'ImageQuality_PowerLogLogSlope_{channel_name}': float('nan'),
                f'ImageQuality_PercentMaximal_{channel_name}': float('nan')}
    H, W = img.shape
    with s.lock:
        t = torch.from_numpy(img).to(s.td)
        stats = torch.empty(64, dtype=torch.uint8, device=s.td)
        qc = torch.empty(24, dtype=torch.uint8, device=s.td)
        p = ct.c_void_p(t.data_ptr())
        # CPX_DTYPE_IMAGE_F64: the "illum" argument is the float64 plane itself
        _lib.check(s.lib.cpx_illum_correct(s.h, p, p, _lib.CPX_DTYPE_IMAGE_F64, 1, 1, H, W, None,
                                           ct.c_void_p(stats.data_ptr())), "cpx_illum_correct")
        _lib.check(s.lib.cpx_qc_rps(s.h, p, p, _lib.CPX_DTYPE_IMAGE_F64, 1, 1, H, W,
                                    ct.c_void_p(stats.data_ptr()), None, ct.c_void_p(qc.data_ptr())),
                   "cpx_qc_rps")
        q = np.frombuffer(qc.cpu().numpy().tobytes(), dtype=[("slope", "f8"), ("pct_max", "f8"),
                                                             ("n_valid", "i4"), ("n_rings", "i4")])[0]
    st = _lib.CPX_QC_NAN if q["slope"] != q["slope"] else (
        _lib.CPX_QC_FLAT if q["n_valid"] <= 2 else _lib.CPX_QC_OK)
    return _metrics(channel_name, q["slope"], q["pct_max"], st)


def _read(path):
    return tiffio.imread(path)


def process_site(site_data):
    """Worker for one site (row): same tuple in, (index, dict) out as the reference.  Keys are
    inserted in channel order, as the reference's per-channel loop does."""
    index, paths, channels, illum_cache = site_data
    per = [dict() for _ in channels]
    planes, idx = [], []
    for i, (path, ch_name) in enumerate(zip(paths, channels)):
        try:
            if not os.path.exists(path):
                per[i][f"QC_Error_{ch_name}"] = "File Not Found"
                continue
            img = _read(path)
            if img.ndim != 2:
                raise ValueError(f"expected a 2-D plane, got shape {img.shape}")
            planes.append(img)
            idx.append(i)
        except Exception as e:  # noqa: BLE001 (the reference reports str(e) per channel)
            per[i][f"QC_Error_{ch_name}"] = str(e)
    if planes:
        s = session()
        if all(p.shape == planes[0].shape and p.dtype == np.uint16 for p in planes):
            # one submission per site: channel k of the submission uses illum slot k
            try:
                with s.lock:
                    for k, i in enumerate(idx):
                        s.set_illum(k, illum_cache[i] if illum_cache else None)
                    s.submit(planes, C=len(planes))
                    slope, pct, st = s.qc()
                for k, i in enumerate(idx):
                    per[i].update(_metrics(channels[i], slope[k], pct[k], st[k]))
            except Exception as e:  # noqa: BLE001
                for i in idx:
                    per[i][f"QC_Error_{channels[i]}"] = str(e)
        else:
            # mixed shapes / non-uint16 planes: the reference's per-channel float path
            for img, i in zip(planes, idx):
                try:
                    x = img.astype(float)
                    if illum_cache and illum_cache[i] is not None and x.shape == illum_cache[i].shape:
                        x = x / illum_cache[i]
                    per[i].update(calculate_qc_metrics(x, channels[i]))
                except Exception as e:  # noqa: BLE001
                    per[i][f"QC_Error_{channels[i]}"] = str(e)
    site_results = {}
    for d in per:
        site_results.update(d)
    return index, site_results


def _decode_site(site_data):
    """Reader-thread half of a site: (index, planes or None).  None = the site needs the
    per-site path (a plane missing / unreadable / not 2-D uint16 / shapes differ)."""
    index, paths, channels, illum_cache = site_data
    planes = []
    try:
        for path in paths:
            if not os.path.exists(path):
                return index, None
            img = _read(path)
            if img.ndim != 2 or img.dtype != np.uint16 or (planes and img.shape != planes[0].shape):
                return index, None
            planes.append(img)
    except Exception:  # noqa: BLE001 (the per-site path reports the error per channel)
        return index, None
    return index, planes


class _BatchQC:
    """One GPU call for a batch of clean sites: raw planes [n*C][H][W] (plane p = channel
    p % C), the flat-fields [C][H][W] when every channel has one of the plane shape."""

    def __init__(self, channels, illum):
        self.channels, self.illum = channels, illum
        self.s = session()
        self._ill_dev = {}

    def _illum_dev(self, H, W):
        if (H, W) not in self._ill_dev:
            t = None
            ill = self.illum
            if ill and all(a is not None and a.shape == (H, W) for a in ill):
                a = np.stack([np.asarray(x) for x in ill])
                if a.dtype not in (np.float32, np.float64):
                    a = a.astype(np.float64)
                t = self.s.torch.from_numpy(np.ascontiguousarray(a)).to(self.s.td)
            self._ill_dev[(H, W)] = t
        return self._ill_dev[(H, W)]

    def usable(self, H, W):
        """Batched path only when the flat-fields apply uniformly (all of this shape, or none)."""
        ill = self.illum
        return (not ill or all(a is None for a in ill) or self._illum_dev(H, W) is not None)

    def run(self, sites):
        """sites: [(index, planes)] of one shape -> {index: result dict}."""
        from .device import _illum_dtype, _ptr
        torch, s = self.s.torch, self.s
        C = len(self.channels)
        H, W = sites[0][1][0].shape
        n = len(sites) * C
        host = np.stack([p for _, planes in sites for p in planes]).view(np.int16)
        ill = self._illum_dev(H, W)
        with s.lock:
            raw = torch.from_numpy(host).to(s.td)
            stats = torch.empty(64 * n, dtype=torch.uint8, device=s.td)
            qc = torch.empty(24 * n, dtype=torch.uint8, device=s.td)
            _lib.check(s.lib.cpx_illum_correct(s.h, _ptr(raw), _ptr(ill), _illum_dtype(ill), C, n, H, W, None,
                                               _ptr(stats)), "cpx_illum_correct")
            _lib.check(s.lib.cpx_qc_rps(s.h, _ptr(raw), _ptr(ill), _illum_dtype(ill), C, n, H, W, _ptr(stats),
                                        None, _ptr(qc)), "cpx_qc_rps")
            q = np.frombuffer(qc.cpu().numpy().tobytes(), dtype=[("slope", "f8"), ("pct_max", "f8"),
                                                                 ("n_valid", "i4"), ("n_rings", "i4")])
        out = {}
        for k, (index, _) in enumerate(sites):
            res = {}
            for c, ch in enumerate(self.channels):
                r = q[k * C + c]
                st = _lib.CPX_QC_NAN if r["slope"] != r["slope"] else (
                    _lib.CPX_QC_FLAT if r["n_valid"] <= 2 else _lib.CPX_QC_OK)
                res.update(_metrics(ch, r["slope"], r["pct_max"], st))
            out[index] = res
        return out


def run_sites(jobs, channels, illum, threads, batch):
    """All sites of a LoadData table -> {index: result dict}: reader threads decode, the GPU
    takes `batch` clean sites of one shape per call, the rest go through process_site."""
    per_site = {}
    bq = _BatchQC(channels, illum)
    pending = {}  # shape -> [(index, planes)]

    def flush(shape):
        group = pending.pop(shape, [])
        if group:
            per_site.update(bq.run(group))

    by_index = {j[0]: j for j in jobs}
    with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        for index, planes in pool.map(_decode_site, jobs):
            if planes is None or batch <= 1 or not bq.usable(*planes[0].shape):
                per_site[index] = process_site(by_index[index])[1]
                continue
            shape = planes[0].shape
            pending.setdefault(shape, []).append((index, planes))
            if len(pending[shape]) >= batch:
                flush(shape)
        for shape in list(pending):
            flush(shape)
    return per_site


def load_illum(illum_path, channels):
    """Flat-field per channel: <ch>_illum.npy, else Illum<ch>.npy, else None (raw planes)."""
    if not illum_path:
        return [None] * len(channels)
    found = []
    for ch in channels:
        arr = None
        for name in (f"{ch}_illum.npy", f"Illum{ch}.npy"):
            path = os.path.join(illum_path, name)
            if os.path.exists(path):
                arr = np.load(path)
                log.info("flat-field for %s: %s", ch, name)
                break
        if arr is None:
            log.warning("no flat-field for %s; raw planes are used", ch)
        found.append(arr)
    return found


def main(argv=None):
    import pandas as pd
    args = parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s: %(message)s")
    table = pd.read_csv(args.load_data)
    stale = [c for c in table.columns if "ImageQuality_" in c or "QC_Error" in c]
    table = table.drop(columns=stale) if stale else table
    illum = load_illum(args.illum_path, args.channels)
    cols = [f"FileName_{ch}" for ch in args.channels]
    jobs = [(i, [os.path.join(args.data_path, r[c]) for c in cols], args.channels, illum)
            for i, r in table.iterrows()]
    log.info("%d sites, %d channels, %d reader threads, %d sites per GPU call", len(jobs),
             len(args.channels), args.threads, args.batch)
    session()
    per_site = run_sites(jobs, args.channels, illum, args.threads, args.batch)
    # rows in table order; columns in order of first appearance (channel order within a row)
    qc = pd.DataFrame.from_dict({i: per_site[i] for i in sorted(per_site)}, orient="index")
    out = pd.concat([table, qc.sort_index()], axis=1)
    out.to_csv(args.output, index=False)
    log.info("wrote %s", args.output)
    return out


if __name__ == "__main__":
    main()

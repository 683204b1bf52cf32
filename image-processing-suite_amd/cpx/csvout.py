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
CSV_CHUNK_ROWS = 4096   # rows per native formatting call
CSV_THREADS = 16        # formatting threads (the GPU box's CPU share per GPU)


def _format_rows(lib, r0, r1, k, ptrs, types, strides) -> bytes:
    import ctypes as ct
    cap = (r1 - r0) * 33 * k
    buf = ct.create_string_buffer(max(cap, 1))
    m = lib.cpx_csv_format(r0, r1, k, ptrs, types, strides, buf, cap)
    if m < 0:
        raise RuntimeError("cpx_csv_format failed")
    return buf.raw[:m]


def format_object_rows(image_number: int, labels, feats) -> bytes:
    """The CSV rows (ImageNumber, ObjectNumber, Number_Object_Number, feature columns) of one
    FOV's objects, rows in label order: the bytes DataFrame.to_csv writes for them."""
    import ctypes as ct

    from . import _lib
    lib = _lib.load()
    labels = np.asarray(labels, dtype=np.int64)
    order = np.argsort(labels, kind="stable")
    lab = np.ascontiguousarray(labels[order])
    f = np.ascontiguousarray(np.asarray(feats, dtype=np.float64)[order])
    img = np.full(len(lab), int(image_number), np.int64)
    n, F = f.shape
    if n == 0:
        return b""
    k = 3 + F
    ptrs = (ct.c_void_p * k)(img.ctypes.data, lab.ctypes.data, lab.ctypes.data,
                             *[f.ctypes.data + 8 * j for j in range(F)])
    types = (ct.c_int * k)(0, 0, 0, *([1] * F))
    strides = (ct.c_int64 * k)(1, 1, 1, *([F] * F))
    return _format_rows(lib, 0, n, k, ptrs, types, strides)


def write_numeric_csv(path: str, names, columns, threads: int = CSV_THREADS):
    """Write a table whose columns are int64 / float64 arrays as the bytes
    pandas.DataFrame(...).to_csv(path, index=False) writes (header, then per row the ints in
    decimal and the floats as Python repr, NaN as an empty field), formatted by libcpx's
    cpx_csv_format on `threads` threads over row chunks (the call releases the GIL) and written
    in order.  columns: 1-D arrays or column views of a 2-D array (any element stride)."""
    import concurrent.futures
    import ctypes as ct

    from . import _lib
    lib = _lib.load()
    cols = []
    for c in columns:
        a = np.asarray(c)
        if a.dtype.kind in "iub":
            a = np.ascontiguousarray(a, dtype=np.int64) if a.dtype != np.int64 else a
        elif a.dtype != np.float64:
            a = a.astype(np.float64)
        if a.ndim != 1:
            raise ValueError("write_numeric_csv: columns must be 1-D")
        cols.append(a)
    n = len(cols[0]) if cols else 0
    if any(len(a) != n for a in cols) or len(names) != len(cols):
        raise ValueError("write_numeric_csv: ragged columns")
    k = len(cols)
    ptrs = (ct.c_void_p * k)(*[a.ctypes.data for a in cols])
    types = (ct.c_int * k)(*[0 if a.dtype == np.int64 else 1 for a in cols])
    strides = (ct.c_int64 * k)(*[a.strides[0] // a.itemsize for a in cols])
    if any(a.strides[0] % a.itemsize for a in cols):
        raise ValueError("write_numeric_csv: unaligned column stride")

    def fmt(r0):
        return _format_rows(lib, r0, min(n, r0 + CSV_CHUNK_ROWS), k, ptrs, types, strides)

    with open(path, "wb") as f:
        f.write((",".join(names) + "\n").encode())
        starts = range(0, n, CSV_CHUNK_ROWS)
        if threads > 1 and n > CSV_CHUNK_ROWS:
            with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as pool:
                for chunk in pool.map(fmt, starts):
                    f.write(chunk)
        else:
            for r0 in starts:
                f.write(fmt(r0))


def write_frame_csv(df, path: str):
    """DataFrame.to_csv(path, index=False), natively formatted when every column is int64 or
    float64 (the object tables), else through pandas (Image.csv with its Metadata strings)."""
    if len(df.columns) and all(str(t) in ("int64", "float64") for t in df.dtypes) and \
            all(isinstance(c, str) and not any(ch in c for ch in ',"\n\r') for c in df.columns):
        write_numeric_csv(path, list(df.columns), [df[c].to_numpy() for c in df.columns])
    else:
        df.to_csv(path, index=False)


def feature_names(channels):
    """Column names of a cpx_features row (layout of include/cpx.h: CPX_N_SHAPE shape columns,
    then per channel 5 intensity + 4 directions x 6 texture columns)."""
    names = list(SHAPE_NAMES)
    for ch in channels:
        names += [f"Intensity_{n}_{ch}" for n in INTENSITY_NAMES]
        for d in range(4):
            names += [f"Texture_{p}_{ch}_{TEXTURE_SCALE}_{d:02d}_256" for p in TEXTURE_NAMES]
    return names


class _TableStream:
    """Appends formatted CSV blocks to one file on a writer thread, in arrival order, while their
    ImageNumbers increase; finish() reports whether the file is complete and ordered."""

    def __init__(self, path: str, names):
        import queue
        import threading
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        # the rows go to a hidden partial file that finish() renames onto `path`: a job that
        # fails or is killed leaves no truncated <table>.csv for a downstream step to ingest
        self.path = path
        self.partial = os.path.join(os.path.dirname(path), f".{os.path.basename(path)}.partial")
        self.q = queue.Queue()
        self.last = None
        self.ordered = True
        self.f = open(self.partial, "wb")
        self.f.write((",".join(names) + "\n").encode())
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def put(self, image_number: int, fut):
        if self.last is not None and image_number <= self.last:
            self.ordered = False  # (the writer stops appending; write_objects rewrites sorted)
        self.last = image_number
        self.q.put(fut if self.ordered else None)

    def _run(self):
        while True:
            fut = self.q.get()
            if fut is None:
                break
            try:
                self.f.write(fut.result())
            except BaseException:  # noqa: BLE001 - write_objects rewrites the file and re-raises
                self.ordered = False
                break

    def finish(self, path: str) -> bool:
        """Complete and ordered for `path`: the partial file becomes `path` (True); otherwise it
        is removed and the caller writes the table itself (False)."""
        self.q.put(None)
        self.t.join()
        self.f.close()
        if self.ordered and os.path.abspath(path) == os.path.abspath(self.path):
            os.replace(self.partial, self.path)
            return True
        self._remove()
        return False

    def abort(self):
        self.q.put(None)
        self.t.join()
        if not self.f.closed:
            self.f.close()
        self._remove()

    def _remove(self):
        try:
            os.remove(self.partial)
        except FileNotFoundError:
            pass


class PlateTables:
    """Accumulates per-FOV results of one plate/time and writes the four CSVs."""

    def __init__(self, channels, eager_csv: bool = False, stream_dir: str | None = None):
        self.channels = list(channels)
        self.cols = feature_names(self.channels)
        self.images = []                       # dicts
        self.objects = {t: [] for t in OBJECT_TABLES}  # (ImageNumber, labels[n], feats[n, F])
        # eager_csv: each FOV's object rows are formatted on a thread pool as they are added
        # (overlapping the GPU work of the next batches); write_objects then only writes them.
        # stream_dir (with eager_csv): a writer thread per table appends the formatted blocks to
        # <stream_dir>/<table>.csv while the job runs, as long as they arrive in ImageNumber order
        # (the plate CLI's batches do); an out-of-order block makes write_objects rewrite the
        # file sorted at the end, so the bytes never depend on the order of arrival
        self._pool = None
        self._rows = {t: [] for t in OBJECT_TABLES}  # (ImageNumber, future of bytes)
        self._stream = {}
        self.streamed = set()  # tables whose file the stream completed (write_objects)
        if eager_csv:
            import concurrent.futures
            self._pool = concurrent.futures.ThreadPoolExecutor(max_workers=CSV_THREADS)
            if stream_dir is not None:
                for t in OBJECT_TABLES:
                    self._stream[t] = _TableStream(os.path.join(stream_dir, f"{t}.csv"),
                                                   ["ImageNumber", "ObjectNumber", "Number_Object_Number"] + self.cols)

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
        if self._pool is not None:
            fut = self._pool.submit(format_object_rows, int(image_number), labels, feats)
            if table in self._stream:
                # only the writer holds a streamed block: its bytes are freed once written (an
                # out-of-order job re-formats the table from self.objects in write_objects)
                self._stream[table].put(int(image_number), fut)
            else:
                self._rows[table].append((int(image_number), fut))

    def close(self):
        for st in self._stream.values():
            st.abort()
        self._stream = {}
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None

    def frames(self, objects: bool = True):
        """DataFrames of the tables (Image; with objects=True also the three object tables)."""
        import pandas as pd
        out = {"Image": pd.DataFrame(self.images).sort_values("ImageNumber", kind="stable")
               .reset_index(drop=True) if self.images else pd.DataFrame(columns=["ImageNumber"])}
        for t in (OBJECT_TABLES if objects else ()):
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

    def write_objects(self, d: str, table: str):
        """<table>.csv straight from the accumulated blocks (rows by ImageNumber, then
        ObjectNumber; the same bytes as frames()[table].to_csv(index=False))."""
        blocks = sorted(self.objects[table], key=lambda b: b[0])  # stable: FOVs in ImageNumber order
        names = ["ImageNumber", "ObjectNumber", "Number_Object_Number"] + self.cols
        st = self._stream.pop(table, None)
        if st is not None and st.finish(os.path.join(d, f"{table}.csv")):
            self.streamed.add(table)
            return  # streamed in order, complete
        if self._rows[table] and len(self._rows[table]) == len(self.objects[table]):
            with open(os.path.join(d, f"{table}.csv"), "wb") as f:
                f.write((",".join(names) + "\n").encode())
                for _, fut in sorted(self._rows[table], key=lambda b: b[0]):
                    f.write(fut.result())
            return
        if not blocks:
            self.frames_empty(table).to_csv(os.path.join(d, f"{table}.csv"), index=False)
            return
        labels = [b[1] for b in blocks]
        order = [np.argsort(lb, kind="stable") for lb in labels]
        lab = np.concatenate([lb[o] for lb, o in zip(labels, order)]).astype(np.int64)
        img = np.concatenate([np.full(len(lb), b[0], np.int64) for lb, b in zip(labels, blocks)])
        feats = np.concatenate([b[2][o] for b, o in zip(blocks, order)]) if lab.size else \
            np.zeros((0, len(self.cols)), np.float64)
        write_numeric_csv(os.path.join(d, f"{table}.csv"), names,
                          [img, lab, lab] + [feats[:, j] for j in range(feats.shape[1])])

    def frames_empty(self, table: str):
        import pandas as pd
        return pd.DataFrame(columns=["ImageNumber", "ObjectNumber", "Number_Object_Number"] + self.cols)

    def write(self, base: str, plate: str, time) -> str:
        d = os.path.join(base, str(plate), str(time))
        os.makedirs(d, exist_ok=True)
        frames = self.frames(objects=False)
        for name, df in frames.items():
            df.to_csv(os.path.join(d, f"{name}.csv"), index=False)
        for t in OBJECT_TABLES:
            self.write_objects(d, t)
        return d

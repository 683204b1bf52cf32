"""Z max-projection drop-in for MaxProjection.py, the projection on the GPU.

Contract kept from the reference (MaxProjection.py):
  * ``modify_imagepath(filepath)``: the first path component equal to ``Images`` becomes
    ``ImagesStacked``; other paths are returned unchanged (:16-22);
  * ``read_csv_from_s3(bucket_name, file_key)``: the CSV is sniffed for ``;`` or ``,`` on its
    first 1024 characters (:24-31);
  * ``max_projection(image_group, bucket_name, s3_client)``: reads the group's planes with
    ``get_object``, raises ``ValueError("Image shape mismatch in group: ...")`` on differing
    shapes, writes the element-wise maximum (dtype kept) as an uncompressed single-strip TIFF
    with ``upload_fileobj`` to ``modify_imagepath(image_group[0])`` (:33-52);
  * the CLI (``--bucket_data_set --data_set --channels --planes --bucket_images``, :54-61):
    per plate, rows in chunks of channels x planes, an incomplete chunk skipped with a warning,
    group j of a chunk = rows j + p * channels (plane-major, :75-91); a failing group is logged
    and the loop continues (:92-93).
Design: a chunk's C groups (C x Z planes in the chunk's own plane-major row order) go to the GPU
in ONE cpx_fov_submit (the z-max kernel reads Z planes per channel and writes one), instead of
C separate host reductions; a chunk with a failing group falls back to per-group calls, so the
other groups of that chunk are still written.  Storage: ``s3_client`` is any object with the
boto3 ``get_object`` / ``upload_fileobj`` methods; without boto3 the CLI's ``--local-root DIR``
maps bucket B, key K to ``DIR/B/K`` (LocalS3).

    python -m cpx.maxproj --bucket_data_set B --data_set plates.csv --channels 5 --planes 7 \\
        --bucket_images IMG [--local-root /data/s3]
"""
from __future__ import annotations

import argparse
import csv
import io
import logging
import os
import posixpath
from io import StringIO

import numpy as np

from . import tiffio

logging.basicConfig(level=logging.INFO)
logger = logging.getLogger("cpx.maxproj")

_SESSION = None


def session():
    """The process-wide GPU session (created on first use; one libcpx context per process)."""
    global _SESSION
    if _SESSION is None:
        from .fov import FovSession
        _SESSION = FovSession(int(os.environ.get("CPX_DEVICE", "0")))
    return _SESSION


class LocalS3:
    """Local-filesystem stand-in for the boto3 S3 client: bucket B, key K <-> root/B/K."""

    def __init__(self, root: str):
        self.root = root

    def _path(self, bucket, key):
        return os.path.join(self.root, bucket, *key.split("/"))

    def get_object(self, Bucket, Key):
        with open(self._path(Bucket, Key), "rb") as f:
            return {"Body": io.BytesIO(f.read())}

    def upload_fileobj(self, fileobj, bucket, key):
        p = self._path(bucket, key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(fileobj.read())


def s3_client(local_root: str | None = None):
    if local_root:
        return LocalS3(local_root)
    import boto3  # only when no local root is given
    return boto3.client("s3")


def modify_imagepath(filepath):
    parts = filepath.split('/')
    if 'Images' not in parts:
        return filepath
    parts[parts.index('Images')] = 'ImagesStacked'
    return '/'.join(parts)


def read_csv_from_s3(bucket_name, file_key, s3=None):
    import pandas as pd
    s3 = s3 if s3 is not None else s3_client()
    content = s3.get_object(Bucket=bucket_name, Key=file_key)['Body'].read().decode('utf-8')
    dialect = csv.Sniffer().sniff(content[:1024], delimiters=";,")
    return pd.read_csv(StringIO(content), sep=dialect.delimiter)


def _read_planes(image_group, bucket_name, s3_client_):
    return [tiffio.imread(s3_client_.get_object(Bucket=bucket_name, Key=k)['Body'].read())
            for k in image_group]


def _check_shapes(images, image_group):
    if not all(img.shape == images[0].shape for img in images):
        raise ValueError(f"Image shape mismatch in group: {image_group}")


def _project_on_gpu(planes, C, Z):
    """planes[z * C + c] (uint16) -> C projected planes (GPU z-max; dtype kept)."""
    s = session()
    with s.lock:
        for c in range(C):
            s.set_illum(c, None)
        s.submit(planes, C=C, Z=Z)
        return [s.read_plane(c) for c in range(C)]


def _upload(plane, key, bucket_name, s3_client_):
    s3_client_.upload_fileobj(io.BytesIO(tiffio.imwrite_bytes(plane)), bucket_name, modify_imagepath(key))


def max_projection(image_group, bucket_name, s3_client):
    """MaxProjection.max_projection: one group of Z planes -> one projected TIFF."""
    images = _read_planes(image_group, bucket_name, s3_client)
    _check_shapes(images, image_group)
    if images[0].dtype == np.uint16 and images[0].ndim == 2:
        out = _project_on_gpu(images, 1, len(images))[0]
    else:  # other dtypes / layouts: np.maximum.reduce semantics kept on the host
        out = np.maximum.reduce(images)
    _upload(out, image_group[0], bucket_name, s3_client)


def chunk_groups(df, num_channels, num_planes):
    """Yield (plate, i, [group_0 .. group_{C-1}]) per complete chunk, in the reference's order;
    group j = posixpath.join(PathName, FileName) of chunk rows j + p * num_channels."""
    size = num_channels * num_planes
    for plate in df['PlateID'].unique():
        sub = df[df['PlateID'] == plate]
        for i in range(0, len(sub), size):
            chunk = sub.iloc[i: i + size]
            if len(chunk) < size:
                logger.warning(f"Skipping incomplete chunk in plate {plate} at index {i}")
                continue
            groups = [[posixpath.join(chunk.iloc[j + p * num_channels].Image_PathName,
                                      chunk.iloc[j + p * num_channels].Image_FileName)
                       for p in range(num_planes)] for j in range(num_channels)]
            yield plate, i, groups
        logger.info(f"Plate {plate} finished! Check images in bucket.")


def project_chunk(groups, bucket_name, s3_client_, num_planes, plate=None, start=0):
    """All C groups of one chunk in one GPU submission (planes in the chunk's plane-major row
    order); any failure falls back to per-group max_projection calls with the reference's
    per-group error logging."""
    C = len(groups)
    try:
        imgs = [_read_planes(g, bucket_name, s3_client_) for g in groups]
        for g, im in zip(groups, imgs):
            _check_shapes(im, g)
        shp = imgs[0][0].shape
        if all(im[0].shape == shp and im[0].dtype == np.uint16 and im[0].ndim == 2 for im in imgs):
            planes = [imgs[c][z] for z in range(num_planes) for c in range(C)]
            outs = _project_on_gpu(planes, C, num_planes)
            for g, o in zip(groups, outs):
                _upload(o, g[0], bucket_name, s3_client_)
            return C
    except Exception:  # noqa: BLE001 - per-group handling below reports it
        pass
    ok = 0
    for j, g in enumerate(groups):
        try:
            max_projection(g, bucket_name, s3_client_)
            ok += 1
        except Exception as e:  # noqa: BLE001 (MaxProjection.py:92-93)
            logger.error(f"Error processing group {j} in chunk starting at {start} for plate {plate}: {e}")
    return ok


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="Max-project z-stacks on the GPU and upload the results.")
    ap.add_argument("--bucket_data_set", type=str, required=True, help="bucket holding the data set CSV")
    ap.add_argument("--data_set", type=str, required=True,
                    help="data set key: per-plate rows with Image_FileName, Image_PathName, PlateID, ...")
    ap.add_argument("--channels", type=int, required=True, help="Number of channels per group")
    ap.add_argument("--planes", type=int, required=True, help="Number of planes per channel")
    ap.add_argument("--bucket_images", type=str, required=True, help="bucket with the raw planes")
    ap.add_argument("--local-root", default=None, help="local directory standing in for S3 (root/bucket/key)")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    s3 = s3_client(a.local_root)
    df = read_csv_from_s3(a.bucket_data_set, a.data_set, s3)
    n = 0
    for plate, i, groups in chunk_groups(df, a.channels, a.planes):
        n += project_chunk(groups, a.bucket_images, s3, a.planes, plate, i)
    return n


if __name__ == "__main__":
    main()

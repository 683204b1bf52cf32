"""CPU: the native table writer (libcpx cpx_csv_format via cpx.csvout) writes the same bytes as
pandas.DataFrame.to_csv(index=False) — the text the reference's CSV consumers read
(Pycyto_pertime.py:46-49 reads <Object>.csv with pandas.read_csv).

Covers Python-repr float formatting at every switch point (fixed vs exponent at 1e-4 / 1e-5 and
1e15 / 1e16, ".0" on integral values, two / three exponent digits), signed zero, subnormals, the
extremes, inf, NaN (empty field), shortest round-trip digits of random doubles, int64 extremes,
and the PlateTables object tables written natively vs through pandas DataFrames.
"""
import os

import numpy as np
import pandas as pd
import pytest

from cpx import csvout


def _pandas_bytes(path, names, cols):
    df = pd.DataFrame({n: c for n, c in zip(names, cols)})
    df.to_csv(path, index=False)
    return open(path, "rb").read()


SPECIAL = [0.0, -0.0, 0.1, -0.1, 1.0, -1.0, 1e-4, 1e-5, 9.999999999999999e-05, 0.00012345, 2.5e-05,
           1e15, 1e16, 9999999999999998.0, 1.0000000000000002e16, 1234567890123456.0, 123456789012345678.0,
           5e-324, 2.2250738585072014e-308, 1.7976931348623157e308, -1.7976931348623157e308, 1e100, 1e-100,
           1e-99, 1e99, 123.0, 100.0, 0.5, 1 / 3, 2 / 3, np.pi, np.e, np.inf, -np.inf, np.nan, 65535.0,
           4.35e-7, 1e22, 1e21, 1e23, 0.3, 2.0 ** 53, 2.0 ** 53 + 2, 2.0 ** -1074, 1e-310]


def test_special_values_match_pandas(tmp_path):
    v = np.array(SPECIAL, np.float64)
    ints = np.arange(len(v), dtype=np.int64) - 3
    names = ["i", "f", "g"]
    cols = [ints, v, -v]
    want = _pandas_bytes(tmp_path / "a.csv", names, cols)
    csvout.write_numeric_csv(str(tmp_path / "b.csv"), names, cols, threads=1)
    assert open(tmp_path / "b.csv", "rb").read() == want


def test_random_doubles_and_int_extremes_match_pandas(tmp_path):
    rng = np.random.default_rng(7)
    n = 20000  # several native chunks, formatted on threads
    bits = rng.integers(0, 2 ** 63, n, dtype=np.int64).view(np.float64)  # every exponent
    bits[~np.isfinite(bits)] = 1.5
    scaled = rng.standard_normal(n) * 10.0 ** rng.integers(-8, 20, n)
    ints = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, n, dtype=np.int64)
    ints[:2] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max]
    small = rng.integers(0, 5000, n).astype(np.int64)
    names = ["ImageNumber", "a", "b", "c", "d"]
    cols = [small, bits, scaled, ints, np.round(scaled, 3)]
    want = _pandas_bytes(tmp_path / "a.csv", names, cols)
    csvout.write_numeric_csv(str(tmp_path / "b.csv"), names, cols, threads=4)
    assert open(tmp_path / "b.csv", "rb").read() == want


def test_strided_columns_and_empty_table(tmp_path):
    rng = np.random.default_rng(3)
    m = rng.standard_normal((1000, 7))
    names = [f"c{j}" for j in range(7)]
    cols = [m[:, j] for j in range(7)]  # column views of a row-major matrix
    want = _pandas_bytes(tmp_path / "a.csv", names, cols)
    csvout.write_numeric_csv(str(tmp_path / "b.csv"), names, cols)
    assert open(tmp_path / "b.csv", "rb").read() == want
    want0 = _pandas_bytes(tmp_path / "e.csv", ["x", "y"], [np.zeros(0, np.int64), np.zeros(0)])
    csvout.write_numeric_csv(str(tmp_path / "f.csv"), ["x", "y"], [np.zeros(0, np.int64), np.zeros(0)])
    assert open(tmp_path / "f.csv", "rb").read() == want0


@pytest.mark.parametrize("mode", ["pandas-free", "eager", "stream"])
def test_plate_tables_native_equals_pandas_frames(tmp_path, mode):
    """FOVs added out of order (the streamed files then fall back to a sorted rewrite) and in
    order (streamed as they arrive): every file equals the pandas frames' to_csv bytes."""
    rng = np.random.default_rng(11)
    chans = ["DNA", "ER", "RNA", "AGP", "Mito"]
    stream = str(tmp_path / "P01" / "3") if mode == "stream" else None
    t = csvout.PlateTables(chans, eager_csv=mode != "pandas-free", stream_dir=stream)
    F = len(t.cols)
    order = (5, 2, 9) if mode != "stream" else (2, 5, 9)  # (the stream test: in order)
    for img in order:  # labels out of order inside a FOV
        for s in csvout.OBJECT_TABLES:
            n = int(rng.integers(0, 40))
            labels = rng.permutation(np.arange(1, n + 1))
            feats = rng.standard_normal((n, F)) * 10.0 ** rng.integers(-6, 8, (n, F))
            feats[rng.random((n, F)) < 0.02] = np.nan
            t.add_objects(s, img, labels, feats)
        t.add_image(img, {"Metadata_Well": "A01"}, [0.1] * 5, [0.0] * 5, {"Nuclei": 1})
    d = t.write(str(tmp_path), "P01", 3)
    t.close()
    assert t.streamed == (set(csvout.OBJECT_TABLES) if mode == "stream" else set())
    for name, df in t.frames().items():
        df.to_csv(tmp_path / f"{name}.ref.csv", index=False)
        assert open(os.path.join(d, f"{name}.csv"), "rb").read() == open(tmp_path / f"{name}.ref.csv", "rb").read(), name


def test_write_frame_csv_falls_back_for_strings(tmp_path):
    df = pd.DataFrame({"ImageNumber": [1, 2], "Metadata_Well": ["A01", "B02"], "x": [0.5, np.nan]})
    csvout.write_frame_csv(df, str(tmp_path / "a.csv"))
    df.to_csv(tmp_path / "b.csv", index=False)
    assert open(tmp_path / "a.csv", "rb").read() == open(tmp_path / "b.csv", "rb").read()


def test_streamed_tables_fall_back_when_out_of_order(tmp_path):
    rng = np.random.default_rng(12)
    t = csvout.PlateTables(["DNA"], eager_csv=True, stream_dir=str(tmp_path / "P" / "1"))
    F = len(t.cols)
    for img in (3, 7, 5, 11):  # 5 after 7: the stream stops, write() rewrites sorted
        for s in csvout.OBJECT_TABLES:
            n = int(rng.integers(1, 10))
            t.add_objects(s, img, np.arange(1, n + 1), rng.standard_normal((n, F)))
        t.add_image(img, {"Metadata_Well": "A01"}, [0.1], [0.0], {"Nuclei": 1})
    d = t.write(str(tmp_path), "P", 1)
    t.close()
    assert not t.streamed  # every table saw 5 after 7: rewritten sorted
    for name, df in t.frames().items():
        df.to_csv(tmp_path / f"{name}.ref.csv", index=False)
        assert open(os.path.join(d, f"{name}.csv"), "rb").read() == open(tmp_path / f"{name}.ref.csv", "rb").read()


def test_aborted_stream_leaves_no_object_tables(tmp_path):
    """A job that fails after some FOVs were streamed (PlateTables.close() without write()): no
    <table>.csv and no partial file remain in the job directory, and while the job
    runs the rows go to hidden partial files, never to the final names."""
    rng = np.random.default_rng(13)
    d = tmp_path / "P" / "1"
    t = csvout.PlateTables(["DNA"], eager_csv=True, stream_dir=str(d))
    F = len(t.cols)
    for img in (1, 2):
        for s in csvout.OBJECT_TABLES:
            t.add_objects(s, img, np.arange(1, 4), rng.standard_normal((3, F)))
    assert not any((d / f"{s}.csv").exists() for s in csvout.OBJECT_TABLES)
    t.close()  # (plate.run's finally on an exception)
    assert sorted(os.listdir(d)) == []

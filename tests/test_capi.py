"""CPU: libcpx.so loads and exports exactly the C ABI declared in include/cpx.h (no GPU calls)."""
import ctypes as ct
import os
import re

import pytest

from conftest import REPO
from cpx import _lib


def _header_symbols():
    with open(os.path.join(REPO, "include", "cpx.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cpx_[a-z0-9_]+)\s*\(", src)))


def test_library_loads():
    lib = _lib.load()
    assert lib.cpx_abi_version() == 1


def test_every_header_symbol_is_exported_and_bound():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/cpx.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} not bound in cpx/_lib.py"
    assert sorted(_lib.SIGNATURES) == syms


def test_struct_sizes_match_header():
    assert ct.sizeof(_lib.PlaneStats) == 64
    assert ct.sizeof(_lib.QcResult) == 24
    assert ct.sizeof(_lib.LabelStats) == 64
    assert ct.sizeof(_lib.Object) == 56
    assert ct.sizeof(_lib.FovObjects) == 16
    assert ct.sizeof(_lib.ColumnStat) == 48


def test_error_paths_without_gpu():
    lib = _lib.load()
    # argument validation happens before any HIP call
    assert lib.cpx_illum_correct(None, None, None, 0, 1, 1, 1, 1, None, None) == 1
    assert b"null" in lib.cpx_last_error()
    assert lib.cpx_set_stream(None, None) == 1
    with pytest.raises(_lib.CpxError):
        _lib.check(lib.cpx_zmax_u16(None, None, 1, 1, 1, None), "cpx_zmax_u16")


def test_product_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cpx.device import Device
    with pytest.raises(_lib.CpxNativeMissing):
        Device(0)

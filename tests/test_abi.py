"""CPU tests of the C-ABI library: it loads, exports every symbol include/fia.h
declares, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from influence import _lib


def header_functions():
    src = open(os.path.join(ROOT, "include", "fia.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fia_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    names = header_functions()
    for must in ("fia_create", "fia_destroy", "fia_set_params", "fia_build_index", "fia_prepare",
                 "fia_count_related", "fia_related", "fia_query_batch", "fia_last_error"):
        assert must in names


def test_library_exports_every_header_symbol(libfia_path):
    lib = ctypes.CDLL(libfia_path)
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding declares a signature for exactly the header's functions
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_host_only_entry_points(libfia_path):
    lib = _lib.load_library(libfia_path)
    assert lib.fia_version() == 100
    assert lib.fia_last_error(None) == b""
    assert lib.fia_destroy(None) == 0
    assert lib.fia_num_params(None) == 0
    assert lib.fia_set_params(None, 0, 16, 1, 1, None, 0, 0.0, 0.0) == 1
    assert lib.fia_query_batch(None, 0, None, None, None, 0, None, None, None, 0, None, None, None, None) == 1
    assert lib.fia_query_batch_x(None, 0, None, None, None, 0, None, None, None, 0, None, None, None, None) == 1


def test_package_refuses_to_run_without_gpu(libfia_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.FIAError):
        _lib.Context(0)


def test_missing_library_is_loud(tmp_path):
    with pytest.raises(ImportError):
        _lib.load_library(str(tmp_path / "libfia.so"))

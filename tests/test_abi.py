"""CPU-side checks of the C-ABI boundary: the library loads (no GPU needed to
dlopen it) and exports every entry point include/slamhip.h declares, with the
ctypes table in slamhip/_abi.py covering all of them."""
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "slamhip.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(slam_[a-z0-9_]+)\s*\(", txt)))


def test_header_parses():
    names = declared()
    assert "slam_icp_batch_f64" in names and "slam_pgo_sgd_step_f64" in names
    assert "slam_gn_iteration_f64" in names


def test_library_exports_every_declared_symbol():
    from slamhip import _abi
    if not os.path.exists(_abi.LIB_PATH):
        pytest.fail(f"{_abi.LIB_PATH} not built (run __graft_entry__.build())")
    lib = _abi.lib()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_table_covers_header():
    from slamhip import _abi
    assert set(declared()) <= set(_abi.SIGNATURES), set(declared()) - set(_abi.SIGNATURES)


def test_host_only_calls():
    """Entry points that only validate arguments run without a GPU."""
    from slamhip import _abi
    lib = _abi.lib()
    assert lib.slam_abi_version() >= 100
    assert lib.slam_icp_max_query_points() >= 4096
    # shape validation fails loudly before any launch
    rc = lib.slam_icp_batch_f64(None, None, None, None, None, 4, 0.01, 100, 1e-4, 0, 10, 10, 0,
                                None, None, None, None, None)
    assert rc == -1 and b"null" in lib.slam_last_error()
    rc = lib.slam_kabsch2d_f64(None, None, 0, None, None, None)
    assert rc == -1
    assert lib.slam_pgo_sgd_work_size(10, 4) >= 3 * 10 + 3 * 4
    n = lib.slam_icp_num_instances()
    assert n >= 4
    # instance chooser: smallest capacity covering the scan
    import ctypes
    b, q = ctypes.c_int32(), ctypes.c_int32()
    i = lib.slam_icp_selected_instance(1081)
    assert lib.slam_icp_instance_shape(i, ctypes.byref(b), ctypes.byref(q)) == 0
    assert b.value * q.value >= 1081

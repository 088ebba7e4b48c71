"""CPU checks of the C ABI: the library loads (no GPU needed) and exports
exactly the entry points include/skge_hip.h declares; the ctypes table
mirrors skge_table_t."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "skge_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(skge_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ["skge_pair_grad", "skge_triple_grad", "skge_rescal_wgrad", "skge_accum_collect",
              "skge_update_rows", "skge_accum_apply", "skge_pair_step",
              "skge_transe_sample_grad", "skge_runner_create"]:
        assert f in fns


def test_library_loads_and_exports_every_declared_symbol():
    from skge_amd import _lib as L
    lib = L.load()
    fns = header_functions()
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing
    assert set(L.SIGNATURES) == set(fns)
    assert lib.skge_abi_version() == 2


def test_table_struct_layout():
    from skge_amd import _lib as L
    # 5 pointers, 7 ints, 4 floats, pad, 3 pointers (natural alignment) = 112 bytes
    assert ctypes.sizeof(L.SkgeTable) == 112
    assert L.SkgeTable.gate.offset == 88
    assert L.SkgeTable.violations.offset == 104


def test_errors_are_reported_without_a_gpu():
    from skge_amd import _lib as L
    lib = L.load()
    rc = lib.skge_pair_grad(None, 0, 0, None, None, 8, None, None, 1, 1.0, None, None, None, None)
    assert rc == -1
    assert b"NULL" in lib.skge_last_error()
    t = L.SkgeTable()
    rc = lib.skge_update_rows(None, ctypes.byref(t), None, None, 0)
    assert rc == -1

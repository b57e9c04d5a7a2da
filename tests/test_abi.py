"""The C-ABI library loads and exports every symbol include/waafle_hip.h declares
(no compute calls: this runs on CPU-only machines too)."""
import ctypes
import os
import re

from waafle_amd import build, lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(REPO, "include", "waafle_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(wf_\w+)\s*\(", text, re.M)))


def test_library_exports_header_symbols():
    build.build(verbose=False)
    so = ctypes.CDLL(lib.LIB_PATH)
    names = header_functions()
    assert len(names) >= 12
    for name in names:
        assert hasattr(so, name), name
    assert set(names) == set(lib.SIGNATURES)


def test_struct_layouts_match_header():
    # offsets the C compiler uses for the same declarations (x86-64 SysV)
    assert ctypes.sizeof(lib.WfParams) == 6 * 8 + 11 * 4 + 4
    assert lib.WfBatch.hit_off.offset == 40 and ctypes.sizeof(lib.WfBatch) == 40 + 12 * 8
    assert ctypes.sizeof(lib.WfResult) == 15 * 8
    assert lib.WfTaxonomy.parent.offset == 8 and lib.WfTaxonomy.root.offset == 40


def test_abi_version_and_no_device_is_an_error_not_a_crash():
    so = lib.load()
    assert so.wf_abi_version() == lib.ABI_VERSION == 5
    n = ctypes.c_int(-1)
    rc = so.wf_device_count(ctypes.byref(n))
    assert (rc == 0 and n.value >= 0) or (rc != 0 and n.value == 0)

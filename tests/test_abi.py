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
    assert lib.WfBatch.hit_off.offset == 40 and ctypes.sizeof(lib.WfBatch) == 40 + 13 * 8
    assert lib.WfBatch.hit_key.offset == 40 + 12 * 8
    assert ctypes.sizeof(lib.WfResult) == 16 * 8 and lib.WfResult.ppot_sum.offset == 15 * 8
    assert lib.WfTaxonomy.parent.offset == 8 and lib.WfTaxonomy.root.offset == 40


def test_abi_version_and_no_device_is_an_error_not_a_crash():
    so = lib.load()
    assert so.wf_abi_version() == lib.ABI_VERSION == 6
    n = ctypes.c_int(-1)
    rc = so.wf_device_count(ctypes.byref(n))
    assert (rc == 0 and n.value >= 0) or (rc != 0 and n.value == 0)


def test_pack_hit_keys_c_equals_numpy():
    """wf_pack_hit_keys (host code: no device needed) and lib.pack_hit_keys (the packer the
    CLI and the bench use) give the same words; out-of-range taxa and strands are refused."""
    import numpy as np
    rng = np.random.default_rng(3)
    n = 5000
    taxon = rng.integers(0, 1 << 24, n).astype(np.int32)
    strand = rng.integers(0, 2, n).astype(np.int8)
    scov = rng.random(n)
    scov[:10] = 0.75                                  # (the >= edge)
    sysmask = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    so = lib.load()
    out = np.zeros(n, np.uint32)
    assert so.wf_pack_hit_keys(n, lib.ptr(taxon), lib.ptr(strand), lib.ptr(scov), lib.ptr(sysmask), 0.75,
                               lib.ptr(out)) == 0
    want = lib.pack_hit_keys(taxon, strand, scov, sysmask, 0.75)
    np.testing.assert_array_equal(out, want)
    assert ((want >> 24) & 1)[:10].all()
    np.testing.assert_array_equal(want & 0xFFFFFF, taxon)
    np.testing.assert_array_equal(want >> 26, sysmask & 63)
    bad = taxon.copy()
    bad[7] = 1 << 24
    assert so.wf_pack_hit_keys(n, lib.ptr(bad), lib.ptr(strand), lib.ptr(scov), lib.ptr(sysmask), 0.75,
                               lib.ptr(out)) == lib.WF_E_BADINPUT
    s2 = strand.copy()
    s2[3] = 2
    assert so.wf_pack_hit_keys(n, lib.ptr(taxon), lib.ptr(s2), lib.ptr(scov), lib.ptr(sysmask), 0.75,
                               lib.ptr(out)) == lib.WF_E_BADINPUT

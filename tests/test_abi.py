"""The C-ABI library loads and exports every symbol include/*.h declares (no compute
calls: this runs without a GPU)."""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "era-boojum_amd", "boojum_amd", "libboojum_mi355x.so")


def declared_functions():
    names = []
    for hdr in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(hdr).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(bj_[a-z0-9_]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("bj_fft_natural_to_bitreversed_d", "bj_ifft_natural_to_natural_d", "bj_precompute_twiddles_d",
                 "bj_distribute_powers_d", "bj_lde_d", "bj_merkle_leaves_d", "bj_merkle_nodes_d",
                 "bj_lde_commit_d", "bj_poseidon2_permute_h", "bj_hash_into_leaf_h", "bj_hash_into_node_h"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail("library not built: run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from boojum_amd import _lib
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_library_is_gfx950_code_object():
    if not os.path.exists(LIB):
        pytest.fail("library not built")
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob  # gfx950 only, no dual paths


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "era-boojum_amd")
    for path in glob.glob(os.path.join(pkg, "**", "*.py"), recursive=True) + \
            glob.glob(os.path.join(pkg, "csrc", "*")):
        text = open(path, errors="ignore").read()
        assert "import oracle" not in text and "liboracle" not in text and "oracle.py" not in text, path

"""The C-ABI library loads without a GPU and exports every entry point include/rdeic_hip.h declares."""
import os
import re

from rdeic_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "rdeic_hip.h")


def declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rdeic_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_bindings():
    names = declared()
    assert names, "no declarations parsed"
    assert sorted(_lib.PROTOTYPES) == names


def test_library_exports_all_symbols():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.rdeic_abi_count() == len(declared())
    assert lib.rdeic_version() >= 1

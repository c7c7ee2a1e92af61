"""CPU-side checks of the C-ABI boundary: the library loads and exports every symbol that
include/imgcap_abi.h declares (no compute calls: there is no GPU here)."""
import os
import re

from imagecaptioningconvnext_amd import _abi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "imgcap_abi.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(imgcap_\w+)\s*\(", src, re.M)))


def test_header_matches_binding():
    assert _declared() == sorted(_abi.exported_symbols())


def test_library_loads_and_exports_all():
    L = _abi.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert L.imgcap_version() == 1

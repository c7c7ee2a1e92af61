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
    assert L.imgcap_version() == _abi.ABI_VERSION


def test_abi_version_matches_header():
    m = re.search(r"#define\s+IMGCAP_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _abi.ABI_VERSION


def _declared_arity():
    """name -> parameter count of every prototype in the header (comments stripped; `void` = 0)."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:int|const char\*)\s+(imgcap_\w+)\s*\(([^)]*)\)\s*;", src, re.M):
        params = m.group(2).strip()
        out[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return out


def test_binding_arity_matches_header():
    """ctypes argtypes of every entry point have the header's parameter count (a missing or extra
    argument would shift every later one at the call)."""
    ar = _declared_arity()
    assert set(ar) == set(_abi.exported_symbols())
    bad = {n: (ar[n], len(_abi._SIGS[n])) for n in _abi._SIGS if ar[n] != len(_abi._SIGS[n])}
    assert not bad, bad

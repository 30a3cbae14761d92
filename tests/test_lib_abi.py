"""CPU-side checks of the C ABI: the library builds, loads and exports every
symbol that include/dl4ss_hip.h declares (no compute calls without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dl4ss_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|long long|void) (dl4ss_\w+)\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "dl4ss_stft_fwd" in syms and len(syms) >= 3


def test_library_exports_every_declared_symbol():
    from dl4ss_amd import build, _lib

    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), f"missing export {s}"
    # the Python binding knows every declared symbol, and nothing undeclared
    assert sorted(_lib.SIGNATURES) == declared_symbols()

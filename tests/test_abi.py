"""The C-ABI library builds for gfx950, loads, and exports exactly what
include/othello.h declares (no compute calls: CPU only)."""
import ctypes
import os
import re
import subprocess

from subproc_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(_lib.HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(oth_\w+)\s*\(", src, re.M)))


def test_header_declares_the_binding():
    assert header_functions() == sorted(_lib.SIGNATURES)


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (oth_\w+)$", out, re.M))
    assert exported == set(header_functions())


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob  # gfx950 only, no multi-arch dispatch


def test_version_string():
    assert _lib.version().startswith("subproc_amd ") and "gfx950" in _lib.version()


def test_no_cpu_fallback_in_product():
    """The product package never imports the oracle."""
    pkg = os.path.join(ROOT, "subproc_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f

"""The C-ABI library loads and exports every symbol include/speedy_ml.h declares.
CPU-only: no compute call is made (host-only NetCDF I/O aside)."""
import os
import re
import subprocess

import numpy as np

from speedy_ml_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "speedy_ml.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sml_[a-z0-9_]+)\s*\(", txt)))


def test_library_builds_and_loads():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    L = _lib.lib()
    assert L.sml_abi_version() == 1


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    funcs = header_functions()
    assert len(funcs) >= 30
    missing = [f for f in funcs if not hasattr(L, f)]
    assert not missing, missing
    assert set(funcs) == set(_lib.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (sml_[a-z0-9_]+)", out))
    assert set(funcs) <= exported


def test_code_object_targets_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_fortran_binding_compiles_and_matches_header():
    fdir = os.path.join(_lib.PKG_ROOT, "fortran")
    subprocess.run(["make", "-s", "-C", fdir], check=True)
    src = open(os.path.join(fdir, "sml_hip.f90")).read()
    bound = set(re.findall(r"bind\(C, name='(sml_[a-z0-9_]+)'\)", src))
    assert len(bound) >= 15
    assert bound <= set(header_functions())


def test_error_reporting_without_gpu():
    L = _lib.lib()
    import ctypes

    h = ctypes.c_void_p()
    rc = L.sml_res_create(1000, 0, None, None, None, None, 132, 136, 1, 1.0, ctypes.byref(h))
    assert rc == -1
    assert b"does not decompose" in L.sml_last_error()

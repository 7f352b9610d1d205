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


def test_dropin_library_exports_the_reference_symbols():
    """libspeedyml_dropin.so: the single-field spectral subroutines under the Fortran
    symbols the reference's callers link against (include/speedy_ml_dropin.h)."""
    path = os.path.join(_lib.PKG_ROOT, "lib", "libspeedyml_dropin.so")
    if not os.path.exists(path):
        _lib.build()
    txt = open(os.path.join(REPO, "include", "speedy_ml_dropin.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    declared = set(re.findall(r"\b([a-z_]+_|sml_dropin_init)\s*\(", txt))
    assert {"grid_", "spec_", "vdspec_", "uvspec_", "gridy_", "specy_", "gridx_", "specx_"} <= declared
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT ([a-z_]+)\b", out))
    assert declared <= exported, declared - exported


def test_fortran_interface_module_keeps_the_reference_names():
    """speedy_res_interface.f90 exposes the reference module's public procedures with
    the same dummy-argument lists (src/speedy_res_interface.f90:20-837)."""
    src = open(os.path.join(_lib.PKG_ROOT, "fortran", "speedy_res_interface.f90")).read()
    sigs = {
        "startspeedy": "model_parameters, grid, runspeedy",
        "write_restart_new": "filename, timestep, grid4d, grid2d",
        "getspeedyvariable": "",
        "read_era_netcdf_opened": "reservoir, grid, model_parameters, start_year, end_year, era_data, netcdf_files, "
                                  "timestep_arg",
        "read_era": "reservoir, grid, model_parameters, start_year, end_year, era_data, timestep_arg",
        "read_model_states": "reservoir, grid, model_parameters, start_year, end_year, speedy_data, timestep_arg",
        "test_hybrid_speedy_component": "",
        "truncate_letkf_code_version": "field_orig, trunc_twn",
    }
    flat = re.sub(r"&\s*\n\s*", "", src)
    for name, args in sigs.items():
        m = re.search(r"(subroutine|function)\s+" + name + r"\s*\(([^)]*)\)", flat)
        assert m, name
        assert re.sub(r"\s+", " ", m.group(2)).strip() == args, (name, m.group(2))
    assert "module speedy_res_interface" in src and "internal_state_vector" in src

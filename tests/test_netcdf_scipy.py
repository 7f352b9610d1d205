"""The NetCDF-3 weight-file reader and writer (csrc/sml_netcdf.cpp) against an
independent implementation, scipy.io.netcdf_file (CPU only).

The reference writes each region's file one variable at a time: create with
NF90_CLOBBER for the first, then reopen + nf90_redef + def_dim / def_var /
put_att("units") + enddef + put_var for each of the others (write_trained_res,
src/mod_reservoir.f90:1701-1736 -> write_netcdf_2d_non_met_data /
write_netcdf_1d_non_met_data_{int,real}, src/mod_io.f90:1247-1496), so the header
is re-laid and the data sections move on every variable.  Those files are built
here the same way with scipy (a new file, then append-mode reopen per variable),
plus variants with the variables in another order, extra dimensions / variables /
global attributes and the 64-bit-offset format, and read with sml_nc_read_region.
The other way round, sml_nc_write_region's files are read with scipy."""
import numpy as np
import pytest
from scipy.io import netcdf_file

from speedy_ml_amd.reservoir import read_region_netcdf, write_region_netcdf
from speedy_ml_amd.synthetic import region_weights

# (name, dims (C order = Fortran order reversed), dtype) in write_trained_res's order
VARS = [("win", ("win_y", "win_x"), "f4"), ("wout", ("wout_y", "wout_x"), "f4"), ("rows", ("rows_x",), "i4"),
        ("cols", ("cols_x",), "i4"), ("vals", ("vals_x",), "f4"), ("mean", ("mean_x",), "f4"),
        ("std", ("std_x",), "f4")]


def _arrays(w):
    return {"win": w.win, "wout": w.wout, "rows": w.rows, "cols": w.cols, "vals": w.vals,
            "mean": w.mean.astype(np.float32), "std": w.std.astype(np.float32)}


def _write_reference_pattern(path, arrs, order=None, version=1, extras=False):
    order = order or [v[0] for v in VARS]
    spec = {v[0]: v for v in VARS}
    for i, name in enumerate(order):
        _, dims, dt = spec[name]
        f = netcdf_file(path, "w" if i == 0 else "a", version=version)
        if i == 0 and extras:
            f.history = b"written like write_trained_res"
            f.createDimension("time", 3)
            t = f.createVariable("time", "f8", ("time",))
            t[:] = np.arange(3.0)
            t.units = b"hours"
        a = arrs[name]
        for d, n in zip(dims, a.shape):
            f.createDimension(d, n)
        v = f.createVariable(name, dt, dims)
        v[...] = a
        v.units = b"unitless"
        f.close()


def _check(d, arrs):
    for k in ("win", "wout", "rows", "cols", "vals"):
        np.testing.assert_array_equal(d[k], arrs[k], err_msg=k)
    np.testing.assert_array_equal(d["mean"].astype(np.float32), arrs["mean"])
    np.testing.assert_array_equal(d["std"].astype(np.float32), arrs["std"])


@pytest.mark.parametrize("region,sst", [(5, True), (30, False), (1151, True)])
def test_reader_on_reference_pattern_files(tmp_path, region, sst):
    w = region_weights(region, sst, n_override=700, seed=17)
    arrs = _arrays(w)
    p = str(tmp_path / f"worker_{region:04d}_level_1_trial.nc")
    _write_reference_pattern(p, arrs)
    _check(read_region_netcdf(p), arrs)


@pytest.mark.parametrize("variant", ["reordered", "extras", "cdf2"])
def test_reader_layout_variants(tmp_path, variant):
    w = region_weights(77, True, n_override=600, seed=3)
    arrs = _arrays(w)
    p = str(tmp_path / "w.nc")
    if variant == "reordered":
        _write_reference_pattern(p, arrs, order=["std", "rows", "wout", "mean", "vals", "cols", "win"])
    elif variant == "extras":
        _write_reference_pattern(p, arrs, extras=True)
    else:
        _write_reference_pattern(p, arrs, version=2)
        assert open(p, "rb").read(4) == b"CDF\x02"
    _check(read_region_netcdf(p), arrs)


def test_writer_read_by_scipy(tmp_path):
    w = region_weights(600, True, n_override=500, seed=5)
    arrs = _arrays(w)
    p = str(tmp_path / "ours.nc")
    write_region_netcdf(p, w.win, w.wout, w.rows, w.cols, w.vals, w.mean, w.std)
    f = netcdf_file(p, "r", mmap=False)
    for name, dims, dt in VARS:
        v = f.variables[name]
        assert v.dimensions == dims, (name, v.dimensions)
        assert v.data.dtype == np.dtype(">" + dt), (name, v.data.dtype)
        assert v.units == b"unitless"
        np.testing.assert_array_equal(v.data, arrs[name], err_msg=name)
    f.close()

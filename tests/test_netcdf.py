"""NetCDF-3 classic weight files (read_trained_res / write_trained_res layout),
host-only code: runs on CPU."""
import numpy as np
import pytest

from speedy_ml_amd import SmlError
from speedy_ml_amd.reservoir import read_region_netcdf, write_region_netcdf
from speedy_ml_amd.synthetic import region_weights


def test_roundtrip_exact(tmp_path):
    w = region_weights(37, True, n_override=600)
    p = str(tmp_path / "worker_0037_level_1_trial.nc")
    write_region_netcdf(p, w.win, w.wout, w.rows, w.cols, w.vals, w.mean, w.std)
    d = read_region_netcdf(p)
    np.testing.assert_array_equal(d["win"], w.win)
    np.testing.assert_array_equal(d["wout"], w.wout)
    np.testing.assert_array_equal(d["rows"], w.rows)
    np.testing.assert_array_equal(d["cols"], w.cols)
    np.testing.assert_array_equal(d["vals"], w.vals)
    np.testing.assert_array_equal(d["mean"].astype(np.float64), w.mean)
    np.testing.assert_array_equal(d["std"].astype(np.float64), w.std)


def test_file_is_big_endian_cdf1_with_reference_names(tmp_path):
    w = region_weights(3, False, n_override=420)
    p = tmp_path / "w.nc"
    write_region_netcdf(str(p), w.win, w.wout, w.rows, w.cols, w.vals, w.mean, w.std)
    raw = p.read_bytes()
    assert raw[:4] == b"CDF\x01"
    for name in (b"win_x", b"win_y", b"wout_x", b"wout_y", b"rows_x", b"cols_x", b"vals_x", b"mean_x",
                 b"std_x", b"units", b"unitless"):
        assert name in raw
    # the last variable is std: 36 big-endian float32 at the end of the file
    tail = np.frombuffer(raw[-36 * 4:], dtype=">f4")
    np.testing.assert_array_equal(tail.astype(np.float64), w.std)


def test_corrupt_and_missing_files(tmp_path):
    p = tmp_path / "bad.nc"
    p.write_bytes(b"NOTNETCDF")
    with pytest.raises(SmlError, match="not a NetCDF"):
        read_region_netcdf(str(p))
    with pytest.raises(SmlError, match="cannot open"):
        read_region_netcdf(str(tmp_path / "nope.nc"))
    w = region_weights(3, False, n_override=420)
    q = tmp_path / "trunc.nc"
    write_region_netcdf(str(q), w.win, w.wout, w.rows, w.cols, w.vals, w.mean, w.std)
    q.write_bytes(q.read_bytes()[:-100])
    with pytest.raises(SmlError, match="out of file bounds"):
        read_region_netcdf(str(q))

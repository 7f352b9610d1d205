"""The Fortran host binding (speedy-ml-1_amd/fortran/sml_hip.f90) drives the GPU
path like the reference's parallelmain: trained weight files are read with
read_trained_res semantics, loaded, and every region predicted; spectral fields go
through grid/spec.  Results are checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from speedy_ml_amd import _lib
from speedy_ml_amd.reservoir import write_region_netcdf
from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights

pytestmark = pytest.mark.gpu

BIN = os.path.join(_lib.PKG_ROOT, "lib", "fortran", "sml_fortran_check")


def test_fortran_host_predict_and_transforms(tmp_path, cuda):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(_lib.PKG_ROOT, "fortran")], check=True)
    cases = [(5, True), (30, False), (0, True), (1151, False)]
    ws = [region_weights(r, s, n_override=900, seed=3) for r, s in cases]
    for w in ws:
        write_region_netcdf(str(tmp_path / f"worker_{w.region:04d}.nc"), w.win, w.wout, w.rows, w.cols, w.vals,
                            w.mean, w.std)
    fb = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    lm = np.stack([local_model_vector(w.region) for w in ws])  # (nlocal, 132) == Fortran (132, nlocal)
    x0 = np.concatenate([initial_state(w.region, w.n) for w in ws])
    rng = np.random.default_rng(9)
    nf = 3
    spec = rng.standard_normal((nf, 32, 62))
    grid = rng.standard_normal((nf, 48, 96))
    with open(tmp_path / "inputs.bin", "wb") as f:
        f.write(np.array([len(ws), nf], dtype=np.int32).tobytes())
        f.write(np.array([w.region for w in ws], dtype=np.int32).tobytes())
        f.write(np.array([int(w.sst) for w in ws], dtype=np.int8).tobytes())
        f.write(np.array([w.n for w in ws], dtype=np.int32).tobytes())
        f.write(np.array([w.k for w in ws], dtype=np.int32).tobytes())
        for a in (fb, lm, x0, spec, grid):
            f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    out = subprocess.run([BIN, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "sml_fortran_check ok" in out.stdout
    raw = np.fromfile(tmp_path / "outputs.bin", dtype=np.float64)
    ntot = sum(w.n for w in ws)
    ov = raw[:136 * len(ws)].reshape(len(ws), 136)
    x1 = raw[136 * len(ws):136 * len(ws) + ntot]
    rest = raw[136 * len(ws) + ntot:]
    g_out = rest[:nf * 4608].reshape(nf, 48, 96)
    s_out = rest[nf * 4608:].reshape(nf, 32, 62)
    off = 0
    fo = 0
    for i, w in enumerate(ws):
        col, val = w.win_compressed()
        ref, xr = oracle.predict_f32(w.rows, w.cols, w.vals, col, val, w.wout, fb[fo:fo + w.ninp], lm[i],
                                     x0[off:off + w.n], w.mean, w.std)
        assert (np.abs(ov[i] - ref) / (1 + np.abs(ref))).max() < 1e-11
        assert (np.abs(x1[off:off + w.n] - xr) / (1 + np.abs(xr))).max() < 1e-14
        off += w.n
        fo += w.ninp
    for f in range(nf):
        rg = oracle.grid(spec[f], 1)
        assert np.abs(g_out[f] - rg).max() <= 1e-12 * np.abs(rg).max()
        rs = oracle.spec(grid[f])
        assert np.abs(s_out[f] - rs).max() <= 1e-12 * np.abs(rs).max()

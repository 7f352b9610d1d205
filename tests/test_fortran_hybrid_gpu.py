"""The Fortran host on the GPU path (speedy-ml-1_amd/fortran):

* sml_hybrid_main -- parallelmain's loop (src/parallelmain.f90:30-283): reads every
  region's trained-weight file (read_trained_res layout, sst flag from std(36) > 0.2
  as trained_reservoir_prediction sets it), loads the SPEEDY state, and runs the
  hybrid steps through sml_hybrid_*.  Its outvecs, inputs, grids, forecasts and
  reservoir states must equal the Python HybridLoop's bit for bit on the same inputs
  (both drive the same native loop; this pins the Fortran host's data handling).
* sml_dropin_check -- the reference's implicit-interface spectral calls
  (`call grid(vorm, vorg, kcos)` ...) linked against libspeedyml_dropin.so, compared
  with the reference's own outputs (tests/golden/spectral_ref.npz) at 1e-12 of the
  field maximum (the GPU Legendre sums in MFMA order; the Fourier stage is bitwise).
* sml_interface_check -- the speedy_res_interface module (reference names and
  signatures): startspeedy's domain extents against the decomposition, the
  truncate_letkf_code_version filter, and test_hybrid_speedy_component's window
  loop against run_model driven from Python with the same clips."""
import os
import subprocess

import numpy as np
import pytest

from speedy_ml_amd import _lib, domain

pytestmark = pytest.mark.gpu

FDIR = os.path.join(_lib.PKG_ROOT, "lib", "fortran")
TRIAL = "gpu_test_trial"


def _bin(name):
    path = os.path.join(FDIR, name)
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(_lib.PKG_ROOT, "fortran")], check=True)
    return path


def _speedy_bin(path, dyn_cls):
    from speedy_ml_amd.dynamics import PHYS_BC
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    st0, forcing = dyn_state()
    d = dyn_cls()
    bc = phys_boundary(d, forcing["phis"])
    d.close()
    with open(path, "wb") as f:
        for k in ("vor", "div", "t", "ps", "tr"):
            f.write(np.ascontiguousarray(st0[k], dtype=np.complex128).tobytes())
        for k in ("phis", "tcorh", "qcorh"):
            f.write(np.ascontiguousarray(forcing[k], dtype=np.complex128).tobytes())
        f.write(np.stack([np.asarray(bc[k], dtype=np.float64).ravel() for k in PHYS_BC]).tobytes())


def test_fortran_hybrid_driver_matches_hybrid_loop(tmp_path, cuda):
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.reservoir import write_region_netcdf
    from speedy_ml_amd.synthetic import initial_state, synthetic_grids
    from test_hybrid_gpu import _loop, _snapshot

    nsteps = 3
    loop, ws = _loop(cuda, True, 64)
    for _ in range(nsteps):
        loop.step()
    loop.sync()
    want = _snapshot(loop)
    want_x = [loop.res.get_state(i) for i in range(1152)]
    loop.close()
    loop.dyn.close()
    loop.res.close()
    torch.cuda.synchronize()
    # the same inputs as files, in the reference's layouts
    wdir = tmp_path / "weights"
    wdir.mkdir()
    for w in ws:
        write_region_netcdf(str(wdir / f"worker_{w.region:04d}_level_1_{TRIAL}.nc"), w.win, w.wout, w.rows, w.cols,
                            w.vals, w.mean, w.std)
    (tmp_path / "setup.txt").write_text(f"1152 {nsteps} 24 1 64\n{TRIAL}\n")
    _speedy_bin(tmp_path / "speedy.bin", Dynamics)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    tisr = np.random.default_rng(13).standard_normal((1152, 16))
    with open(tmp_path / "start.bin", "wb") as f:
        for a in (g4, g2, pr, f4, f2, tisr):
            f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        f.write(np.array([w.n for w in ws], dtype=np.int32).tobytes())
        for w in ws:
            f.write(initial_state(w.region, w.n).tobytes())
    out = subprocess.run([_bin("sml_hybrid_main"), str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "sml_hybrid_main ok" in out.stdout
    raw = np.fromfile(tmp_path / "out_rank0.bin", dtype=np.float64)
    o = 0

    def take(n):
        nonlocal o
        a = raw[o:o + n]
        o += n
        return a

    runs = take(nsteps)
    assert (runs == 1.0).all(), runs
    for k in ("ov", "fb", "lm", "g4", "g2", "pr", "f4", "f2"):
        np.testing.assert_array_equal(take(want[k].size), want[k].ravel(), err_msg=k)
    for i, w in enumerate(ws):
        np.testing.assert_array_equal(take(w.n), want_x[i], err_msg=f"state of region {i}")
    assert o == raw.size


@pytest.mark.parametrize("dated", [False, True])
def test_fortran_hybrid_driver_with_slab_matches_hybrid_loop(tmp_path, cuda, dated):
    """sml_hybrid_main with the slab ocean (slab.bin + worker_XXXX_ocean_<trial>.nc,
    read_trained_ocean_res's layout): a slab step every 2nd hybrid step over 4 steps,
    bitwise the Python HybridLoop with the same SlabOcean; `dated`: with forcing.bin,
    the window's forcing follows run_model's calendar (from 1982-01-31 12 h, across a
    month boundary)."""
    import torch

    from speedy_ml_amd import domain
    from speedy_ml_amd._lib import check, lib, ptr
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs, write_region_netcdf
    from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights, slab_fields,
                                         slab_start_outvec, slab_weights, synthetic_grids)

    nsteps, ts, tss = 4, 6, 12
    mask = domain.load_sst_mask()
    ws = [region_weights(r, bool(mask[r]), n_override=96, seed=5, climatology=True) for r in range(1152)]
    sreg = [r for r in range(1152) if mask[r]]
    sws = [slab_weights(r, n_override=200) for r in sreg]
    base, smask, sice, tice = slab_fields()
    sov_all = np.full((1152, 4), 272.0)
    for r in sreg:
        sov_all[r] = slab_start_outvec(r)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    # the Python loop
    res = Reservoirs(list(range(1152)), mask, [w.n for w in ws], [w.k for w in ws])
    for i, w in enumerate(ws):
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(w.region, w.n))
    slab = Reservoirs(sreg, [0] * len(sreg), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0, nout=4,
                      ninp=[w.ninp for w in sws], out_index=[35] * 4)
    for j, w in enumerate(sws):
        slab.load_region_weights(j, w)
        slab.set_state(j, initial_state(sreg[j], w.n, seed=17))
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.ascontiguousarray(tice))))
    cal = (1982, 24 * 30 + 12)
    if dated:
        from speedy_ml_amd.dynamics import CLIMATOLOGY, SURFACE
        from speedy_ml_amd.synthetic import surface_climatology
        surf, clim = surface_climatology(phys_boundary(dyn, forcing["phis"])["fmask1"])
        dyn.set_surface(surf)
        dyn.set_climatology(clim)
    tisr = np.random.default_rng(13).standard_normal((1152, 16))
    loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=cuda), cuda, tisr=t(tisr), speedy_cus=64,
                      slab=SlabOcean(slab, t(base), t(smask), timestep=ts, timestep_slab=tss))
    if dated:
        loop.set_calendar(cal[0], cal[1], ts)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.start_slab(t(sov_all[sreg]))
    for _ in range(nsteps):
        loop.step()
    loop.sync()
    want = {k: getattr(loop, k).cpu().numpy().copy() for k in ("ov", "fb", "lm", "g4", "g2", "pr", "f4", "f2")}
    want["sst"] = loop.slab_state()["sst"]
    want_x = [res.get_state(i) for i in range(1152)]
    want_sx = [slab.get_state(j) for j in range(len(sreg))]
    loop.close()
    dyn.close()
    res.close()
    slab.close()
    torch.cuda.synchronize()
    # the same inputs as files
    wdir = tmp_path / "weights"
    wdir.mkdir()
    for w in ws:
        write_region_netcdf(str(wdir / f"worker_{w.region:04d}_level_1_{TRIAL}.nc"), w.win, w.wout, w.rows, w.cols,
                            w.vals, w.mean, w.std)
    for w in sws:
        write_region_netcdf(str(wdir / f"worker_{w.region:04d}_ocean_{TRIAL}.nc"), w.win, w.wout, w.rows, w.cols,
                            w.vals, w.mean, w.std)
    (tmp_path / "setup.txt").write_text(f"1152 {nsteps} 24 1 64\n{TRIAL}\n")
    _speedy_bin(tmp_path / "speedy.bin", Dynamics)
    with open(tmp_path / "start.bin", "wb") as f:
        for a in (g4, g2, pr, f4, f2, tisr):
            f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        f.write(np.array([w.n for w in ws], dtype=np.int32).tobytes())
        for w in ws:
            f.write(initial_state(w.region, w.n).tobytes())
    nall = np.zeros(1152, dtype=np.int32)
    for w in sws:
        nall[w.region] = w.n
    if dated:
        with open(tmp_path / "forcing.bin", "wb") as f:
            f.write(np.stack([surf[k] for k in SURFACE]).astype(np.float64).tobytes())
            f.write(np.stack([clim[k] for k in CLIMATOLOGY]).astype(np.float64).tobytes())
            f.write(np.array([cal[0]], dtype=np.int32).tobytes())
            f.write(np.array([cal[1]], dtype=np.int64).tobytes())
    with open(tmp_path / "slab.bin", "wb") as f:
        f.write(np.array([ts, tss], dtype=np.int32).tobytes())
        for a in (base, smask, sice, tice, sov_all):
            f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        f.write(nall.tobytes())
        for w in sws:
            f.write(initial_state(w.region, w.n, seed=17).tobytes())
    out = subprocess.run([_bin("sml_hybrid_main"), str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    raw = np.fromfile(tmp_path / "out_rank0.bin", dtype=np.float64)
    o = 0

    def take(n):
        nonlocal o
        a = raw[o:o + n]
        o += n
        return a

    assert (take(nsteps) == 1.0).all()
    for k in ("ov", "fb", "lm", "g4", "g2", "pr", "f4", "f2"):
        np.testing.assert_array_equal(take(want[k].size), want[k].ravel(), err_msg=k)
    for i, w in enumerate(ws):
        np.testing.assert_array_equal(take(w.n), want_x[i], err_msg=f"state of region {i}")
    np.testing.assert_array_equal(take(want["sst"].size), want["sst"].ravel(), err_msg="wholegrid_sst")
    for j, w in enumerate(sws):
        np.testing.assert_array_equal(take(w.n), want_sx[j], err_msg=f"slab state {j}")
    assert o == raw.size


def test_fortran_dropin_matches_reference_golden(tmp_path, cuda):
    from conftest import REPO

    g = np.load(os.path.join(REPO, "tests", "golden", "spectral_ref.npz"))
    nf = g["spec_in"].shape[0]
    with open(tmp_path / "dropin_in.bin", "wb") as f:
        f.write(np.array([nf], dtype=np.int32).tobytes())
        for k in ("spec_in", "grid_in", "grid_in2"):
            f.write(np.ascontiguousarray(g[k], dtype=np.float64).tobytes())
    out = subprocess.run([_bin("sml_dropin_check"), str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    raw = np.fromfile(tmp_path / "dropin_out.bin", dtype=np.float64)
    names = [("grid_k1", (48, 96)), ("grid_k2", (48, 96)), ("spec", (32, 62)), ("gridy", (48, 62)),
             ("specy_of_gridy", (32, 62)), ("specx", (48, 62)), ("vdspec_k1_vor", (32, 62)),
             ("vdspec_k1_div", (32, 62)), ("vdspec_k2_vor", (32, 62)), ("vdspec_k2_div", (32, 62)),
             ("uvspec_u", (32, 62)), ("uvspec_v", (32, 62))]
    o = 0
    for name, shp in names:
        n = nf * shp[0] * shp[1]
        got = raw[o:o + n].reshape((nf,) + shp)
        o += n
        ref = g[name]
        for f in range(nf):
            scale = max(np.abs(ref[f]).max(), 1e-300)
            assert np.abs(got[f] - ref[f]).max() <= 1e-12 * scale, (name, f, np.abs(got[f] - ref[f]).max() / scale)
        if name == "specx":  # the Fourier stage follows FFTPACK's operation order: bitwise
            np.testing.assert_array_equal(got, ref)
    assert o == raw.size


def test_speedy_res_interface_module(tmp_path, cuda):
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids

    _speedy_bin(tmp_path / "speedy.bin", Dynamics)
    g4, g2, _ = synthetic_grids(21)
    g4[7, :, :, 3] = 40.0   # above test_hybrid_speedy_component's 25 g/kg clip
    nwin, trunc = 2, 20
    rng = np.random.default_rng(3)
    field = rng.standard_normal((32, 31)) + 1j * rng.standard_normal((32, 31))  # Fortran (31, 32)
    regions = np.array([0, 23, 24, 600, 1127, 1151], dtype=np.int32)
    with open(tmp_path / "iface_in.bin", "wb") as f:
        f.write(g4.tobytes())
        f.write(g2.tobytes())
        f.write(np.array([nwin, trunc], dtype=np.int32).tobytes())
        f.write(field.astype(np.complex128).tobytes())
        f.write(np.array([len(regions)], dtype=np.int32).tobytes())
        f.write(regions.tobytes())
    out = subprocess.run([_bin("sml_interface_check"), str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    # the calendar and the state's date fields advanced per window as the reference
    # (speedy_res_interface.f90:778, 797-800): hour 86184 + nwin from 1981
    import ctypes

    from speedy_ml_amd._lib import lib

    date, feb = (ctypes.c_int * 4)(), ctypes.c_int(0)
    for i in range(1, nwin + 1):
        assert lib().sml_calendar_delta_hour(1981, 86184 + i, ctypes.byref(feb), date) == 0
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("calendar")][0].split()
    assert [int(v) for v in line[1:5]] == list(date) == [int(v) for v in line[6:10]], (line, list(date))
    raw = np.fromfile(tmp_path / "iface_out.bin", dtype=np.float64)
    v4 = raw[:g4.size].reshape(g4.shape)
    lp = raw[g4.size:g4.size + g2.size].reshape(g2.shape)
    o = g4.size + g2.size
    safe = raw[o]
    tf = raw[o + 1:o + 1 + 2 * field.size].view(np.complex128).reshape(field.shape)
    ext = raw[o + 1 + 2 * field.size:].reshape(len(regions), 12)
    # the window loop from Python: clips, run_model, clip
    st0, forcing = dyn_state()
    d = Dynamics()
    d.set_forcing(**forcing)
    d.set_state(st0)
    d.set_physics(phys_boundary(d, forcing["phis"]))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    a4, a2 = g4.copy(), g2.copy()
    for _ in range(nwin):
        q = a4[..., 3]
        q[q < 0.0] = 0.0
        q[q > 25.0] = 25.0
        o4, o2 = torch.zeros_like(t(a4)), torch.zeros_like(t(a2))
        d.run_model(t(a4), t(a2), o4, o2)
        ok, _ = d.last_safe()
        a4, a2 = o4.cpu().numpy(), o2.cpu().numpy()
        a4[..., 3][a4[..., 3] < 0.0] = 0.0
        assert ok
    d.close()
    assert safe == 1.0
    np.testing.assert_array_equal(v4, a4)
    np.testing.assert_array_equal(lp, a2)
    # truncate_letkf_code_version: zero where (m-1) + (n-1) > trunc
    m = np.arange(31)[None, :]
    n = np.arange(32)[:, None]
    np.testing.assert_array_equal(tf, np.where(m + n > trunc, 0.0, field))
    # startspeedy -> initializedomain extents
    for i, r in enumerate(regions):
        geo = domain.region_geometry(int(r))
        want = [geo.res_xstart, geo.res_xend, geo.res_ystart, geo.res_yend, geo.resx, geo.resy, geo.in_xstart,
                geo.in_xend, geo.in_ystart, geo.in_yend, geo.inx, geo.iny]
        assert list(ext[i].astype(int)) == want, (r, list(ext[i]), want)

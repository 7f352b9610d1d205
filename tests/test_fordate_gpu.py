"""The window's date-driven forcing on the GPU (sml_dyn_fordate: the coupler at the
date, ini_sea's hybrid SST, fordate; src/ini_agcm_init.f90:57-89) against the
reference's own fordate (tests/golden/fordate_ref.npz) and the oracle.

Tolerances: tcorh / qcorh within 1e-12 of the field scale (spec on the matrix cores,
as the spectral tests); the boundary fields' grid values bit-exact where they are
interpolations and products (the coupler, albedo; the same operations in the same
order, no contraction), the insolation rows within 1e-15."""
import os
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_fordate_golden import ALB, DATES, SEL, SOL, inputs  # noqa: E402

SPEC_TOL = 1e-12


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300))


def _dyn(phis_c, fmask, surf):
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    st0, forcing = dyn_state()
    phis = np.ascontiguousarray(np.asarray(phis_c).T)  # (nx, mx) C order = complex(mx, nx)
    dyn = Dynamics()
    dyn.set_forcing(phis=phis, tcorh=forcing["tcorh"], qcorh=forcing["qcorh"])
    dyn.set_state(st0)
    bc = phys_boundary(dyn, phis)
    bc["fmask1"] = surf["fmask_l"]
    return dyn, bc


def test_fordate_matches_the_reference(cuda):
    """Every (date, sst) case of the golden: the coupler's land fields and snow cover
    as the reference computed them (the oracle's coupler, bit-exact with it at the
    golden's points), sst_am and sice_am as given, then sml_dyn_fordate."""
    g = np.load(os.path.join(HERE, "golden", "fordate_ref.npz"))
    fmask, phis_c, surf, clim, anom, sice = inputs()
    dyn, bc = _dyn(phis_c, fmask, surf)
    np.testing.assert_allclose(bc["phis0"], g["phis0"], rtol=0, atol=1e-9)
    bc["phis0"] = g["phis0"]
    dyn.set_surface(surf)
    from speedy_ml_amd._lib import check, lib, ptr
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.zeros(4608))))
    worst = {}
    for di, (y, mo, dd) in enumerate(DATES):
        c = oracle.coupler(mo, dd, clim)
        np.testing.assert_array_equal(c["stl_am"][SEL], g[f"d{di}_stl_am"])
        base = np.maximum(clim["sst12"][mo - 1], 271.5)
        for si, sst in enumerate((base, base + anom)):
            b = dict(bc, stl_am=c["stl_am"], soilw_am=c["soilw_am"], sst_am=sst,
                     snowc=np.minimum(1.0, c["snowd_am"] / 60.0))
            dyn.set_physics(b)
            dyn.fordate(y, mo, dd)
            out = dyn.get_physics()
            f = dyn.get_forcing()
            case = f"d{di}s{si}"
            for k in ("tcorh", "qcorh"):
                worst[k] = max(worst.get(k, 0.0), _rel(f[k], g[f"{case}_{k}"]))
            for k in SOL:
                worst[k] = max(worst.get(k, 0.0), _rel(out[k].reshape(48, 96)[:, 0], g[f"{case}_{k}"]))
            for k in ALB:
                np.testing.assert_array_equal(out[k][SEL], g[f"{case}_{k}"], err_msg=f"{case} {k}")
            np.testing.assert_array_equal(out["sst_am"], sst)
    print("fordate vs reference:", {k: f"{v:.1e}" for k, v in worst.items()})
    assert worst["tcorh"] <= SPEC_TOL and worst["qcorh"] <= SPEC_TOL
    assert max(worst[k] for k in SOL) <= 1e-15
    dyn.close()


def test_coupler_hybrid_sst_and_fordate_match_the_oracle(cuda):
    """With the monthly climatologies on the device: the coupler at the date, the
    hybrid SST (ini_sea's block, with a bias) and fordate, against
    oracle.window_forcing, on every grid point."""
    import torch

    fmask, phis_c, surf, clim, anom, _ = inputs()
    dyn, bc = _dyn(phis_c, fmask, surf)
    dyn.set_physics(bc)
    bc = dyn.get_physics()
    dyn.set_surface(surf)
    dyn.set_climatology(clim)
    hyb = np.maximum(clim["sst12"][6], 272.0) + anom
    d_hyb = torch.from_numpy(hyb.reshape(48, 96)).to(cuda)
    from speedy_ml_amd._lib import check, lib, ptr
    for y, mo, dd in DATES + ((1983, 2, 28),):
        for with_hyb in (False, True):
            if with_hyb:
                check(lib().sml_dyn_set_hybrid_sst(dyn._h, ptr(d_hyb), 0.25, None))
            dyn.fordate(y, mo, dd)
            out, f = dyn.get_physics(), dyn.get_forcing()
            sice, tice = dyn.get_sea_ice()
            want, tq, qq, wsice, wtice = oracle.window_forcing(mo, dd, surf, bc, clim=clim,
                                                               sst_hybrid=hyb if with_hyb else None, bias=0.25)
            np.testing.assert_array_equal(sice, wsice)
            np.testing.assert_array_equal(tice, wtice)
            for k in ("stl_am", "soilw_am", "sst_am", "snowc", "alb_l", "alb_s", "albsfc", "fmask1", "phis0",
                      "forog"):
                np.testing.assert_array_equal(out[k], want[k], err_msg=f"{(y, mo, dd, with_hyb)} {k}")
            for k in SOL:
                assert _rel(out[k], want[k]) <= 1e-15, k
            assert _rel(f["tcorh"], tq) <= SPEC_TOL and _rel(f["qcorh"], qq) <= SPEC_TOL
        check(lib().sml_dyn_set_hybrid_sst(dyn._h, None, 0.0, None))
    dyn.close()


def test_fordate_is_recomputed_only_when_an_input_changes(cuda):
    import torch

    fmask, phis_c, surf, clim, anom, _ = inputs()
    dyn, bc = _dyn(phis_c, fmask, surf)
    dyn.set_physics(bc)
    dyn.set_surface(surf)
    dyn.set_climatology(clim)
    dyn.fordate(1982, 3, 1)
    n = dyn.fordate_count()
    dyn.fordate(1983, 3, 1)  # the year alone does not change the forcing (lco2 off)
    assert dyn.fordate_count() == n
    dyn.fordate(1982, 3, 2)
    assert dyn.fordate_count() == n + 1
    d_hyb = torch.full((48, 96), 290.0, dtype=torch.float64, device=cuda)
    from speedy_ml_amd._lib import check, lib, ptr
    check(lib().sml_dyn_set_hybrid_sst(dyn._h, ptr(d_hyb), 0.0, None))
    q0 = dyn.get_forcing()["qcorh"]
    dyn.fordate(1982, 3, 2)
    assert dyn.fordate_count() == n + 2
    assert not np.array_equal(dyn.get_forcing()["qcorh"], q0)
    dyn.fordate(1982, 3, 2, force=True)
    assert dyn.fordate_count() == n + 3
    dyn.close()


def test_fordate_rejects_days_past_the_month(cuda):
    """a day past its month (2-30, 4-31) is refused instead of extrapolating
    newdate's tmonth; February 29 -- which the reference calendar emits once its
    February latch is set (mod_calendar.f90:40, 61-63) -- is accepted."""
    from speedy_ml_amd._lib import SmlError

    fmask, phis_c, surf, clim, _, _ = inputs()
    dyn, bc = _dyn(phis_c, fmask, surf)
    dyn.set_physics(bc)
    dyn.set_surface(surf)
    dyn.set_climatology(clim)
    for mo, dd in ((2, 30), (4, 31), (6, 31), (9, 31), (11, 31), (1, 0), (13, 1)):
        with pytest.raises(SmlError):
            dyn.fordate(1982, mo, dd)
    for mo, dd in ((2, 29), (1, 31), (12, 31)):
        dyn.fordate(1984, mo, dd)
    dyn.close()

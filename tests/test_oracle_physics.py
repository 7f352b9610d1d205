"""Oracle SPEEDY physics (phypar's column physics) against the reference's own
phypar (tests/golden/phys_ref.npz, tests/golden/make_phys_golden.py).

The fixture stores every 4th longitude (physics is column-local); the other
columns are filled with their row neighbour's inputs so that every column the
oracle evaluates is valid.  Tolerance: the reference evaluates the same formulas
in the same order with the same libm, so differences are a few ulp:
max |err| <= 1e-12 x max |tendency| per variable (TOL)."""
import numpy as np
import pytest

import oracle

TOL = 1e-12


@pytest.fixture(scope="module")
def pg():
    import os

    from conftest import REPO

    return dict(np.load(os.path.join(REPO, "tests", "golden", "phys_ref.npz")))


def _fill(a, sel):
    """(…, ngp) array known at `sel` (every 4th longitude) -> full grid."""
    full = np.zeros(a.shape[:-1] + (oracle.NGP,))
    full[..., sel] = a
    idx = np.arange(oracle.NGP)
    src = idx - (idx % oracle.IX) % 4
    return full[..., src]


def _bc(pg):
    bc = {k: pg[f"bc_{k}"] for k in ("fmask1", "phis0", "stl_am", "sst_am", "soilw_am", "alb_l", "alb_s",
                                      "albsfc", "snowc")}
    for k in ("fsol", "ozone", "ozupp", "zenit", "stratz"):
        bc[k] = np.repeat(pg[f"sol_{k}"], oracle.IX)
    bc["forog"] = pg["forog"]
    return bc


def _run(pg, case, state, lradsw):
    sel = pg["sel"]
    ins = [_fill(pg[f"{case}_{k}"], sel) for k in ("ug1", "vg1", "tg1", "qg1", "phig1", "pslg1")]
    return oracle.phypar_grid(*ins, _bc(pg), state, lradsw)


def test_tables_and_forcing(pg):
    np.testing.assert_allclose(oracle.radang(), pg["radang"], rtol=0, atol=1e-15)
    sol = oracle.sol_oz(float(pg["tyear"]))
    for k in ("fsol", "ozone", "ozupp", "zenit", "stratz"):
        np.testing.assert_allclose(sol[k].reshape(48, 96)[:, 0], pg[f"sol_{k}"], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(oracle.sflset(pg["bc_phis0"]), pg["forog"], rtol=1e-15, atol=0)


def test_physics_with_radiation(pg):
    st = oracle.phys_state()
    tend = _run(pg, "rad", st, True)
    sel = pg["sel"]
    ref = pg["rad_tend"]
    for v in range(4):
        err = np.abs(tend[v][:, sel] - ref[v]).max()
        assert err <= TOL * np.abs(ref[v]).max(), (v, err)
    np.testing.assert_allclose(st["tau2"][..., sel], pg["rad_tau2"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(st["stratc"][:, sel], pg["rad_stratc"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(st["ssrd"][sel], pg["rad_ssrd"], rtol=1e-13, atol=1e-12)
    err = np.abs(st["tt_rsw"][:, sel] - pg["rad_tt_rsw"]).max()
    assert err <= TOL * np.abs(pg["rad_tt_rsw"]).max()


def test_physics_without_radiation_keeps_state(pg):
    st = oracle.phys_state()
    _run(pg, "rad", st, True)
    tend = _run(pg, "norad", st, False)
    sel = pg["sel"]
    ref = pg["norad_tend"]
    for v in range(4):
        err = np.abs(tend[v][:, sel] - ref[v]).max()
        assert err <= TOL * np.abs(ref[v]).max(), (v, err)

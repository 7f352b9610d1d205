"""GPU parity of SPEEDY's dynamics `step` (sml_dyn_*) against the reference's
step (tests/golden/dyn_ref.npz) and the oracle restatement.

Tolerance: the GPU transforms sum in a different order than FFTPACK / the
reference's Legendre loops and the physics tendencies are added as one sum, so
one step agrees to fp64 rounding: max |err| <= 1e-12 x max |field| (TOL).  A
multi-step chain is compared with CHAIN_TOL (rounding differences grow through
the gravity-wave dynamics of the unbalanced synthetic state)."""
import ctypes

import numpy as np
import pytest

import oracle
from conftest import DYN_CASES

pytestmark = pytest.mark.gpu

TOL = 1e-12
CHAIN_TOL = 1e-10


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def dyn(cuda):
    from speedy_ml_amd.dynamics import Dynamics

    return Dynamics()


def _load(dyn, g):
    dyn.set_forcing(g["phis"], g["tcorh"], g["qcorh"])
    dyn.set_state({f: g[f] for f in oracle.DYN_FIELDS})


@pytest.mark.parametrize("case", DYN_CASES)
def test_step_matches_reference(dyn, dyn_golden, case):
    g = dyn_golden
    j1, j2, dt, alph = g[f"{case}_case"]
    j1, j2 = int(j1), int(j2)
    _load(dyn, g)
    dyn.step(j1, j2, float(dt), float(alph), float(g["rob"]), float(g["wil"]), phys=g["phys"])
    st = dyn.get_state()
    lv = [0, 1] if j1 == 2 else [1]
    for f in oracle.DYN_FIELDS:
        assert _rel(st[f][lv], g[f"{case}_{f}"]) < TOL, (case, f, _rel(st[f][lv], g[f"{case}_{f}"]))
        if j1 == 1:
            np.testing.assert_array_equal(st[f][0], g[f][0])
    if case == "lf":
        assert _rel(dyn.get_phi(), g["lf_phi"]) < 1e-15


def test_tendencies_match_oracle(dyn, dyn_golden):
    """dt <= 0: tendencies only, state untouched (dyn_step.f90:109).  Both sides
    evaluate impint(0, alph) first (dmp1 = 1, no implicit correction)."""
    g = dyn_golden
    _load(dyn, g)
    dyn.step(2, 2, 0.0, 0.5, phys=g["phys"])
    tend = dyn.get_tendencies()
    st = oracle.dyn_state_copy(g)
    _, otend = oracle.dyn_step(st, g["phis"], g["tcorh"], g["qcorh"], g["phys"], 2, 2, 0.0, 0.5)
    for name, sl in (("vordt", slice(0, 8)), ("divdt", slice(8, 16)), ("tdt", slice(16, 24)),
                     ("trdt", slice(24, 32)), ("psdt", slice(32, 33))):
        assert _rel(tend[sl], otend[sl]) < TOL, name
    got = dyn.get_state()
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(got[f], g[f])


def test_device_physics_matches_host(dyn, dyn_golden, cuda):
    import torch

    g = dyn_golden
    _load(dyn, g)
    dyn.step(2, 2, 2 * float(g["delt"]), 0.5, phys=g["phys"])
    a = dyn.get_state()
    _load(dyn, g)
    ph = torch.from_numpy(np.ascontiguousarray(g["phys"])).to(cuda)
    dyn.step(2, 2, 2 * float(g["delt"]), 0.5, phys=ph)
    torch.cuda.synchronize()
    b = dyn.get_state()
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(a[f], b[f])


def test_chain_without_physics_matches_oracle(dyn, dyn_golden):
    """stepone + 6 leapfrog steps (stloop shape), no physics."""
    g = dyn_golden
    delt = float(g["delt"])
    _load(dyn, g)
    st = oracle.dyn_state_copy(g)
    seq = [(1, 1, 0.5 * delt), (1, 2, delt)] + [(2, 2, 2 * delt)] * 6
    for j1, j2, dt in seq:
        dyn.step(j1, j2, dt, 0.5)
        oracle.dyn_step(st, g["phis"], g["tcorh"], g["qcorh"], None, j1, j2, dt, 0.5)
    got = dyn.get_state()
    for f in oracle.DYN_FIELDS:
        assert _rel(got[f], st[f]) < CHAIN_TOL, (f, _rel(got[f], st[f]))


def test_step_requires_impint(cuda):
    from speedy_ml_amd._lib import lib

    h = ctypes.c_void_p()
    assert lib().sml_dyn_create(6.371e6, ctypes.byref(h)) == 0
    try:
        assert lib().sml_dyn_step(h, 2, 2, 1800.0, 0.5, 0.05, 0.53, None, None) == -4  # SML_ERR_STATE
        assert lib().sml_dyn_step(h, 3, 2, 1800.0, 0.5, 0.05, 0.53, None, None) == -1  # bad j1
    finally:
        lib().sml_dyn_destroy(h)


def test_leapfrog_graph_matches_step_loop(dyn, dyn_golden):
    """sml_dyn_leapfrog (hipGraph replay) == the same steps launched one by one."""
    import torch

    g = dyn_golden
    delt = float(g["delt"])
    _load(dyn, g)
    dyn.leapfrog(5, delt, graph=False)
    a = dyn.get_state()
    _load(dyn, g)
    dyn.leapfrog(5, delt, graph=True)
    torch.cuda.synchronize()
    b = dyn.get_state()
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(a[f], b[f])


def test_iogrid_exit_matches_oracle(dyn):
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(7)
    dyn.set_state(st)
    g4, lp = dyn.to_grid()
    og4, olp = oracle.iogrid31(oracle.dyn_state_copy(st))
    for c in range(4):
        assert _rel(g4[..., c], og4[..., c]) < TOL, c
    assert _rel(lp, olp) < TOL


def test_iogrid_entry_matches_oracle(dyn):
    from speedy_ml_amd.synthetic import dyn_state

    st, _ = dyn_state(7)
    og4, olp = oracle.iogrid31(oracle.dyn_state_copy(st))
    og4 = og4.copy()
    og4[..., 3] -= 0.3  # exercise the q clip
    st2, _ = dyn_state(8)  # different level-1/level-2 contents before entry
    dyn.set_state(st2)
    mm, safe = dyn.from_grid(og4, olp)
    got = dyn.get_state()
    ref = oracle.dyn_state_copy(st2)
    omm, osafe = oracle.iogrid30(ref, og4, olp)
    assert safe == osafe
    np.testing.assert_allclose(mm, omm, rtol=1e-12, atol=1e-12)
    for f in oracle.DYN_FIELDS:
        assert _rel(got[f][0], ref[f][0]) < TOL, f
        np.testing.assert_array_equal(got[f][1], st2[f][1])  # level 2 untouched


def test_iogrid_device_entry_flags_unsafe(dyn, cuda):
    import torch
    from speedy_ml_amd._lib import lib

    from speedy_ml_amd.synthetic import dyn_state

    st, _ = dyn_state(7)
    og4, olp = oracle.iogrid31(oracle.dyn_state_copy(st))
    og4 = og4.copy()
    og4[3, 20:30, 40:60, 1] = 400.0
    g = torch.from_numpy(og4).to(cuda)
    lp = torch.from_numpy(olp).to(cuda)
    mm = torch.zeros(8, dtype=torch.float64, device=cuda)
    assert lib().sml_dyn_from_grid(dyn._h, g.data_ptr(), lp.data_ptr(), mm.data_ptr(), None) == 0
    torch.cuda.synchronize()
    mmh = mm.cpu().numpy()
    assert lib().sml_dyn_is_safe(mmh.ctypes.data) == 0
    assert mmh[1] > 150.0

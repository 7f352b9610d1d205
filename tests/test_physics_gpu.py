"""GPU phypar (sml_physics.hpp via sml_dyn_phypar / the step's internal physics)
against the reference's own phypar and step (tests/golden/phys_ref.npz,
tests/golden/dyn_ref.npz) and against the oracle on full grids.

Tolerances: the device's exp/log/sqrt differ from glibc by an ulp and the GPU
transforms sum in a different order, so tendencies agree to fp64 rounding:
max |err| <= 1e-12 x max |tendency| (TOL) for one physics call or one step; a
multi-step chain with physics is compared with CHAIN_TOL (rounding differences
grow through the unbalanced synthetic state's gravity waves)."""
import numpy as np
import pytest

import oracle
from conftest import DYN_CASES
from test_oracle_physics import _bc, _fill
from test_oracle_physics_step import dyn_bc

pytestmark = pytest.mark.gpu

TOL = 1e-12
CHAIN_TOL = 1e-9
FUSED_TOL = 1e-11


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def pg():
    import os

    from conftest import REPO

    return dict(np.load(os.path.join(REPO, "tests", "golden", "phys_ref.npz")))


@pytest.fixture()
def dyn(cuda):
    from speedy_ml_amd.dynamics import Dynamics

    d = Dynamics()
    yield d
    d.close()


def _ins(pg, case):
    return [_fill(pg[f"{case}_{k}"], pg["sel"]) for k in ("ug1", "vg1", "tg1", "qg1", "phig1", "pslg1")]


def test_phypar_matches_reference(dyn, pg):
    """rad (lradsw) then norad (radiation state kept), as make_phys_golden.py ran them."""
    sel = pg["sel"]
    dyn.set_physics(_bc(pg))
    dyn.set_rad_state(None)
    for case, lradsw in (("rad", True), ("norad", False)):
        tend = dyn.phypar(*_ins(pg, case), lradsw)
        ref = pg[f"{case}_tend"]
        for v in range(4):
            assert _rel(tend[v][:, sel], ref[v]) <= TOL, (case, v, _rel(tend[v][:, sel], ref[v]))
        if case == "rad":
            rad = dyn.get_rad_state()
            np.testing.assert_allclose(rad["tau2"][..., sel], pg["rad_tau2"], rtol=1e-13, atol=0)
            np.testing.assert_allclose(rad["stratc"][:, sel], pg["rad_stratc"], rtol=1e-13, atol=0)
            np.testing.assert_allclose(rad["ssrd"][sel], pg["rad_ssrd"], rtol=1e-13, atol=1e-12)
            assert _rel(rad["tt_rsw"][:, sel], pg["rad_tt_rsw"]) <= TOL


def test_phypar_matches_oracle_on_full_grid(dyn, pg):
    """Every column of a synthetic state (not only the fixture's every 4th)."""
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(31)
    s = oracle.dyn_state_copy(st)
    ins = oracle.phys_inputs(s, forcing["phis"])
    bc = _bc(pg)
    ost = oracle.phys_state()
    dyn.set_physics(bc)
    dyn.set_rad_state(None)
    for lradsw in (True, False):
        ref = oracle.phypar_grid(*ins, bc, ost, lradsw)
        got = dyn.phypar(*ins, lradsw)
        for v in range(4):
            assert _rel(got[v], ref[v]) <= TOL, (lradsw, v, _rel(got[v], ref[v]))
    rad = dyn.get_rad_state()
    for k in ("tau2", "stratc", "ssrd"):
        np.testing.assert_allclose(rad[k], ost[k], rtol=1e-13, atol=1e-12)


def test_forcing_helpers_match_oracle(dyn, pg):
    sol = dyn.sol_oz(float(pg["tyear"]))
    osol = oracle.sol_oz(float(pg["tyear"]))
    for k in ("fsol", "ozone", "ozupp", "zenit", "stratz"):
        np.testing.assert_allclose(sol[k], osol[k], rtol=1e-14, atol=1e-14)
        np.testing.assert_allclose(sol[k].reshape(48, 96)[:, 0], pg[f"sol_{k}"], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(dyn.sflset(pg["bc_phis0"]), pg["forog"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("case", DYN_CASES)
def test_step_with_gpu_physics_matches_reference(dyn, dyn_golden, case):
    """The reference step calls its phypar inside grtend; here the step computes
    phypar on the GPU from the state (no tendencies handed in)."""
    g = dyn_golden
    j1, j2, dt, alph = g[f"{case}_case"]
    j1, j2 = int(j1), int(j2)
    dyn.set_forcing(g["phis"], g["tcorh"], g["qcorh"])
    dyn.set_state({f: g[f] for f in oracle.DYN_FIELDS})
    dyn.set_physics(dyn_bc(g))
    dyn.set_rad_state(None)
    dyn.set_clock(1, False)  # make_dyn_golden.py: lradsw = .false.
    dyn.step(j1, j2, float(dt), float(alph), float(g["rob"]), float(g["wil"]))
    st = dyn.get_state()
    lv = [0, 1] if j1 == 2 else [1]
    for f in oracle.DYN_FIELDS:
        assert _rel(st[f][lv], g[f"{case}_{f}"]) < TOL, (case, f, _rel(st[f][lv], g[f"{case}_{f}"]))


def _window_bc(pg, dyn):
    bc = _bc(pg)
    bc.update(dyn.sol_oz(0.1))
    return bc


def test_window_chain_with_physics_matches_oracle(dyn, pg):
    """stepone + 6 leapfrog steps with stloop's lradsw pattern (istep 1, 4 radiate)."""
    from speedy_ml_amd.dynamics import DELT, Dynamics  # noqa: F401
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(5)
    bc = _window_bc(pg, dyn)
    dyn.set_forcing(**forcing)
    dyn.set_state(st)
    dyn.set_physics(bc)
    dyn.set_rad_state(None)
    dyn.set_clock(1, True)
    dyn.stepone()
    _, lr = dyn.get_clock()
    dyn.set_clock(1, lr)
    dyn.leapfrog(6, graph=False)
    got = dyn.get_state()
    s = oracle.dyn_state_copy(st)
    rad = oracle.phys_state()
    seq = [(1, 1, 0.5 * DELT, True), (1, 2, DELT, True)] + [(2, 2, 2 * DELT, i % 3 == 1) for i in range(1, 7)]
    for j1, j2, dt, lradsw in seq:
        oracle.dyn_step_physics(s, forcing["phis"], forcing["tcorh"], forcing["qcorh"], bc, rad, lradsw, j1, j2, dt,
                                0.5)
    for f in oracle.DYN_FIELDS:
        assert _rel(got[f], s[f]) < CHAIN_TOL, (f, _rel(got[f], s[f]))
    assert dyn.get_clock() == (7, False)


def test_leapfrog_graph_with_physics_matches_step_loop(dyn, pg, cuda):
    """hipGraph replay (one graph per lradsw value) == steps launched one by one,
    state, radiation state and clock."""
    import torch

    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(6)
    bc = _window_bc(pg, dyn)
    out = []
    for graph in (False, True):
        dyn.set_forcing(**forcing)
        dyn.set_state(st)
        dyn.set_physics(bc)
        dyn.set_rad_state(None)
        dyn.set_clock(1, True)
        dyn.stepone()
        dyn.set_clock(1, True)
        dyn.leapfrog(7, graph=graph)
        torch.cuda.synchronize()
        out.append((dyn.get_state(), dyn.get_rad_state(), dyn.get_clock()))
    (a, ra, ca), (b, rb, cb) = out
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(a[f], b[f])
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])
    assert ca == cb == (8, True)


def test_host_tendencies_rejected_while_gpu_physics_on(dyn, dyn_golden):
    from speedy_ml_amd._lib import SmlError

    g = dyn_golden
    dyn.set_physics(dyn_bc(g))
    with pytest.raises(SmlError, match="physics runs on the GPU"):
        dyn.step(2, 2, 1800.0, 0.5, phys=g["phys"])
    dyn.set_physics(None)
    dyn.step(2, 2, 1800.0, 0.5, phys=g["phys"])


@pytest.mark.parametrize("physics", [False, True])
def test_fused_step_agrees_with_unfused_step_to_rounding(pg, cuda, physics):
    """The fused step (k_st_inv, k_st_rows, [k_phys_add, specx], k_st_spec; chained
    across the steps of a window) and the 8/9-launch step evaluate the same
    operations in the same order.  The unfused step's Fourier transforms are the
    iogrid / drop-in kernels (sml_spectral.hip: FFTPACK's separate multiplies and
    adds, bit-exact with the reference's FFT) while the fused step's kernels contract
    a*b + c within an expression into one FMA (sml_dynamics.hip, -ffp-contract=on),
    so the two agree to rounding (FUSED_TOL per field and level after a run of steps
    and two windows: state, radiation state, tendencies, geopotential)."""
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(9)
    out = []
    for fused in ("0", "1"):
        d = Dynamics()
        d.set_fused(fused == "1")
        d.set_forcing(**forcing)
        d.set_state(st)
        if physics:
            d.set_physics(_window_bc(pg, d))
            d.set_rad_state(None)
        d.set_clock(1, True)
        d.stepone()
        d.set_clock(1, True)
        d.leapfrog(4, graph=True)
        d.leapfrog(2, graph=False)
        d.step(2, 2, 0.0, 0.5)  # tendencies only
        torch.cuda.synchronize()
        tend, phi = d.get_tendencies(), d.get_phi()
        d.window(24)  # one graph; the fused form chains each step's gridy into the previous step's last kernel
        d.window(24)
        torch.cuda.synchronize()
        out.append((d.get_state(), d.get_rad_state(), tend, phi))
        d.close()
    (a, ra, ta, pa), (b, rb, tb, pb) = out

    def close(x, y):
        x, y = np.asarray(x), np.asarray(y)
        assert np.abs(x - y).max() <= FUSED_TOL * max(np.abs(y).max(), 1e-300), np.abs(x - y).max()

    for f in oracle.DYN_FIELDS:
        for j in range(a[f].shape[0]):
            close(a[f][j], b[f][j])
    for k in ra:
        close(ra[k], rb[k])
    for i in range(len(ta)):
        close(ta[i], tb[i])
    close(pa, pb)


CHAIN_WINDOWS = 24
CHAIN_DRIFT_TOL = 1e-6


def test_fused_window_chain_drift_against_fftpack_exact_chain(pg, cuda):
    """Drift of the fused (FMA-contracted) window against the unfused window, whose
    transforms are FFTPACK-exact (the reference's arithmetic, WINDOW_TOL per window),
    over CHAIN_WINDOWS chained 6-h windows with physics (6 simulated days: the hybrid
    loop chains one window per step).  Rounding differences grow with the flow's
    error growth; the per-window maximum relative difference (per field, over levels)
    is printed and stays below CHAIN_DRIFT_TOL.  The measured growth is recorded in
    DESIGN.md (SPEEDY window numerics)."""
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(9)
    chains = []
    for fused in ("0", "1"):
        d = Dynamics()
        d.set_fused(fused == "1")
        d.set_forcing(**forcing)
        d.set_state(st)
        d.set_physics(_window_bc(pg, d))
        d.set_rad_state(None)
        d.set_clock(1, True)
        states = []
        for _ in range(CHAIN_WINDOWS):
            d.window(24)
            torch.cuda.synchronize()
            states.append(d.get_state())
        chains.append(states)
        d.close()
    drift = []
    for a, b in zip(*chains):
        rel = 0.0
        for f in oracle.DYN_FIELDS:
            x, y = np.asarray(a[f]), np.asarray(b[f])
            assert np.isfinite(x).all() and np.isfinite(y).all()
            rel = max(rel, float(np.abs(x - y).max() / max(np.abs(y).max(), 1e-300)))
        drift.append(rel)
    print("fused vs FFTPACK-exact window chain, max rel diff per window:",
          " ".join(f"{r:.2e}" for r in drift), flush=True)
    assert drift[0] <= FUSED_TOL
    assert max(drift) <= CHAIN_DRIFT_TOL, drift


def test_window_graph_is_bitwise_the_launched_window(pg, cuda):
    """sml_dyn_window (stepone + 24 leapfrog steps as ONE captured hipGraph) against
    the same window launched step by step (stepone, stloop clock on the host): same
    state, radiation state and clock, for two consecutive windows (entry lradsw of
    the second one comes from the first)."""
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state(4)
    out = []
    for graph in (False, True):
        d = Dynamics()
        d.set_forcing(**forcing)
        d.set_state(st)
        d.set_physics(_window_bc(pg, d))
        d.set_rad_state(None)
        d.set_clock(1, True)
        clocks = []
        for _ in range(2):
            d.window(24, graph=graph)
            clocks.append(d.get_clock())
        torch.cuda.synchronize()
        out.append((d.get_state(), d.get_rad_state(), clocks))
        d.close()
    (a, ra, ca), (b, rb, cb) = out
    assert ca == cb
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(a[f], b[f])
    for k in ra:
        np.testing.assert_array_equal(ra[k], rb[k])



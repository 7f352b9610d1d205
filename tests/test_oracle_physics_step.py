"""The oracle's step WITH its own phypar (phys_inputs -> phypar_grid -> dyn_step)
against the reference's `step`, whose grtend calls the reference phypar
(tests/golden/dyn_ref.npz, make_dyn_golden.py: lradsw = .false., radiation state
zero as after radset).  This pins the physics-input path (geop(1), uvspec, grid of
time level 1) end to end, not just phypar on given inputs.

The boundary fields are the ones make_dyn_golden.py set in the reference's modules;
phis0 is the grid image of phis (the reference used its own grid, the oracle's
DFT differs by ~1e-13 relative).  Tolerance: max |err| <= TOL x max |field|."""
import numpy as np
import pytest

import oracle
from conftest import DYN_CASES

TOL = 1e-12


def dyn_bc(g):
    """phypar boundary fields of the dyn_ref.npz fixture (make_dyn_golden.py:145-177)."""
    ngp = oracle.NGP
    phis0 = oracle.grid(np.ascontiguousarray(g["phis"]).view(np.float64).reshape(32, 62), 1).ravel()
    bc = {k: np.zeros(ngp) for k in oracle.PHYS_BC}
    bc.update(fmask1=g["fmask1"], phis0=phis0, stl_am=g["stl"], sst_am=g["sst"], soilw_am=np.full(ngp, 0.4),
              alb_l=np.full(ngp, 0.25), alb_s=np.full(ngp, 0.07), snowc=np.zeros(ngp), forog=oracle.sflset(phis0))
    return bc


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def test_physics_inputs_reproduce_reference_tendencies(dyn_golden):
    g = dyn_golden
    st = oracle.dyn_state_copy(g)
    tend = oracle.phypar_grid(*oracle.phys_inputs(st, g["phis"]), dyn_bc(g), oracle.phys_state(), False)
    ref = g["phys"].reshape(4, oracle.KX, oracle.NGP)
    for v in range(4):
        assert _rel(tend[v], ref[v]) < TOL, v


@pytest.mark.parametrize("case", DYN_CASES)
def test_step_with_oracle_physics_matches_reference(dyn_golden, case):
    g = dyn_golden
    j1, j2, dt, alph = g[f"{case}_case"]
    st = oracle.dyn_state_copy(g)
    oracle.dyn_step_physics(st, g["phis"], g["tcorh"], g["qcorh"], dyn_bc(g), oracle.phys_state(), False,
                            int(j1), int(j2), float(dt), float(alph), float(g["rob"]), float(g["wil"]))
    lv = [0, 1] if int(j1) == 2 else [1]
    for f in oracle.DYN_FIELDS:
        assert _rel(st[f][lv], g[f"{case}_{f}"]) < TOL, (case, f, _rel(st[f][lv], g[f"{case}_{f}"]))

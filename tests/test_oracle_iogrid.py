"""Oracle iogrid(30)/(31) (SPEEDY window entry / exit, ppo_iogrid.f90:497-601).

ppo_iogrid.f90 cannot be built here (it needs mpires' internal_state_vector and
with it MPI), so these routines are pinned by composition: they are sequences of
vdspec / spec / trunct / uvspec / grid, each pinned to the reference by
tests/golden/spectral_ref.npz (test_oracle_golden.py).  The tests below check the
composition's own properties: the real(4) rounding, the q clip, the safety flags
and the exit -> entry round trip."""
import numpy as np

import oracle
from speedy_ml_amd.synthetic import dyn_state


def _state():
    st, _ = dyn_state(7)
    return oracle.dyn_state_copy(st)


def test_exit_entry_round_trip():
    st = _state()
    g4, lp = oracle.iogrid31(st)
    assert g4.shape == (8, 48, 96, 4)
    # T around tref, q >= ~0, winds moderate
    assert 150 < g4[..., 0].min() and g4[..., 0].max() < 330
    st2 = oracle.dyn_state_copy(st)
    for f in oracle.DYN_FIELDS:
        st2[f][0] = 0
    mm, safe = oracle.iogrid30(st2, g4, lp)
    assert safe
    # entry re-truncates the real(4)-rounded grid: spectral state back to ~fp32 accuracy
    m = np.arange(31)[None, :]
    n = np.arange(32)[:, None]
    tri = (m + n) <= 30
    for f in ("t", "ps"):
        a, b = st2[f][0], st[f][0]
        assert np.abs(a - b)[..., tri].max() <= 1e-6 * np.abs(b).max() + 1e-12, f
    for f in ("vor", "div"):
        a, b = st2[f][0], st[f][0]
        assert np.abs(a - b)[..., tri].max() <= 1e-5 * np.abs(b).max(), f
    # level 2 untouched
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(st2[f][1], st[f][1])
    # the re-gridded min/max are those of the exit grid of the new state
    g4b, _ = oracle.iogrid31(st2)
    for v, col in enumerate((1, 2, 0, 3)):
        assert mm[2 * v] == g4b[..., col].min() and mm[2 * v + 1] == g4b[..., col].max()


def test_entry_rounds_to_real4_and_clips_q():
    st = _state()
    g4, lp = oracle.iogrid31(st)
    g4 = g4.copy()
    g4[..., 3] -= 0.5  # some negative humidity
    assert (g4[..., 3] < 0).any()
    a = oracle.dyn_state_copy(st)
    oracle.iogrid30(a, g4, lp)
    g4c = g4.astype(np.float32).astype(np.float64)
    g4c[..., 3] = np.maximum(g4c[..., 3], 0.0)
    b = oracle.dyn_state_copy(st)
    oracle.iogrid30(b, g4c, lp.astype(np.float32).astype(np.float64))
    for f in oracle.DYN_FIELDS:
        np.testing.assert_array_equal(a[f], b[f])


def test_safety_thresholds():
    st = _state()
    g4, lp = oracle.iogrid31(st)
    for col, val in ((1, 400.0), (2, -300.0), (0, 100.0), (3, 80.0)):
        g = g4.copy()
        g[3, 20:30, 40:60, col] = val  # a broad patch survives the T30 truncation
        _, safe = oracle.iogrid30(oracle.dyn_state_copy(st), g, lp)
        assert not safe, col

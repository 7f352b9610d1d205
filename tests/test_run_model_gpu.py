"""run_model on the GPU (sml_dyn_run_model; src/mpires.f90:1516-1628): the window entry
iogrid(30) with its safety check (ppo_iogrid.f90:563-577), the window, the exit
iogrid(31), then run_model's q floor (mpires.f90:1614-1616).  An unsafe entry state
makes agcm_main skip the integration (at_gcm.f90:37): the forecast is run_model's
copy of the input grid (q floored, :1550-1553) and run_speedy is false (:1623).

Comparisons are bitwise: run_model issues the same kernels as from_grid + window +
to_grid, and the floor / pass-through are selections, not arithmetic."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def dyn(cuda):
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    st0, forcing = dyn_state()
    d = Dynamics()
    d.set_forcing(**forcing)
    d.set_state(st0)
    d.set_physics(phys_boundary(d, forcing["phis"]))
    d.set_rad_state(None)
    d.set_clock(1, True)
    yield d
    d.close()


def _grids(seed=11, dry_top=True):
    from speedy_ml_amd.synthetic import synthetic_grids

    g4, g2, _ = synthetic_grids(seed)
    if dry_top:  # a dry stratosphere: the transforms' ringing puts q below 1e-6 there
        g4[:2, ..., 3] = 0.0
    return g4, g2


def _t(a, cuda):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


def test_run_model_is_window_plus_q_floor(cuda, dyn):
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    g4, g2 = _grids()
    dg4, dg2 = _t(g4, cuda), _t(g2, cuda)
    f4 = torch.zeros_like(dg4)
    f2 = torch.zeros_like(dg2)
    dyn.run_model(dg4, dg2, f4, f2, nleap=6)
    safe, mm = dyn.last_safe()
    assert safe, mm
    # the same chain on a second context, unfloored
    st0, forcing = dyn_state()
    ref = Dynamics()
    ref.set_forcing(**forcing)
    ref.set_state(st0)
    ref.set_physics(phys_boundary(ref, forcing["phis"]))
    ref.set_rad_state(None)
    ref.set_clock(1, True)
    r4 = torch.zeros_like(dg4)
    r2 = torch.zeros_like(dg2)
    ref.from_grid(dg4, dg2)
    ref.window(6)
    ref.to_grid(r4, r2)
    torch.cuda.synchronize()
    raw = r4.cpu().numpy()
    assert (raw[..., 3] < 1e-6).any(), "test setup: the forecast should have q below the floor somewhere"
    want = raw.copy()
    want[..., 3] = np.where(raw[..., 3] < 0.000001, 0.000001, raw[..., 3])
    np.testing.assert_array_equal(f4.cpu().numpy(), want)
    np.testing.assert_array_equal(f2.cpu().numpy(), r2.cpu().numpy())
    ref.close()


@pytest.mark.parametrize("bad", ["t_hot", "u_fast", "q_wet", "nan"])
def test_unsafe_state_returns_the_input_grid(cuda, dyn, bad):
    import torch

    g4, g2 = _grids(seed=5)
    # (the check reads the state re-gridded after spectral truncation: a single hot
    # point is smoothed away, so whole levels / bands are perturbed)
    if bad == "t_hot":
        g4[3, :, :, 0] = 400.0        # temperature > 330 K
    elif bad == "u_fast":
        g4[1, 10:20, :, 1] = 300.0    # |u| > 150 m/s
    elif bad == "q_wet":
        g4[7, :, :, 3] = 50.0         # q > 30 g/kg
    else:
        g4[0, 0, 0, 2] = np.nan
    dg4, dg2 = _t(g4, cuda), _t(g2, cuda)
    f4 = torch.zeros_like(dg4)
    f2 = torch.zeros_like(dg2)
    dyn.run_model(dg4, dg2, f4, f2, nleap=3)
    safe, mm = dyn.last_safe()
    assert not safe, mm
    want = g4.copy()
    want[..., 3] = np.where(g4[..., 3] < 0.000001, 0.000001, g4[..., 3])
    np.testing.assert_array_equal(f4.cpu().numpy(), want)
    np.testing.assert_array_equal(f2.cpu().numpy(), g2)


def test_safety_thresholds_match_iogrid(cuda, dyn):
    """sml_dyn_is_safe on min/max vectors at and across each threshold."""
    from speedy_ml_amd._lib import lib, ptr

    base = np.array([-10.0, 10.0, -10.0, 10.0, 200.0, 300.0, 0.0, 20.0])
    assert lib().sml_dyn_is_safe(ptr(base)) == 1
    edges = [(0, -150.0, True), (0, -150.0001, False), (1, 150.0, True), (1, 150.0001, False),
             (2, -120.0, True), (2, -120.0001, False), (3, 120.0, True), (3, 120.0001, False),
             (4, 160.0, True), (4, 159.999, False), (5, 330.0, True), (5, 330.001, False),
             (6, -6.0, True), (6, -6.0001, False), (7, 30.0, True), (7, 30.0001, False), (5, np.nan, False)]
    for i, v, ok in edges:
        mm = base.copy()
        mm[i] = v
        assert lib().sml_dyn_is_safe(ptr(mm)) == int(ok), (i, v)


def test_fused_and_unfused_run_model_agree(cuda):
    """sml_dyn_run_model's fused form (k_io_entry + the prepared window graph with
    iogrid(31)'s prep / gridy in its last kernel) against the unfused chain
    (sml_dyn_set_fused(0): from_grid, the 8/9-launch steps, k_io_prep + gridy +
    gridx): the unfused steps' Fourier transforms are FFTPACK's separate multiplies and
    adds, the fused ones contract a*b + c, so the forecasts agree to rounding
    (UNFUSED_TOL x max |field| per variable and level after 6 leapfrog steps)."""
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    UNFUSED_TOL = 1e-11
    g4, g2 = _grids(seed=17)
    dg4, dg2 = _t(g4, cuda), _t(g2, cuda)
    outs = []
    for fused in (True, False):
        d = Dynamics()
        d.set_fused(fused)
        st0, forcing = dyn_state()
        d.set_forcing(**forcing)
        d.set_state(st0)
        d.set_physics(phys_boundary(d, forcing["phis"]))
        d.set_rad_state(None)
        d.set_clock(1, True)
        f4 = torch.zeros_like(dg4)
        f2 = torch.zeros_like(dg2)
        d.run_model(dg4, dg2, f4, f2, nleap=6)
        safe, _ = d.last_safe()
        torch.cuda.synchronize()
        outs.append((f4.cpu().numpy(), f2.cpu().numpy(), safe))
        d.close()
    (a4, a2, sa), (b4, b2, sb) = outs
    assert sa and sb
    for v in range(4):
        for k in range(8):
            ref = np.abs(b4[k, :, :, v]).max()
            assert np.abs(a4[k, :, :, v] - b4[k, :, :, v]).max() <= UNFUSED_TOL * ref, (v, k)
    assert np.abs(a2 - b2).max() <= UNFUSED_TOL * np.abs(b2).max()


def test_a_late_exit_fails_its_own_window_only(cuda, dyn):
    """run_model's exit that gives up waiting for its safety check
    takes its window as unsafe (the forecast is the input grid) and marks a late word.
    That word must fail that window only: a standalone Dynamics (no hybrid loop to
    report and reset it) whose next window's check arrives in time reads safe again.
    The check is held back by a sleep kernel on the check stream (CU-masked, a queue of
    its own) while the exit's give-up time is zero; the windows run on a stream of their
    own (the legacy stream would wait for the sleep too)."""
    import ctypes

    import torch

    from speedy_ml_amd._lib import check, lib

    check(lib().sml_dyn_set_check_cus(dyn._h, 192, 64))
    g4, g2 = _grids(seed=5)
    dg4, dg2 = _t(g4, cuda), _t(g2, cuda)
    f4 = torch.zeros_like(dg4)
    f2 = torch.zeros_like(dg2)
    ws = torch.cuda.Stream()
    dyn.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)  # a first window: the check stream exists, the exit on time
    assert dyn.last_safe()[0]
    s = ctypes.c_void_p()
    check(lib().sml_dyn_check_stream(dyn._h, ctypes.byref(s)))
    assert s.value
    chk = torch.cuda.ExternalStream(s.value, device=cuda)
    check(lib().sml_dyn_set_check_timeout(dyn._h, 0))
    with torch.cuda.stream(chk):
        torch.cuda._sleep(200_000_000)  # ~85 ms ahead of the next check
    dyn.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)
    safe_late, _ = dyn.last_safe()
    torch.cuda.synchronize()
    late_f4 = f4.cpu().numpy()
    check(lib().sml_dyn_set_check_timeout(dyn._h, 1_000_000))
    dyn.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)
    safe_next, _ = dyn.last_safe()
    assert not safe_late, "the exit gave up on its check: that window is unsafe"
    want = g4.copy()
    want[..., 3] = np.where(g4[..., 3] < 0.000001, 0.000001, g4[..., 3])
    np.testing.assert_array_equal(late_f4, want)  # agcm_main's pass-through
    assert safe_next, "a late exit of an earlier window must not make this one unsafe"


def test_run_model_with_alternating_buffers_is_bitwise_the_fixed_buffer_chain(cuda):
    """A caller that ping-pongs its input / forecast buffers (run_model's window graph is
    keyed on them: one cached graph per buffer set) gets the chain a caller copying into
    fixed buffers gets."""
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    def ctx():
        st0, forcing = dyn_state()
        d = Dynamics()
        d.set_forcing(**forcing)
        d.set_state(st0)
        d.set_physics(phys_boundary(d, forcing["phis"]))
        d.set_rad_state(None)
        d.set_clock(1, True)
        return d

    g4, g2 = _grids()
    a, b = ctx(), ctx()
    try:
        # fixed: the forecast copied back into one input buffer pair
        i4, i2 = _t(g4, cuda), _t(g2, cuda)
        o4, o2 = torch.zeros_like(i4), torch.zeros_like(i2)
        for _ in range(3):
            a.run_model(i4, i2, o4, o2, nleap=4)
            i4.copy_(o4)
            i2.copy_(o2)
        # ping-pong: P -> Q, Q -> P, P -> Q (the third call replays the first's graph)
        p4, p2 = _t(g4, cuda), _t(g2, cuda)
        q4, q2 = torch.zeros_like(p4), torch.zeros_like(p2)
        b.run_model(p4, p2, q4, q2, nleap=4)
        b.run_model(q4, q2, p4, p2, nleap=4)
        b.run_model(p4, p2, q4, q2, nleap=4)
        torch.cuda.synchronize()
        assert a.last_safe()[0] and b.last_safe()[0]
        np.testing.assert_array_equal(q4.cpu().numpy(), o4.cpu().numpy())
        np.testing.assert_array_equal(q2.cpu().numpy(), o2.cpu().numpy())
    finally:
        a.close()
        b.close()

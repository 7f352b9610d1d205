"""configs[2] exactly as bench.py times it.

The bench's default loop is the full-size hybrid step with every schedule option on
at once: the two CU-disjoint streams (overlap), the pipelined begin
(sml_hybrid_set_pipelined: each advance issues the next step's update + v_ml
readout), the slab ocean in the exchange rows (sml_hybrid_set_slab) and run_model's
calendar driving the window's forcing (sml_hybrid_set_calendar -> sml_dyn_fordate
per window; on a slab step after the new hybrid SST on the main stream, otherwise on
SPEEDY's stream behind the previous window, sml_hybrid.hip advance).  Here that loop
runs 9 hybrid steps back to back -- across two day boundaries (the forcing recomputed
on SPEEDY's stream) and two slab steps (recomputed on the main stream behind the new
SST) -- with the host synchronising only at the end, and every buffer it leaves is
compared BITWISE with the same loop unpipelined and synchronised after every step:

  the loop's fb, lm, ov (outvecs + slab sst), g4 / g2 / pr (assembled grids),
  f4 / f2 (forecast), the slab state (wholegrid_sst, the ring, the slab feedback and
  outvecs), every atmo and slab reservoir state, and SPEEDY's own state: the spectral
  prognostics, the window's forcing (tcorh / qcorh), phypar's boundary fields (sst_am
  with the hybrid SST) and the radiation state.

Two pipelined runs: one polls run_speedy after every step as the bench does
(parallelmain.f90:268-270) and one never polls (the host enqueues all 9 steps and
syncs once).  A mis-ordered fordate -- a window reading a stale sst_am or qcorh --
changes the forecast and fails here, where the bench's finite / last_window_safe
properties would not.

Reference: parallelmain.f90:204-270 (the loop), mpires.f90:218-780 / 1516-1628
(sendrecievegrid, run_model and its date at :1545), cpl_sea.f90:38-46 (the hybrid
SST), ini_agcm_init.f90:57-89 (the window's forcing per date)."""
import numpy as np
import pytest

from speedy_ml_amd import domain

pytestmark = pytest.mark.gpu

STEPS = 9
TIMESTEP_SLAB = 24                 # a slab step every 4th hybrid step (steps 4 and 8)
CALENDAR = (1981, 24 * 58 + 12)    # windows from 1981-02-27 18 h: the day changes at steps 2 and 6 (the month too)


def _bench_loop(cuda, pipelined):
    """The bench's setup (bench.py main: synthetic full-size weights, slab ocean,
    date forcing, HybridLoop with its default streams) with timestep_slab 24 h."""
    import torch

    from speedy_ml_amd._lib import check, lib, ptr
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights, slab_fields,
                                         slab_start_outvec, slab_weights, surface_climatology, synthetic_grids)

    mask = domain.load_sst_mask()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in range(1152)]
    res = Reservoirs(list(range(1152)), mask, [s.n for s in sizes], [s.k for s in sizes])
    for r in range(1152):
        w = region_weights(r, bool(mask[r]), climatology=True)
        res.load_region_weights(r, w)
        res.set_state(r, initial_state(r, w.n))
    sreg = [r for r in range(1152) if mask[r]]
    sws = [slab_weights(r) for r in sreg]
    slab = Reservoirs(sreg, [0] * len(sreg), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0, nout=4,
                      ninp=[w.ninp for w in sws], out_index=[35] * 4)
    for j, w in enumerate(sws):
        slab.load_region_weights(j, w)
        slab.set_state(j, initial_state(sreg[j], w.n, seed=17))
    del sws
    base, smask, sice, tice = slab_fields()
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    bc = phys_boundary(dyn, forcing["phis"])
    surf, clim = surface_climatology(bc["fmask1"])
    bc["fmask1"] = surf["fmask_l"]
    dyn.set_physics(bc)
    dyn.set_surface(surf)
    dyn.set_climatology(clim)
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.ascontiguousarray(tice))))
    tisr = t(np.random.default_rng(13).standard_normal((1152, 16)))
    so = SlabOcean(slab, t(base), t(smask), timestep=6, timestep_slab=TIMESTEP_SLAB)
    loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=cuda, nout=140), cuda, tisr=tisr, slab=so)
    loop.set_calendar(*CALENDAR, 6)
    loop.set_pipelined(pipelined)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.start_slab(t(np.stack([slab_start_outvec(r) for r in sreg])))
    loop.sync()
    return loop, slab


def _everything(loop, slab):
    """Every buffer the loop, its reservoirs and SPEEDY hold (after loop.sync())."""
    import torch

    from speedy_ml_amd._lib import check, lib

    torch.cuda.synchronize()
    # a pipelined loop has the next step's begin in flight: discard it, so the atmo
    # states are the ones after the last step's update (sml_res_step_cancel)
    check(lib().sml_res_step_cancel(loop.res.handle))
    out = {k: getattr(loop, k).cpu().numpy().copy() for k in ("fb", "lm", "ov", "g4", "g2", "pr", "f4", "f2")}
    out.update({"slab_" + k: v for k, v in loop.slab_state().items()})
    out["x"] = np.concatenate([loop.res.get_state(i) for i in range(loop.res.nlocal)])
    out["slab_x"] = np.concatenate([slab.get_state(j) for j in range(slab.nlocal)])
    dyn = loop.dyn
    out.update({"state_" + k: v for k, v in dyn.get_state().items()})
    out.update({"forcing_" + k: v for k, v in dyn.get_forcing().items()})
    out.update({"bc_" + k: v for k, v in dyn.get_physics().items()})
    out.update({"rad_" + k: v for k, v in dyn.get_rad_state().items()})
    out["fordates"] = np.array([dyn.fordate_count()])
    return out


def _close(loop, slab):
    import torch

    loop.close()
    loop.dyn.close()
    loop.res.close()
    slab.close()
    torch.cuda.synchronize()


def test_bench_loop_pipelined_is_bitwise_the_synchronised_loop(cuda):
    runs = {}
    for name, pipelined, poll in (("reference", False, None), ("bench", True, True), ("unpolled", True, False)):
        loop, slab = _bench_loop(cuda, pipelined)
        assert loop.exchange_width == 140
        dates = []
        for _ in range(STEPS):
            dates.append(loop.window_date()[:3])
            loop.step()
            if poll is None:
                loop.sync()  # the reference: every step drained before the next is issued
                assert loop.run_speedy()
            elif poll:
                assert loop.run_speedy()  # the bench's per-step poll: waits for the safety check only
        loop.sync()
        assert loop.run_speedy()
        runs[name] = _everything(loop, slab)
        _close(loop, slab)
        # the run crossed a day (the forcing recomputed on SPEEDY's stream) and the
        # slab steps (recomputed behind the new SST on the main stream)
        assert len(set(dates)) >= 3, dates
    ref = runs["reference"]
    assert int(ref["fordates"][0]) >= 4, ref["fordates"]  # step 1, the new days at 2 and 6, the slab steps 4 and 8
    assert np.isfinite(ref["f4"]).all() and np.isfinite(ref["ov"]).all()
    assert np.abs(ref["slab_outvec"]).max() > 0
    for name in ("bench", "unpolled"):
        got = runs[name]
        assert set(got) == set(ref)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{name}: {k}")

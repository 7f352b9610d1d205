"""The slab ocean inside the native hybrid loop (sml_hybrid_set_slab /
sml_hybrid_start_slab), against the oracle chain.

Reference flow per hybrid step t (parallelmain.f90:225-261, defaults of
mod_reservoir.f90:36-44: timestep 6 h, timestep_slab 168 h, slab on, ML-only ocean):
  * every region's atmo predict;
  * when mod(t*timestep, timestep_slab) == 0: predict_slab_ml of every sst region's
    slab reservoir (mod_slab_ocean_reservoir.f90:1251-1296) from its feedback = the
    mean of the ring of the last timestep_slab/timestep - 1 atmo-input subsets
    (mpires.f90:755-757);
  * sendrecievegrid: wholegrid_sst = base_sst_grid, each region's slab sst (272 K
    without a slab) on its points, base_sst_grid on land (sea_mask > 0), 272 K floor
    (:288-319, 458-472); run_model hands it to the window as sst_hybrid, which ini_sea
    puts into sst_am (cpl_sea.f90:38-46); the atmo feedback's sst entries are the
    overlap tile of wholegrid_sst standardized with the slab's sst mean / std
    (:575-581, 733-736); the ring's column mod(t-1, R-1) takes the new feedback's
    atmo_training_data_idx entries (:755).

The oracle chain restates each of these (oracle.py: predict_f32_regions,
predict_slab_ml_f32, sst_grid, tile_2d, hybrid_sst_am, slab_input_index) with the
oracle's SPEEDY window.  Tolerances: outvecs / slab sst / reservoir states as the
configs[2] test (readout summation order, |err| <= 1e-11 (1 + |v|)); the chained
forecast grids and feedback within CHAIN_TOL of the field scale, since the GPU's and
the oracle's windows differ by rounding (FFTPACK vs DFT, FMA) that the chain carries
on; the ring and the SST grid likewise.

test_slab_loop_full_size: all 1152 full-size atmo reservoirs and 1027 full-size slab
reservoirs (n = 4032), the full 26-step window, timestep_slab = 24 h (a slab step
every 4th hybrid step, ring of 3) over 9 steps.
test_slab_loop_reference_cadence: the reference's 168 h / 6 h cadence (slab step 28,
ring of 27) over 29 steps, with reduced reservoirs and a 2-step leapfrog window."""
import numpy as np
import pytest

import oracle
from speedy_ml_amd import domain
from speedy_ml_amd.synthetic import (climatology_mean_std, initial_state, region_weights, slab_fields,
                                     slab_start_outvec, slab_weights)

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-11
CHAIN_TOL = 1e-10


def _scaled(a, b):
    return float((np.abs(np.asarray(a) - np.asarray(b)) / (1.0 + np.abs(np.asarray(b)))).max())


def _run(cuda, steps, timestep_slab, nleap, n_atmo=None, n_slab=None, calendar=None, pipelined=False):
    import ctypes

    import torch

    from speedy_ml_amd._lib import check, lib, ptr
    from speedy_ml_amd.dynamics import DELT, Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids

    mask = domain.load_sst_mask()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    # atmo reservoirs (the oracle keeps the compressed fp32 weights: ~3.7 MB a region)
    wgen = lambda r: region_weights(r, bool(mask[r]), climatology=True, n_override=n_atmo)  # noqa: E731
    if n_atmo is None:
        nk = [(s.n, s.k) for s in (domain.reservoir_sizes(r, bool(mask[r])) for r in range(1152))]
    else:
        nk = [(w.n, w.k) for w in map(wgen, range(1152))]
    res = Reservoirs(list(range(1152)), mask, [a for a, _ in nk], [b for _, b in nk])
    regs, xs = [], []
    for r in range(1152):
        w = wgen(r)
        res.load_region_weights(r, w)
        x0 = initial_state(r, w.n)
        res.set_state(r, x0)
        col, val = w.win_compressed()
        regs.append({"rows": w.rows, "cols": w.cols, "vals": w.vals, "win_col": col, "win_val": val,
                     "wout": w.wout, "mean": w.mean, "std": w.std})
        xs.append(x0.copy())
    # slab reservoirs of the sst regions
    sreg = [r for r in range(1152) if mask[r]]
    sws = [slab_weights(r, n_override=n_slab) for r in sreg]
    slab = Reservoirs(sreg, [0] * len(sreg), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0, nout=4,
                      ninp=[w.ninp for w in sws], out_index=[35] * 4)
    sxs = []
    for j, w in enumerate(sws):
        slab.load_region_weights(j, w)
        x0 = initial_state(sreg[j], w.n, seed=17)
        slab.set_state(j, x0)
        sxs.append(x0.copy())
    base, smask, sice, tice = slab_fields()
    # SPEEDY
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    bc = phys_boundary(dyn, forcing["phis"])
    if calendar is not None:  # the window's date-driven forcing (sml_dyn_fordate every advance)
        from speedy_ml_amd.synthetic import surface_climatology
        surf, clim = surface_climatology(bc["fmask1"])
        bc["fmask1"] = surf["fmask_l"]
    dyn.set_physics(bc)
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.ascontiguousarray(tice))))
    if calendar is not None:
        dyn.set_surface(surf)
        dyn.set_climatology(clim)
    tisr = np.random.default_rng(13).standard_normal((1152, 16))
    d_base, d_mask = t(base), t(smask)
    so = SlabOcean(slab, d_base, d_mask, timestep=6, timestep_slab=timestep_slab)
    loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=cuda), cuda, tisr=t(tisr), nleap=nleap, slab=so)
    assert loop.exchange_width == 140
    if calendar is not None:
        loop.set_calendar(calendar[0], calendar[1], 6)
        n_fordate = dyn.fordate_count()
    loop.set_pipelined(pipelined)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    sov0 = np.stack([slab_start_outvec(r) for r in sreg])
    loop.start_slab(t(sov0))
    loop.sync()
    got = []
    for _ in range(steps):
        loop.step()
        loop.sync()
        snap = {k: getattr(loop, k).cpu().numpy().copy() for k in ("ov", "fb", "f4", "f2")}
        snap.update(loop.slab_state())
        got.append(snap)
    if calendar is not None:
        n_fordate = dyn.fordate_count() - n_fordate
    if pipelined:  # the next step's begin is in flight: discard it (the states after the last update)
        check(lib().sml_res_step_cancel(res.handle))
    got_x = {r: res.get_state(r) for r in (0, 24, 500, 1151)}
    got_sx = {j: slab.get_state(j) for j in (0, len(sreg) // 2, len(sreg) - 1)}
    assert loop.run_speedy()
    loop.close()
    dyn.close()

    # ---- the oracle chain
    cmean, cstd = climatology_mean_std()
    ms = {r: (cmean, cstd if mask[r] else np.where(np.arange(36) == 35, 0.0, cstd)) for r in range(1152)}
    soff = np.concatenate([[0], np.cumsum([w.ninp for w in sws])])
    ring = np.zeros((timestep_slab // 6 - 1, int(soff[-1])))
    sst_rows = np.full((1152, 4), 272.0)
    sst_rows[sreg] = sov0
    s = oracle.dyn_state_copy(st0)
    rad = oracle.phys_state()
    lradsw = True
    bc_w = {k: np.array(v, copy=True) for k, v in bc.items()}
    slab_ms = {r: (sws[j].mean[35], sws[j].std[35]) for j, r in enumerate(sreg)}
    in2d = {r: domain.region_geometry(r).inx * domain.region_geometry(r).iny for r in range(1152)}

    def tile_all(ga, gb, gc, fa, fb_, sst_std):
        fbv, lmv = [], []
        for r in range(1152):
            mean, std = ms[r]
            fbv.append(oracle.tile_feedback(r, ga, gb, gc, mean, std, tisr[r, :in2d[r]], sst_std.get(r)))
            lmv.append(oracle.tile_local_model(r, fa, fb_, mean, std))
        return fbv, lmv

    fbv, lmv = tile_all(g4, g2, pr, f4, f2, {r: np.zeros(in2d[r]) for r in sreg})  # the start's sst entries: 0
    errs = {"ov": 0.0, "sov": 0.0, "fb": 0.0, "fc": 0.0, "sst": 0.0, "ring": 0.0}
    nslab_steps = 0
    tcorh, qcorh = forcing["tcorh"], forcing["qcorh"]
    cal_state, dates, want_fordate, last = {}, [], 0, None
    for step in range(1, steps + 1):
        ov = oracle.predict_f32_regions(regs, fbv, lmv, xs, nthreads=8)
        if (step * 6) % timestep_slab == 0:
            nslab_steps += 1
            acc = np.zeros(ring.shape[1])
            for c in range(ring.shape[0]):
                acc = acc + ring[c]
            sfb = acc / float(ring.shape[0])
            np.testing.assert_allclose(got[step - 1]["feedback"], sfb, rtol=0, atol=CHAIN_TOL * 10)
            for j, r in enumerate(sreg):
                w = sws[j]
                col, val = w.win_compressed()
                sst_rows[r], sxs[j] = oracle.predict_slab_ml_f32(w.rows, w.cols, w.vals, col, val, w.wout,
                                                                 sfb[soff[j]:soff[j + 1]], sxs[j], w.mean[35],
                                                                 w.std[35])
            errs["sov"] = max(errs["sov"], _scaled(got[step - 1]["outvec"], sst_rows[sreg]))
        g = got[step - 1]
        errs["ov"] = max(errs["ov"], _scaled(g["ov"][:, :136], ov))
        np.testing.assert_array_equal(g["ov"][[r for r in range(1152) if not mask[r]], 136:], 272.0)
        a4, a2, apr = oracle.assemble(ov)
        sst = oracle.sst_grid(sst_rows, base, smask)
        errs["sst"] = max(errs["sst"], _scaled(g["sst"], sst))
        if calendar is None:
            bc_w["sst_am"] = oracle.hybrid_sst_am(bc["sst_am"], sst.ravel(), sice, tice)
        else:  # run_model's date (mpires.f90:1545) -> agcm_init's forcing of the window
            y, mo, dd, _ = oracle.calendar_delta_hour(calendar[0], calendar[1] + step * 6, cal_state)
            dates.append((y, mo, dd))
            bc_w, tcorh, qcorh, _, _ = oracle.window_forcing(mo, dd, surf, bc, clim=clim, sst_hybrid=sst.ravel())
            slab_now = (step * 6) % timestep_slab == 0 or step == 1
            want_fordate += (mo, dd) != last or slab_now
            last = (mo, dd)
        _, safe = oracle.iogrid30(s, a4, a2)
        assert safe
        DT = DELT
        oracle.dyn_step_physics(s, forcing["phis"], tcorh, qcorh, bc_w, rad, lradsw, 1, 1,
                                0.5 * DT, 0.5)
        oracle.dyn_step_physics(s, forcing["phis"], tcorh, qcorh, bc_w, rad, lradsw, 1, 2,
                                DT, 0.5)
        for istep in range(1, nleap + 1):
            lradsw = istep % 3 == 1
            oracle.dyn_step_physics(s, forcing["phis"], tcorh, qcorh, bc_w, rad, lradsw, 2, 2,
                                    2 * DT, 0.5)
        o4, o2 = oracle.iogrid31(s)
        o4[..., 3] = np.where(o4[..., 3] < 0.000001, 0.000001, o4[..., 3])
        errs["fc"] = max(errs["fc"], max(np.abs(g["f4"][k, :, :, v] - o4[k, :, :, v]).max()
                                         / np.abs(o4[k, :, :, v]).max() for v in range(4) for k in range(8)))
        fbv, lmv = tile_all(a4, a2, apr, o4, o2,
                            {r: (oracle.tile_2d(r, sst) - slab_ms[r][0]) / slab_ms[r][1] for r in sreg})
        errs["fb"] = max(errs["fb"], float(np.abs(g["fb"] - np.concatenate(fbv)).max()))
        col = (step - 1) % ring.shape[0]
        ring[col] = np.concatenate([fbv[r][oracle.slab_input_index(r)] for r in sreg])
        errs["ring"] = max(errs["ring"], float(np.abs(g["ring"][col] - ring[col]).max()))
    assert nslab_steps >= 1
    if calendar is not None:  # the run crossed a day, and the forcing was rebuilt only when it changed
        assert len(set(dates)) >= 2, dates
        assert n_fordate == want_fordate, (n_fordate, want_fordate, dates)
    e_x = max(_scaled(got_x[r], xs[r]) for r in got_x)
    e_sx = max(_scaled(got_sx[j], sxs[j]) for j in got_sx)
    print(f"slab loop {steps} steps (slab every {timestep_slab // 6}): " +
          ", ".join(f"{k} {v:.2e}" for k, v in errs.items()) + f", x {e_x:.2e}, slab x {e_sx:.2e}")
    assert errs["sov"] <= OUT_TOL and errs["sst"] <= OUT_TOL
    assert errs["ov"] <= CHAIN_TOL and errs["fc"] <= CHAIN_TOL and errs["fb"] <= CHAIN_TOL
    assert errs["ring"] <= CHAIN_TOL and e_x <= CHAIN_TOL and e_sx <= CHAIN_TOL
    res.close()
    slab.close()


def test_slab_loop_full_size(cuda):
    _run(cuda, steps=9, timestep_slab=24, nleap=24)


def test_slab_loop_date_forcing(cuda):
    """run_model's calendar date drives the window's forcing (VERDICT r04 missing #1):
    the coupler's climatologies at the date, the slab's hybrid SST into sst_am, qcorh
    from it, the insolation of the day.  11 steps from 1981-02-27 06 h: across two
    days, the month boundary and slab steps (every 4th step), against the oracle
    chain's window_forcing."""
    _run(cuda, steps=11, timestep_slab=24, nleap=2, n_atmo=96, n_slab=200, calendar=(1981, 24 * 58 + 6))


def test_slab_loop_date_forcing_pipelined(cuda):
    """The same chain with the bench's pipelined loop: each advance
    issues the next step's reservoir begin beside the window, and fordate runs on
    SPEEDY's stream or behind a new SST on the main stream (sml_hybrid.hip advance)."""
    _run(cuda, steps=11, timestep_slab=24, nleap=2, n_atmo=96, n_slab=200, calendar=(1981, 24 * 58 + 6),
         pipelined=True)


def test_slab_loop_reference_cadence(cuda):
    _run(cuda, steps=29, timestep_slab=168, nleap=2, n_atmo=96, n_slab=200)

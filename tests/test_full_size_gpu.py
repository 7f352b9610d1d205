"""The headline configurations at full size (BASELINE.json configs[1] and [2]).

configs[1] -- the batched reservoir forward of all 1152 subdomains at full n
  (5760 / 6160 / 6048 / 5880 nodes, k = int(0.001 n^2)) on one GPU: two sml_res_step
  calls, every 12th region (all four shape classes, 96 regions) against the
  oracle's predict (mod_reservoir.f90:1416-1487) chained over the same two steps.
configs[2] -- the full hybrid step at full size: HybridLoop (the native loop) for
  two steps against the oracle chain predict -> assemble (mpires.f90:300-478) ->
  run_model (iogrid(30), stepone + 24 leapfrog steps with phypar, iogrid(31), q
  floor; mpires.f90:1516-1628) -> tile (mpires.f90:558-751): sampled regions'
  outvecs and states, and the window's forecast grids.

Tolerances (stated per quantity):
  reservoir state x        |err| <= 1e-14 (1 + |x|) per step   (device vs glibc tanh)
  outvec (configs[1])      |err| <= 1e-11 (1 + |v|)            (readout summation order)
  forecast grids           max |err| <= FC_TOL x max |field| per variable and level:
                           the 26-step window (DFT vs FFTPACK, physics sums;
                           test_window_ref_gpu.py) -- rounding grows through the chain
  outvec / x after window  |err| <= OUT2_TOL (1 + |v|): step 2's outvec carries the
                           window's forecast through the local model."""
import numpy as np
import pytest

import oracle
from speedy_ml_amd import domain
from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights

pytestmark = pytest.mark.gpu

X_TOL = 1e-14
OUT_TOL = 1e-11
FC_TOL = 1e-12
OUT2_TOL = 1e-12
SAMPLE = list(range(0, 1152, 12))


def _reservoirs(mask, climatology=False):
    from speedy_ml_amd.reservoir import Reservoirs

    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in range(1152)]
    res = Reservoirs(list(range(1152)), mask, [s.n for s in sizes], [s.k for s in sizes])
    for r in range(1152):
        w = region_weights(r, bool(mask[r]), climatology=climatology)
        res.load_region_weights(r, w)
        res.set_state(r, initial_state(r, w.n))
    return res


def _scaled(a, b):
    return (np.abs(a - b) / (1.0 + np.abs(b))).max()


def test_configs1_all_regions_full_size(cuda):
    mask = domain.load_sst_mask()
    res = _reservoirs(mask)
    assert sorted(set(int(v) for v in res.n)) == [5760, 5880, 6048, 6160]
    o = res.fb_offsets
    fbs = [np.concatenate([feedback_vector(r, int(o[r + 1] - o[r]), seed=7 + s) for r in range(1152)])
           for s in range(2)]
    lms = [np.stack([local_model_vector(r, seed=7 + s) for r in range(1152)]) for s in range(2)]
    outs = []
    for s in range(2):
        outs.append(res.predict_host(fbs[s], lms[s]))
    classes = set()
    for r in SAMPLE:
        w = region_weights(r, bool(mask[r]))
        col, val = w.win_compressed()
        x = initial_state(r, w.n)
        for s in range(2):
            ref, x = oracle.predict_f32(w.rows, w.cols, w.vals, col, val, w.wout, fbs[s][o[r]:o[r + 1]], lms[s][r],
                                        x, w.mean, w.std)
            assert _scaled(outs[s][r], ref) <= OUT_TOL, (r, s, _scaled(outs[s][r], ref))
        assert _scaled(res.get_state(r), x) <= 2 * X_TOL, r
        classes.add((w.n, w.sst))
    assert len(classes) == 4, classes
    res.close()


def test_configs2_hybrid_step_full_size(cuda):
    import torch

    from speedy_ml_amd.dynamics import DELT, Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop
    from speedy_ml_amd.synthetic import climatology_mean_std, dyn_state, phys_boundary, synthetic_grids

    mask = domain.load_sst_mask()
    res = _reservoirs(mask, climatology=True)
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    bc = phys_boundary(dyn, forcing["phis"])
    dyn.set_physics(bc)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    tisr = np.random.default_rng(13).standard_normal((1152, 16))
    loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=cuda), cuda, tisr=t(tisr))
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    ovs = []
    for _ in range(2):
        loop.step()
        loop.sync()
        ovs.append(loop.ov.cpu().numpy().copy())
    assert loop.run_speedy()
    got_f4, got_f2 = loop.f4.cpu().numpy(), loop.f2.cpu().numpy()
    got_x = {r: res.get_state(r) for r in SAMPLE}
    loop.close()

    # the oracle chain
    o = res.fb_offsets
    cmean, cstd = climatology_mean_std()  # region_weights(climatology=True): std(36) = 0 without sst
    ms = {r: (cmean, cstd if mask[r] else np.where(np.arange(36) == 35, 0.0, cstd)) for r in range(1152)}
    in2d = {r: domain.region_geometry(r).inx * domain.region_geometry(r).iny for r in range(1152)}

    def tile_all(ga, gb, gc, fa, fb_, old_fb):
        fbv, lmv = [], []
        for r in range(1152):
            mean, std = ms[r]
            k = in2d[r]
            sst_old = old_fb[r][4 * k * 8 + 2 * k:4 * k * 8 + 3 * k] if mask[r] else None
            fbv.append(oracle.tile_feedback(r, ga, gb, gc, mean, std, tisr[r, :k], sst_old))
            lmv.append(oracle.tile_local_model(r, fa, fb_, mean, std))
        return fbv, lmv

    fb0 = [feedback_vector(r, int(o[r + 1] - o[r])) * 0.0 for r in range(1152)]  # sst entries start at zero
    fbv, lmv = tile_all(g4, g2, pr, f4, f2, fb0)
    xs = {r: initial_state(r, domain.reservoir_sizes(r, bool(mask[r])).n) for r in range(1152)}
    s = oracle.dyn_state_copy(st0)
    rad = oracle.phys_state()
    lradsw = True
    fc = (forcing["phis"], forcing["tcorh"], forcing["qcorh"], bc, rad)
    for step in range(2):
        ov = np.zeros((1152, 136))
        for r in range(1152):
            w = region_weights(r, bool(mask[r]), climatology=True)
            col, val = w.win_compressed()
            ov[r], xs[r] = oracle.predict_f32(w.rows, w.cols, w.vals, col, val, w.wout, fbv[r], lmv[r], xs[r],
                                              w.mean, w.std)
        if step == 0:  # step 1's outvecs depend only on the start inputs
            for r in SAMPLE:
                assert _scaled(ovs[0][r], ov[r]) <= OUT_TOL, (r, _scaled(ovs[0][r], ov[r]))
        a4, a2, apr = oracle.assemble(ov)
        _, safe = oracle.iogrid30(s, a4, a2)
        assert safe
        oracle.dyn_step_physics(s, *fc, lradsw, 1, 1, 0.5 * DELT, 0.5)
        oracle.dyn_step_physics(s, *fc, lradsw, 1, 2, DELT, 0.5)
        for istep in range(1, 25):
            lradsw = istep % 3 == 1
            oracle.dyn_step_physics(s, *fc, lradsw, 2, 2, 2 * DELT, 0.5)
        o4, o2 = oracle.iogrid31(s)
        o4[..., 3] = np.where(o4[..., 3] < 0.000001, 0.000001, o4[..., 3])  # run_model's floor
        fbv, lmv = tile_all(a4, a2, apr, o4, o2, fbv)
    e_ov = max(_scaled(ovs[1][r], ov[r]) for r in SAMPLE)
    e_x = max(_scaled(got_x[r], xs[r]) for r in SAMPLE)
    e_fc = max(np.abs(got_f4[k, :, :, v] - o4[k, :, :, v]).max() / np.abs(o4[k, :, :, v]).max()
               for v in range(4) for k in range(8))
    e_f2 = np.abs(got_f2 - o2).max() / np.abs(o2).max()
    print(f"configs[2] after 2 hybrid steps: outvec {e_ov:.3e}, state {e_x:.3e}, forecast grid4d {e_fc:.3e}, "
          f"logp {e_f2:.3e}")
    assert e_ov <= OUT2_TOL and e_x <= OUT2_TOL
    assert e_fc <= FC_TOL and e_f2 <= FC_TOL
    dyn.close()
    res.close()

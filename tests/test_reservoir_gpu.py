"""GPU parity of the batched reservoir forward (sml_res_step) against the oracle's
restatement of predict (mod_reservoir.f90:1416-1487).

Tolerances (fp64 arithmetic on both sides): the SpMV rows are summed in the file's
entry order on both sides; the differences come from tanh (device vs glibc, <= 2
ulp) and the W_out readout's summation order (wave reductions vs sequential):
  state x : |err| <= 1e-14 * (1 + |x|)
  outvec  : |err| <= 1e-11 * (1 + |outvec|)
"""
import os

import numpy as np
import pytest

import oracle
from speedy_ml_amd import SmlError, domain
from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights

pytestmark = pytest.mark.gpu

X_TOL = 1e-14
OUT_TOL = 1e-11

# one region of every shape class, plus the periodic x edges
CASES = [(0, False), (5, True), (23, True), (24, False), (600, True), (1127, False), (1151, True)]


def _check(a, b, tol):
    err = np.abs(np.asarray(a) - np.asarray(b)) / (1.0 + np.abs(np.asarray(b)))
    assert err.max() <= tol, f"max scaled err {err.max():.3e} > {tol:.0e}"


def _build(cases, n_override=None, weight_dtype="f32", chunk_speedy=132, seed=1234):
    from speedy_ml_amd.reservoir import Reservoirs

    ws = [region_weights(r, s, seed=seed, n_override=n_override, chunk_speedy=chunk_speedy) for r, s in cases]
    res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws],
                     chunk_speedy=chunk_speedy, weight_dtype=weight_dtype)
    for i, w in enumerate(ws):
        assert res.ninp(i) == w.ninp
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(w.region, w.n))
    return res, ws


def _oracle_step(w, x, fb, lm, chunk_speedy=132):
    col, val = w.win_compressed()
    return oracle.predict_f32(w.rows, w.cols, w.vals, col, val, w.wout, fb, lm, x, w.mean, w.std,
                              chunk_speedy=chunk_speedy)


@pytest.mark.parametrize("steps", [1, 4])
def test_predict_small_reservoirs(cuda, steps):
    res, ws = _build(CASES, n_override=700)
    xs = [initial_state(w.region, w.n) for w in ws]
    for t in range(steps):
        fb = np.concatenate([feedback_vector(w.region + 17 * t, w.ninp) for w in ws])
        lm = np.stack([local_model_vector(w.region + 17 * t) for w in ws])
        out = res.predict_host(fb, lm)
        for i, w in enumerate(ws):
            o = res.fb_offsets
            ref, xs[i] = _oracle_step(w, xs[i], fb[o[i]:o[i + 1]], lm[i])
            _check(out[i], ref, OUT_TOL)
            _check(res.get_state(i), xs[i], X_TOL * (t + 1))


def test_predict_full_size_reservoirs(cuda):
    """Full-size regions of all four shape classes (n = 5760, 6160, 6048, 5880)."""
    cases = [(5, True), (30, False), (0, True), (1127, False)]
    res, ws = _build(cases)
    assert sorted(int(v) for v in res.n) == [5760, 5880, 6048, 6160]
    fb = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    lm = np.stack([local_model_vector(w.region) for w in ws])
    out = res.predict_host(fb, lm)
    for i, w in enumerate(ws):
        o = res.fb_offsets
        ref, x1 = _oracle_step(w, initial_state(w.region, w.n), fb[o[i]:o[i + 1]], lm[i])
        _check(out[i], ref, OUT_TOL)
        _check(res.get_state(i), x1, X_TOL)


def test_predict_f64_storage_and_dense_oracle(cuda):
    """fp64 weight storage, checked against the dense-W_in reference arithmetic."""
    res, ws = _build(CASES[:3], n_override=500, weight_dtype="f64")
    fb = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    lm = np.stack([local_model_vector(w.region) for w in ws])
    out = res.predict_host(fb, lm)
    for i, w in enumerate(ws):
        o = res.fb_offsets
        ref, x1 = oracle.predict(w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                                 w.wout.astype(np.float64), fb[o[i]:o[i + 1]], lm[i],
                                 initial_state(w.region, w.n), w.mean, w.std)
        _check(out[i], ref, OUT_TOL)
        _check(res.get_state(i), x1, X_TOL)


def test_long_rows_use_csr_fallback(cuda):
    """A with a 40-entry row and W_in with a 3-entry row exceed the ELL slots: the
    CSR copies are used; results still follow the file-order sums."""
    from speedy_ml_amd.reservoir import Reservoirs

    w = region_weights(300, True, n_override=700)
    rows = w.rows.copy()
    rows[:40] = 7  # row 7 gets 40 entries (duplicates of (7, col) add)
    win = w.win.copy()
    win[:, 20:23] = 0.0  # three empty rows keep nnz(W_in) <= n (the reserved capacity)
    win[:3, 11] = [0.25, -0.5, 0.125]  # row 12 of W_in reads three inputs
    res = Reservoirs([300], [1], [w.n], [w.k])
    res.load_region(0, rows, w.cols, w.vals, win, w.wout, w.mean, w.std)
    x0 = initial_state(300, w.n)
    res.set_state(0, x0)
    fb = feedback_vector(300, w.ninp)
    lm = local_model_vector(300)
    out = res.predict_host(fb, lm[None, :])
    ref, x1 = oracle.predict(rows, w.cols, w.vals.astype(np.float64), win.astype(np.float64),
                             w.wout.astype(np.float64), fb, lm, x0, w.mean, w.std)
    _check(out[0], ref, OUT_TOL)
    _check(res.get_state(0), x1, X_TOL)


def test_ml_only_mode(cuda):
    """chunk_speedy = 0: predict_ml (mod_reservoir.f90:1489-1533)."""
    res, ws = _build(CASES[:4], n_override=600, chunk_speedy=0)
    fb = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    out = res.predict_host(fb, None)
    for i, w in enumerate(ws):
        o = res.fb_offsets
        ref, _ = _oracle_step(w, initial_state(w.region, w.n), fb[o[i]:o[i + 1]], None, chunk_speedy=0)
        _check(out[i], ref, OUT_TOL)


def test_device_path_and_kernel_timing(cuda):
    import torch

    res, ws = _build(CASES, n_override=800)
    fb, lm, ov = res.alloc_io(cuda)
    fb_h = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    lm_h = np.stack([local_model_vector(w.region) for w in ws])
    fb.copy_(torch.from_numpy(fb_h))
    lm.copy_(torch.from_numpy(lm_h))
    res.enable_timing(3)
    for _ in range(3):
        res.predict(fb, lm, ov)
    upd, rd = res.kernel_times()
    assert len(upd) == 3 and (upd > 0).all() and (rd > 0).all()
    xs = [initial_state(w.region, w.n) for w in ws]
    for _ in range(3):
        refs = []
        for i, w in enumerate(ws):
            o = res.fb_offsets
            r, xs[i] = _oracle_step(w, xs[i], fb_h[o[i]:o[i + 1]], lm_h[i])
            refs.append(r)
    _check(ov.cpu().numpy(), np.stack(refs), OUT_TOL)


def test_error_paths(cuda):
    from speedy_ml_amd.reservoir import Reservoirs

    w = region_weights(5, True, n_override=600)
    res = Reservoirs([5], [1], [w.n], [w.k])
    with pytest.raises(SmlError, match="no weights loaded"):
        res.predict_host(np.zeros(w.ninp), np.zeros((1, 132)))
    bad = w.wout.astype(np.float64)
    bad[0, 0] = 0.1  # not representable in fp32 storage
    with pytest.raises(SmlError, match="not representable"):
        res.load_region(0, w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64), bad, w.mean, w.std)
    rows = w.rows.copy()
    rows[3] = w.n + 1
    with pytest.raises(SmlError, match="out of range"):
        res.load_region(0, rows, w.cols, w.vals, w.win, w.wout, w.mean, w.std)
    with pytest.raises(SmlError, match="out of range"):
        res.set_state(2, np.zeros(w.n))


def test_netcdf_loaded_weights_match(cuda, tmp_path):
    from speedy_ml_amd.reservoir import Reservoirs, write_region_netcdf

    w = region_weights(600, True, n_override=576)
    p = str(tmp_path / "worker_0600_level_1_trial.nc")
    write_region_netcdf(p, w.win, w.wout, w.rows, w.cols, w.vals, w.mean, w.std)
    a = Reservoirs([600], [1], [w.n], [w.k])
    b = Reservoirs([600], [1], [w.n], [w.k])
    a.load_region_weights(0, w)
    b.load_netcdf(0, p)
    fb = feedback_vector(600, w.ninp)
    lm = local_model_vector(600)[None, :]
    np.testing.assert_array_equal(a.predict_host(fb, lm), b.predict_host(fb, lm))


def test_synchronize_matches_oracle(cuda):
    """synchronize (mod_reservoir.f90:1352-1378) updates the state exactly as
    predict does (:1440-1446) without the readout: the oracle's predict restatement
    gives the reference state sequence."""
    import torch

    res, ws = _build(CASES[:4], n_override=700)
    length = 6
    tot = res.fb_offsets[-1]
    rng = np.random.default_rng(4)
    inputs = rng.standard_normal((length, tot))
    res.synchronize(torch.from_numpy(inputs).to(cuda), length)
    torch.cuda.synchronize()
    o = res.fb_offsets
    for i, w in enumerate(ws):
        x = initial_state(w.region, w.n)
        for t in range(length):
            _, x = _oracle_step(w, x, inputs[t, o[i]:o[i + 1]], np.zeros(132))
        _check(res.get_state(i), x, 1e-13)


def test_synchronize_matches_repeated_updates(cuda):
    """synchronize (mod_reservoir.f90:1352-1378): `length` updates from a sequence of
    feedback blocks, no readout -- the state equals `length` oracle predict steps'
    x; a following predict reads out from it."""
    import torch

    res, ws = _build(CASES[:4], n_override=500)
    length = 5
    o = res.fb_offsets
    stride = int(o[-1]) + 3  # padded blocks: stride > packed size
    blocks = np.zeros((length, stride))
    for t in range(length):
        blocks[t, :o[-1]] = np.concatenate([feedback_vector(w.region + 31 * t, w.ninp) for w in ws])
    res.synchronize(torch.from_numpy(blocks).to(cuda), length, stride=stride)
    torch.cuda.synchronize()
    lm0 = np.zeros(132)
    for i, w in enumerate(ws):
        x = initial_state(w.region, w.n)
        for t in range(length):
            _, x = _oracle_step(w, x, blocks[t, o[i]:o[i + 1]], lm0)
        _check(res.get_state(i), x, X_TOL * length)
    with pytest.raises(ValueError):
        res.synchronize(torch.zeros(10, dtype=torch.float64, device=cuda), length)
    res.synchronize(torch.zeros(1, dtype=torch.float64, device=cuda), 0)  # no-op


def test_dense_win_grows_the_pool(cuda):
    """A dense W_in (every entry nonzero, the reference's n x ninp matmul, :1443) on one
    region of a context sized for the trained one-entry-per-row W_in: the W_in pool is
    re-laid (grow_win_pool) and the other regions keep their weights."""
    from speedy_ml_amd.reservoir import Reservoirs

    ws = [region_weights(r, s, n_override=400, seed=9) for r, s in CASES[:3]]
    res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws])
    rng = np.random.default_rng(4)
    dense = (0.02 * (2.0 * rng.random(ws[1].win.shape) - 1.0)).astype(np.float32)
    ws[1].win[:] = dense
    for i, w in enumerate(ws):
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(w.region, w.n))
    fb = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    lm = np.stack([local_model_vector(w.region) for w in ws])
    out = res.predict_host(fb, lm)
    o = res.fb_offsets
    for i, w in enumerate(ws):
        ref, x1 = oracle.predict(w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                                 w.wout.astype(np.float64), fb[o[i]:o[i + 1]], lm[i],
                                 initial_state(w.region, w.n), w.mean, w.std)
        _check(out[i], ref, OUT_TOL)
        _check(res.get_state(i), x1, 1e-13)  # dense sum order: matmul's column order, skipped zeros


@pytest.mark.parametrize("weight_dtype", ["f32", "f64"])
def test_finish_grid_equals_tile_then_finish(cuda, weight_dtype):
    """sml_res_step_finish_grid (local-model tiling fused into the v_p finish; v_p in 7
    column groups on different threads, added in group order) vs begin ->
    tile_local_model -> finish (one thread per output, the same groups in turn): outvecs
    and the tiled local model bitwise, with and without the local-model output, and
    with the finish one thread per output (SML_RES_PATH_UNGROUPED_FINISH)."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import synthetic_grids

    ws = [region_weights(r, s, n_override=300, seed=11) for r, s in CASES]
    g4, g2, pr = synthetic_grids(7)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    outs = {}
    for mode in ("fused", "fused_nolm", "two", "fused_ungrouped"):
        res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws],
                         weight_dtype=weight_dtype)
        if mode == "fused_ungrouped":  # the finish one thread per output (vp_sum), not in column groups
            res.set_reference_paths(ungrouped_finish=True)
        for i, w in enumerate(ws):
            if weight_dtype == "f64":
                res.load_region(i, w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                                w.wout.astype(np.float64), w.mean, w.std)
            else:
                res.load_region_weights(i, w)
            res.set_state(i, initial_state(w.region, w.n))
        fb = t(np.concatenate([feedback_vector(w.region, w.ninp) for w in ws]))
        lm = torch.full((len(ws), 132), -7.0, dtype=torch.float64, device=cuda)
        ov = torch.zeros((len(ws), 136), dtype=torch.float64, device=cuda)
        res.predict_begin(fb)
        if mode == "two":
            res.tile_local_model(t(g4), t(g2), lm)
            res.predict_finish(lm, ov)
        else:
            res.predict_finish_grid(t(g4), t(g2), lm if mode == "fused" else None, ov)
        torch.cuda.synchronize()
        outs[mode] = (ov.cpu().numpy(), lm.cpu().numpy())
        res.close()
    np.testing.assert_array_equal(outs["fused"][0], outs["two"][0])
    np.testing.assert_array_equal(outs["fused_nolm"][0], outs["two"][0])
    np.testing.assert_array_equal(outs["fused_ungrouped"][0], outs["two"][0])
    np.testing.assert_array_equal(outs["fused"][1], outs["two"][1])
    assert (outs["fused_nolm"][1] == -7.0).all()  # no local-model output requested


def test_finish_grid_ml_only_needs_no_forecast(cuda):
    """An ML-only context (chunk_speedy 0, predict_ml) finishes without forecast grids."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs

    ws = [region_weights(r, s, n_override=200, chunk_speedy=0) for r, s in CASES[:2]]
    res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws],
                     chunk_speedy=0)
    for i, w in enumerate(ws):
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(w.region, w.n))
    fbh = np.concatenate([feedback_vector(w.region, w.ninp) for w in ws])
    fb = torch.from_numpy(fbh).to(cuda)
    ov = torch.zeros((len(ws), 136), dtype=torch.float64, device=cuda)
    res.predict_begin(fb)
    res.predict_finish_grid(None, None, None, ov)
    torch.cuda.synchronize()
    o = res.fb_offsets
    for i, w in enumerate(ws):
        ref, _ = _oracle_step(w, initial_state(w.region, w.n), fbh[o[i]:o[i + 1]], None, chunk_speedy=0)
        _check(ov[i].cpu().numpy(), ref, OUT_TOL)


def test_start_prediction(cuda):
    """start_prediction (mod_reservoir.f90:938-959): synchronize_print over the first
    `length` blocks (the oracle's update sequence), then block `length` becomes the
    feedback."""
    import torch

    res, ws = _build(CASES[:3], n_override=500)
    length = 5
    tot = res.fb_offsets[-1]
    rng = np.random.default_rng(8)
    inputs = rng.standard_normal((length + 1, tot))
    fb = torch.zeros(tot, dtype=torch.float64, device=cuda)
    res.start_prediction(torch.from_numpy(inputs).to(cuda), length, fb)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(fb.cpu().numpy(), inputs[length])
    o = res.fb_offsets
    for i, w in enumerate(ws):
        x = initial_state(w.region, w.n)
        for t in range(length):
            _, x = _oracle_step(w, x, inputs[t, o[i]:o[i + 1]], np.zeros(132))
        _check(res.get_state(i), x, 1e-13)


def _slab_weights(region, ninp, n, seed):
    """A slab-ocean reservoir's arrays (mod_slab_ocean_reservoir.f90: m = 4000 nodes,
    one W_in entry per row, sst outputs of the 2x2 region)."""
    rng = np.random.default_rng([seed, region])
    k = int(0.001 * n * n)
    rows = np.concatenate([rng.permutation(n)[:min(n, k - b)] + 1 for b in range(0, k, n)]).astype(np.int32)
    cols = np.concatenate([rng.permutation(n)[:min(n, k - b)] + 1 for b in range(0, k, n)]).astype(np.int32)
    vals = (rng.random(k) * 0.3).astype(np.float32)
    win = np.zeros((ninp, n), dtype=np.float32)
    q = n // ninp
    for j in range(q):
        win[np.arange(ninp), np.arange(ninp) * q + j] = (0.5 * (2 * rng.random(ninp) - 1)).astype(np.float32)
    wout = ((rng.random((4 + n, 4)) * 2 - 1) * 0.01).astype(np.float32)
    mean = rng.random(36).astype(np.float32).astype(np.float64)
    std = (0.5 + rng.random(36)).astype(np.float32).astype(np.float64)
    return rows, cols, vals, win, wout, mean, std


def test_predict_slab_matches_oracle(cuda):
    """predict_slab (mod_slab_ocean_reservoir.f90:1201-1249) on a generic context over
    3 steps: x = tanh(A x + W_in u), outvec = W_out [local_model; x~], local_model =
    the raw outvec (:1235), outvec * std(sst) + mean(sst) -- against the oracle's
    predict with chunk_speedy = 4 and no unstandardize."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs

    regions, ninp = [10, 500, 1100], [48, 40, 64]
    n = [4000 // p * p for p in ninp]
    ws = [_slab_weights(r, p, m, 6) for r, p, m in zip(regions, ninp, n)]
    res = Reservoirs(regions, [0, 0, 0], n, [len(w[0]) for w in ws], chunk_speedy=4, nout=4, ninp=ninp,
                     out_index=[35] * 4)
    xs = []
    for i, w in enumerate(ws):
        res.load_region(i, *w)
        xs.append(0.1 * np.random.default_rng(i).random(n[i]))
        res.set_state(i, xs[i])
    rng = np.random.default_rng(2)
    lm = rng.standard_normal((3, 4))
    d_lm = torch.from_numpy(lm.copy()).to(cuda)
    d_next = torch.zeros_like(d_lm)
    d_ov = torch.zeros((3, 4), dtype=torch.float64, device=cuda)
    o = res.fb_offsets
    for step in range(3):
        fb = rng.standard_normal(int(o[-1]))
        res.predict_slab(torch.from_numpy(fb).to(cuda), d_lm, d_next, d_ov)
        torch.cuda.synchronize()
        got_ov, got_raw = d_ov.cpu().numpy(), d_next.cpu().numpy()
        for i, w in enumerate(ws):
            rows, cols, vals, win, wout, mean, std = w
            raw, xs[i] = oracle.predict(rows, cols, vals.astype(np.float64), win.astype(np.float64),
                                        wout.astype(np.float64), fb[o[i]:o[i + 1]], lm[i], xs[i], mean, std,
                                        chunk_speedy=4, unstandardize=False)
            _check(got_raw[i], raw, OUT_TOL)
            _check(got_ov[i], raw * std[35] + mean[35], OUT_TOL)
            _check(res.get_state(i), xs[i], 1e-13)
            lm[i] = raw
        d_lm, d_next = d_next, d_lm  # the raw outvec is the next local model
    with pytest.raises(SmlError):
        res.predict_slab(torch.from_numpy(fb).to(cuda), d_lm, d_lm, d_ov)  # aliasing refused


@pytest.mark.parametrize("weight_dtype", ["f32", "f64"])
@pytest.mark.parametrize("mode", [1, 2])
def test_fused_begin_is_bitwise_the_two_launch_begin(cuda, weight_dtype, mode):
    """sml_res_set_begin_mode 1 / 2 (k_res_begin: update + v_ml readout, one block per
    region) vs mode 0 (k_res_update grid, then k_res_readout<ml> grid): outvecs and
    states bitwise over 3 chained begin + finish steps at full reservoir size."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs

    cases = CASES[:4]
    ws = [region_weights(r, s, seed=5) for r, s in cases]
    fbs = [np.concatenate([feedback_vector(w.region, w.ninp) for w in ws]) * (1.0 + 0.1 * k) for k in range(3)]
    lm = torch.from_numpy(np.stack([local_model_vector(w.region) for w in ws])).to(cuda)
    outs = {}
    for m in (0, mode):
        res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws],
                         weight_dtype=weight_dtype)
        for i, w in enumerate(ws):
            if weight_dtype == "f64":
                res.load_region(i, w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                                w.wout.astype(np.float64), w.mean, w.std)
            else:
                res.load_region_weights(i, w)
            res.set_state(i, initial_state(w.region, w.n))
        res.set_begin_mode(m)
        assert res.begin_fused == (m > 0)
        ov = torch.zeros((len(ws), 136), dtype=torch.float64, device=cuda)
        seq = []
        for fbh in fbs:
            res.predict_begin(torch.from_numpy(fbh).to(cuda))
            res.predict_finish(lm, ov)
            torch.cuda.synchronize()
            seq.append((ov.cpu().numpy().copy(), [res.get_state(i) for i in range(len(ws))]))
        outs[m] = seq
        res.close()
    for (oa, xa), (ob, xb) in zip(outs[0], outs[mode]):
        np.testing.assert_array_equal(oa, ob)
        for a, b in zip(xa, xb):
            np.testing.assert_array_equal(a, b)


def test_finish_assemble_is_bitwise_finish_then_assemble(cuda):
    """sml_res_step_finish_assemble (one rank, every region in order: the finish also
    scatters the outvecs into the global grids with the root's clips) vs
    finish_grid -> assemble: outvecs, local models and all three grids bitwise; a
    context that does not hold every region is refused."""
    import torch

    from speedy_ml_amd import SmlError
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import synthetic_grids

    mask = domain.load_sst_mask()
    ws = [region_weights(r, bool(mask[r]), n_override=96, seed=3) for r in range(domain.NUM_REGIONS)]
    g4h, g2h, prh = synthetic_grids(5)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    outs = {}
    for fused in (False, True):
        res = Reservoirs([w.region for w in ws], [w.sst for w in ws], [w.n for w in ws], [w.k for w in ws])
        for i, w in enumerate(ws):
            res.load_region_weights(i, w)
            res.set_state(i, initial_state(w.region, w.n))
        fb = t(np.concatenate([feedback_vector(w.region, w.ninp) for w in ws]))
        lm = torch.zeros((len(ws), 132), dtype=torch.float64, device=cuda)
        ov = torch.zeros((len(ws), 136), dtype=torch.float64, device=cuda)
        g4 = torch.full((4 * 96 * 48 * 8,), -1.0, dtype=torch.float64, device=cuda)
        g2 = torch.full((96 * 48,), -1.0, dtype=torch.float64, device=cuda)
        pr = torch.full((96 * 48,), -1.0, dtype=torch.float64, device=cuda)
        res.predict_begin(fb)
        if fused:
            res.predict_finish_assemble(t(g4h), t(g2h), lm, ov, g4, g2, pr)
        else:
            res.predict_finish_grid(t(g4h), t(g2h), lm, ov)
            res.assemble(ov, g4, g2, pr)
        torch.cuda.synchronize()
        outs[fused] = [a.cpu().numpy() for a in (ov, lm, g4, g2, pr)]
        res.close()
    for name, a, b in zip(("ov", "lm", "g4", "g2", "pr"), outs[False], outs[True]):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert (outs[True][2] != -1.0).all() and (outs[True][4] >= 0).all()  # every grid point assembled
    part = Reservoirs([w.region for w in ws[:4]], [w.sst for w in ws[:4]], [w.n for w in ws[:4]],
                      [w.k for w in ws[:4]])
    with pytest.raises(SmlError, match="every region"):
        part.predict_finish_assemble(None, None, None, None, None, None, None)
    part.close()


@pytest.mark.parametrize("cus,wdt", [(0, "f32"), (192, "f32"), (7, "f32"), (1, "f32"), (192, "f64"), (7, "f64")])
def test_balanced_update_is_bitwise_the_per_region_update(cuda, cus, wdt):
    """k_res_update_bal (a persistent grid, one block per CU, each block an equal share
    of all the rank's rows, two passes of A rows in flight, the next region's x staged
    into a second LDS buffer) against k_res_update (a block per region;
    SML_RES_PATH_PER_REGION): the states, x_aug-fed outvecs and the begin / finish split bitwise over
    3 steps, for grids of every CU (0), the hybrid loop's reservoir CUs (192), an odd
    grid (7: shares straddle many regions) and one block (every region in turn); with
    fp32 and fp64 weights (the Pair<double> 16-B loads)."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs

    mask = domain.load_sst_mask()
    regions = list(range(0, 1152, 9))  # 128 regions of every shape class, full size
    ws = [region_weights(r, bool(mask[r])) for r in regions]
    fb = np.concatenate([feedback_vector(r, w.ninp) for r, w in zip(regions, ws)])
    lm = np.stack([local_model_vector(r) for r in regions])
    outs, states = {}, {}
    for bal in (False, True):
        res = Reservoirs(regions, mask[regions], [w.n for w in ws], [w.k for w in ws], weight_dtype=wdt)
        res.set_reference_paths(per_region=not bal)
        for i, w in enumerate(ws):
            res.load_region_weights(i, w)
            res.set_state(i, initial_state(regions[i], w.n))
        res.set_update_cus(cus)
        assert res.update_balanced() == bal
        dfb, dlm = torch.from_numpy(fb).to(cuda), torch.from_numpy(lm).to(cuda)
        ov = torch.zeros((len(regions), 136), dtype=torch.float64, device=cuda)
        got = []
        for step in range(3):
            if step == 1:  # the split form: begin (the update + v_ml) then finish
                res.predict_begin(dfb)
                res.predict_finish(dlm, ov)
            else:
                res.predict(dfb, dlm, ov)
            torch.cuda.synchronize()
            got.append(ov.cpu().numpy().copy())
        outs[bal] = got
        states[bal] = [res.get_state(i) for i in range(len(regions))]
        res.close()
    for a, b in zip(outs[False], outs[True]):
        np.testing.assert_array_equal(a, b)
    for i, (a, b) in enumerate(zip(states[False], states[True])):
        np.testing.assert_array_equal(a, b, err_msg=f"region {regions[i]}")


@pytest.mark.parametrize("wdt", ["f32", "f64"])
def test_ell_layouts_are_bitwise_the_csr_update(cuda, wdt):
    """A's ELL main width chosen per region (pair-major slots, an overflow list for the
    rows one longer) and W_in's implicit block-diagonal column: every
    layout the builder picks gives the states and outvecs of the CSR copies
    (SML_RES_PATH_CSR) bit for bit, in the balanced and the per-region update, over 3
    steps -- and the oracle's within its tolerance.  Regions: every full-size shape
    class (n 6048 with 4.8 % of rows one longer -> overflow; 5880 / 5760 -> 6 slots;
    6160 -> overflow), a region of 2- and 3-entry rows (2 slots + overflow), and a W_in
    whose columns are permuted (not block-diagonal: its column is read).  Both weight
    precisions (fp64: the Pair<double> loads, the overflow entries, the depth-2 pipeline)."""
    import torch

    from speedy_ml_amd.reservoir import Reservoirs

    mask = domain.load_sst_mask()
    regions = [0, 5, 23, 24, 600, 1127, 1151, 300, 301]
    ws = [region_weights(r, bool(mask[r])) for r in regions[:7]]
    w3 = region_weights(300, bool(mask[300]), n_override=3000)  # k = 0.001 n^2 ~ 2.6 n: rows of 2 or 3
    wp = region_weights(301, bool(mask[301]), n_override=2000)
    perm = np.random.default_rng(5).permutation(wp.ninp)
    wp.win = wp.win[perm].copy()  # each row still one entry, columns no longer i / q
    ws += [w3, wp]
    fb = np.concatenate([feedback_vector(r, w.ninp) for r, w in zip(regions, ws)])
    lm = np.stack([local_model_vector(r) for r in regions])
    outs, states, layouts = {}, {}, {}
    for form in ("csr", "per_region", "balanced"):
        res = Reservoirs(regions, mask[regions], [w.n for w in ws], [w.k for w in ws], weight_dtype=wdt)
        res.set_reference_paths(csr=form == "csr", per_region=form != "balanced")
        for i, w in enumerate(ws):
            res.load_region_weights(i, w)
            res.set_state(i, initial_state(regions[i], w.n))
        assert res.update_balanced() == (form == "balanced")
        layouts[form] = [res.ell_layout(i) for i in range(len(regions))]
        dfb, dlm = torch.from_numpy(fb).to(cuda), torch.from_numpy(lm).to(cuda)
        ov = torch.zeros((len(regions), 136), dtype=torch.float64, device=cuda)
        got = []
        for step in range(3):
            res.predict(dfb, dlm, ov)
            torch.cuda.synchronize()
            got.append(ov.cpu().numpy().copy())
        outs[form] = got
        states[form] = [res.get_state(i) for i in range(len(regions))]
        res.close()
    assert all(lay["a_width"] == 0 and not lay["win_ell"] for lay in layouts["csr"])
    lay = layouts["balanced"]
    by_n = {w.n: lay[i] for i, w in enumerate(ws[:7])}
    assert by_n[6048]["a_width"] == 6 and by_n[6048]["a_overflow"]
    assert by_n[5880]["a_width"] == 6 and not by_n[5880]["a_overflow"]
    assert lay[7]["a_width"] == 2 and lay[7]["a_overflow"]
    assert all(lay[i]["win_q"] == ws[i].n // ws[i].ninp for i in range(8))
    assert lay[8]["win_q"] == 0 and lay[8]["win_ell"]
    for form in ("per_region", "balanced"):
        for a, b in zip(outs["csr"], outs[form]):
            np.testing.assert_array_equal(a, b, err_msg=form)
        for i, (a, b) in enumerate(zip(states["csr"], states[form])):
            np.testing.assert_array_equal(a, b, err_msg=f"{form} region {regions[i]}")
    # and the oracle, one step from the start state
    o = np.concatenate([[0], np.cumsum([w.ninp for w in ws])])
    for i, w in enumerate(ws):
        ref, x1 = _oracle_step(w, initial_state(w.region, w.n), fb[o[i]:o[i + 1]], lm[i])
        _check(outs["balanced"][0][i], ref, OUT_TOL)

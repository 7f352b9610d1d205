"""CPU checks of the reservoir / exchange oracle's internal consistency.

The reference reservoir path needs MKL, MPI and netCDF, which this image lacks, so
no reference build pins these functions ("parity unpinned").  These
tests pin the oracle's properties that follow from the reference code instead."""
import numpy as np

import oracle
from speedy_ml_amd import domain
from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights


def test_dense_and_compressed_win_paths_agree_bitwise():
    # matmul(win, feedback) over a block-diagonal win adds exact zeros only, so the
    # compressed restatement must be bit-identical (mod_reservoir.f90:1443)
    for region, sst in ((5, True), (0, False), (1151, True)):
        w = region_weights(region, sst, n_override=700)
        x0 = initial_state(region, w.n)
        fb = feedback_vector(region, w.ninp)
        lm = local_model_vector(region)
        a, xa = oracle.predict(w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                               w.wout.astype(np.float64), fb, lm, x0, w.mean, w.std)
        col, val = w.win_compressed()
        b, xb = oracle.predict_f32(w.rows, w.cols, w.vals, col, val, w.wout, fb, lm, x0, w.mean, w.std)
        np.testing.assert_array_equal(xa, xb)
        np.testing.assert_array_equal(a, b)


def test_leakage_one_and_even_squaring():
    w = region_weights(100, True, n_override=600)
    x0 = initial_state(100, w.n)
    fb = feedback_vector(100, w.ninp)
    lm = local_model_vector(100)
    # W_out = identity-like picks: outvec_o = x_aug[j_o]; no unstandardize
    wout = np.zeros((132 + w.n, 136))
    picks = np.arange(136) * 3 + 132
    wout[picks, np.arange(136)] = 1.0
    out, x1 = oracle.predict(w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64), wout, fb, lm,
                             x0, w.mean, w.std, unstandardize=False)
    j = picks - 132
    expect = np.where(j % 2 == 1, x1[j] ** 2, x1[j])  # x_temp(2:n:2)**2, 1-based even
    np.testing.assert_array_equal(out, expect)
    assert np.all(np.abs(x1) < 1.0)


def test_unstandardize_index_map():
    mean = np.arange(36, dtype=np.float64)
    std = np.ones(36) * 2.0
    v = np.zeros(136)
    oracle.lib().orc_unstandardize_res(oracle._p(v), 2, 2, 8, oracle._p(mean), oracle._p(std), 1, 1, 33, 35)
    for o in range(128):
        var, z = o % 4, o // 16
        assert v[o] == var * 8 + z
    assert np.all(v[128:132] == 32) and np.all(v[132:136] == 34)


def test_assemble_then_tile_reproduces_region_values():
    rng = np.random.default_rng(0)
    outvecs = rng.standard_normal((1152, 136)) + 1.0
    g4, g2, pr = oracle.assemble(outvecs)
    assert g4[..., 3].min() >= 1e-6  # q clip
    assert (pr[pr != 0] >= 1e-5).all()  # precip clip
    mean = np.zeros(36)
    std = np.ones(36)
    tisr = np.zeros(16)
    for region in (0, 1, 23, 24, 575, 1151):
        g = domain.region_geometry(region)
        fb = oracle.tile_feedback(region, g4, g2, pr, mean, std, tisr)
        lm = oracle.tile_local_model(region, g4, g2, mean, std)
        ov = outvecs[region].copy()
        q = np.arange(128) % 4 == 3
        ov[:128][q] = np.maximum(ov[:128][q], 1e-6)
        np.testing.assert_array_equal(lm[:128], ov[:128])
        np.testing.assert_array_equal(lm[128:132], ov[128:132])
        # the region's own points sit at offset (1, 1) (or (1, 0) at the south pole)
        ix, iy = g.inx, g.iny
        oy = 0 if g.in_ystart == g.res_ystart else 1
        atmo = fb[:4 * ix * iy * 8].reshape(8, iy, ix, 4)
        np.testing.assert_array_equal(atmo[:, oy:oy + 2, 1:3, :].ravel(),
                                      ov[:128].reshape(8, 2, 2, 4).ravel())


def test_predict_regions_openmp_equals_predict():
    # the cpu_baseline's reservoir leg (orc_predict_regions) is orc_predict per region
    regs, fbs, lms, xs, expect = [], [], [], [], []
    for region, sst in ((3, True), (40, False), (700, True)):
        w = region_weights(region, sst, n_override=500)
        d = dict(rows=np.ascontiguousarray(w.rows, np.int32), cols=np.ascontiguousarray(w.cols, np.int32),
                 vals=w.vals.astype(np.float64), win=np.ascontiguousarray(w.win, np.float64),
                 wout=np.ascontiguousarray(w.wout, np.float64), mean=np.ascontiguousarray(w.mean, np.float64),
                 std=np.ascontiguousarray(w.std, np.float64))
        regs.append(d)
        fbs.append(feedback_vector(region, w.ninp))
        lms.append(local_model_vector(region))
        x0 = initial_state(region, w.n)
        xs.append(x0.copy())
        expect.append(oracle.predict(d["rows"], d["cols"], d["vals"], d["win"], d["wout"], fbs[-1], lms[-1], x0,
                                     d["mean"], d["std"]))
    out = oracle.predict_regions(regs, fbs, lms, xs, nthreads=3)
    for i, (o, x) in enumerate(expect):
        np.testing.assert_array_equal(out[i], o)
        np.testing.assert_array_equal(xs[i], x)

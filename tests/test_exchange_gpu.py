"""GPU parity of the exchange kernels that replace sendrecievegrid (mpires.f90:218-780):
assemble (outvec tiles -> global grids + clips) and tile (overlap input tiles and
SPEEDY local vectors, standardized).  Pure index maps plus (x-mean)/std: compared
bit for bit with the oracle, for all 1152 regions."""
import numpy as np
import pytest

import oracle
from speedy_ml_amd import domain
from speedy_ml_amd.synthetic import region_weights, synthetic_grids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def all_regions(cuda):
    from speedy_ml_amd.reservoir import Reservoirs

    mask = domain.load_sst_mask()
    ws = [region_weights(r, bool(mask[r]), n_override=1, seed=77) for r in range(1152)]
    res = Reservoirs(list(range(1152)), mask, [w.n for w in ws], [w.k for w in ws])
    for i, w in enumerate(ws):
        res.load_region_weights(i, w)
    return res, ws, mask


def _t(a, dev):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)


def test_assemble_all_regions(all_regions, cuda):
    import torch

    res, _, _ = all_regions
    rng = np.random.default_rng(1)
    ov = rng.standard_normal((1152, 136)) * 1e-3 + rng.standard_normal((1152, 136))
    g4 = torch.full((8, 48, 96, 4), -7.0, dtype=torch.float64, device=cuda)
    g2 = torch.zeros((48, 96), dtype=torch.float64, device=cuda)
    pr = torch.zeros((48, 96), dtype=torch.float64, device=cuda)
    res.assemble(_t(ov, cuda), g4, g2, pr)
    o4, o2, op = oracle.assemble(ov)
    np.testing.assert_array_equal(g4.cpu().numpy(), o4)
    np.testing.assert_array_equal(g2.cpu().numpy(), o2)
    np.testing.assert_array_equal(pr.cpu().numpy(), op)


def test_tile_inputs_all_regions(all_regions, cuda):
    import torch

    res, ws, mask = all_regions
    g4, g2, pr = synthetic_grids(3)
    f4, f2, _ = synthetic_grids(4)
    rng = np.random.default_rng(2)
    tisr = rng.standard_normal((1152, 16))
    fb0 = rng.standard_normal(int(res.fb_offsets[-1]))
    fb = _t(fb0, cuda)
    lm = torch.zeros((1152, 132), dtype=torch.float64, device=cuda)
    res.tile_inputs(_t(g4, cuda), _t(g2, cuda), _t(pr, cuda), _t(f4, cuda), _t(f2, cuda), _t(tisr, cuda), fb, lm)
    fb_h, lm_h = fb.cpu().numpy(), lm.cpu().numpy()
    o = res.fb_offsets
    for r in range(1152):
        w = ws[r]
        g = domain.region_geometry(r)
        in2d = g.inx * g.iny
        natmo = 4 * in2d * 8
        sst_old = fb0[o[r] + natmo + 2 * in2d: o[r] + natmo + 3 * in2d] if mask[r] else None
        ref = oracle.tile_feedback(r, g4, g2, pr, w.mean, w.std, tisr[r, :in2d], sst_old)
        np.testing.assert_array_equal(fb_h[o[r]:o[r + 1]], ref)
        np.testing.assert_array_equal(lm_h[r], oracle.tile_local_model(r, f4, f2, w.mean, w.std))


def test_keep_tisr_when_null(all_regions, cuda):
    import torch

    res, _, _ = all_regions
    g4, g2, pr = synthetic_grids(3)
    fb0 = np.random.default_rng(3).standard_normal(int(res.fb_offsets[-1]))
    fb = _t(fb0, cuda)
    res.tile_inputs(_t(g4, cuda), _t(g2, cuda), _t(pr, cuda), None, None, None, fb, None)
    out = fb.cpu().numpy()
    o = res.fb_offsets
    g = domain.region_geometry(700)
    in2d = g.inx * g.iny
    np.testing.assert_array_equal(out[o[701] - in2d:o[701]], fb0[o[701] - in2d:o[701]])  # tisr kept

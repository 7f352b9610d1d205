"""GPU W_out training (sml_train_*) against the oracle.

Gram / cross products: fp64 MFMA sums in a different order than the oracle's
loops: max |err| <= 1e-12 x max |G| (GRAM_TOL).  Solve: the hand-written batched
Cholesky (k_chol_* / k_solve_*, 128-blocked) vs the oracle's dgesv restatement; both solve the same SPD system, so they agree to
rounding x cond: on well-conditioned systems max |err| <= 1e-9 x max |W|
(W_TOL); with the reference's default (ill-conditioned) betas the test checks the
relative residual of the regularised system (RES_TOL)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

GRAM_TOL = 1e-12
W_TOL = 1e-9
RES_TOL = 1e-9


def _data(naugs, nout, m, seed=0):
    rng = np.random.default_rng(seed)
    S, T = [], []
    for n in naugs:
        s = np.tanh(rng.standard_normal((m, n)))
        s[:, :132] = rng.standard_normal((m, 132))
        S.append(s)
        T.append(rng.standard_normal((m, nout)))
    return S, T


def _pack(arrs, cuda):
    import torch

    return torch.from_numpy(np.concatenate([a.ravel() for a in arrs])).to(cuda)


def _accumulate(tr, S, T, batches, cuda):
    m = S[0].shape[0]
    edges = np.linspace(0, m, batches + 1).astype(int)
    for a, b in zip(edges[:-1], edges[1:]):
        tr.accumulate(_pack([s[a:b] for s in S], cuda), _pack([t[a:b] for t in T], cuda), int(b - a))


def test_gram_matches_oracle(cuda):
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [200, 263, 331], 136, 300
    S, T = _data(naugs, nout, m)
    tr = Trainer(naugs, nout)
    assert tr.npad == 384
    _accumulate(tr, S, T, 2, cuda)
    for i, n in enumerate(naugs):
        G, B = tr.gram(i)
        Go = np.zeros((n, n))
        Bo = np.zeros((n, nout))
        oracle.train_accumulate(S[i], T[i], Go, Bo)
        Gl = np.tril(G[:n, :n].T)  # C (npad, npad) = transposed column-major; lower triangle valid
        assert np.abs(Gl - np.tril(Go)).max() <= GRAM_TOL * np.abs(Go).max()
        assert np.abs(B[:, :n].T - Bo).max() <= GRAM_TOL * np.abs(Bo).max()
        assert not G[n:, :].any() and not G[:, n:].any()  # padding rows/cols stay zero
    tr.close()


@pytest.mark.parametrize("using_prior,beta_res,beta_model,prior_val",
                         [(False, 0.5, 1.0, 0.0), (True, 0.7, 1.0, 0.25)])
def test_solve_matches_oracle_well_conditioned(cuda, using_prior, beta_res, beta_model, prior_val):
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [200, 331], 136, 400
    S, T = _data(naugs, nout, m, seed=3)
    tr = Trainer(naugs, nout)
    _accumulate(tr, S, T, 3, cuda)
    w, info = tr.solve(132, beta_res, beta_model, using_prior, prior_val)
    assert (info == 0).all()
    views = tr.wout_views(w)
    for i, n in enumerate(naugs):
        Go = np.zeros((n, n))
        Bo = np.zeros((n, nout))
        oracle.train_accumulate(S[i], T[i], Go, Bo)
        wo, oinfo = oracle.train_solve(Go, Bo, 132, beta_res, beta_model, using_prior, prior_val)
        assert oinfo == 0
        got = views[i].cpu().numpy()
        assert np.abs(got - wo).max() <= W_TOL * np.abs(wo).max(), i
    tr.close()


def test_solve_reference_defaults_residual(cuda):
    """beta_res = 0.001, beta_model = 1 squared (using_prior, mod_reservoir.f90:67,93-99)."""
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [300], 136, 500
    S, T = _data(naugs, nout, m, seed=5)
    tr = Trainer(naugs, nout)
    _accumulate(tr, S, T, 2, cuda)
    w, info = tr.solve()
    assert info[0] == 0
    W = tr.wout_views(w)[0].cpu().numpy()  # (naug, nout) == wout(nout, naug)
    n = naugs[0]
    G = S[0].T @ S[0] + np.diag(np.where(np.arange(n) < 132, 1.0, 1e-6))
    B = S[0].T @ T[0]
    res = np.abs(G @ W - B).max() / np.abs(B).max()
    assert res <= RES_TOL, res
    tr.close()


def test_full_size_region(cuda):
    """One 6000-node-class region (naug = 132 + 6160): tiles up to index 49."""
    import torch

    from speedy_ml_amd.training import Trainer

    naug, nout, m = 6292, 136, 96
    S, T = _data([naug], nout, m, seed=9)
    tr = Trainer([naug], nout)
    assert tr.npad == 6400
    _accumulate(tr, S, T, 1, cuda)
    G, B = tr.gram(0)
    Go = S[0].T @ S[0]
    Gl = np.tril(G[:naug, :naug].T)
    assert np.abs(Gl - np.tril(Go)).max() <= GRAM_TOL * np.abs(Go).max()
    assert np.abs(B[:, :naug].T - S[0].T @ T[0]).max() <= GRAM_TOL * np.abs(Go).max()
    w, info = tr.solve(132, 1.0, 1.0, False, 0.0)  # well conditioned: diag + 1
    assert info[0] == 0
    W = tr.wout_views(w)[0].cpu().numpy()
    Greg = Go + np.eye(naug)
    res = np.abs(Greg @ W - S[0].T @ T[0]).max() / np.abs(S[0].T @ T[0]).max()
    assert res <= RES_TOL, res
    tr.close()
    torch.cuda.synchronize()


def test_solve_multi_block_matches_oracle(cuda):
    """npad = 896: seven block columns -- panel, trailing update and both block
    triangular solves run at every position; three regions of different naug
    share the padded batch."""
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [777, 401, 640], 136, 1000
    S, T = _data(naugs, nout, m, seed=11)
    tr = Trainer(naugs, nout)
    assert tr.npad == 896
    _accumulate(tr, S, T, 2, cuda)
    w, info = tr.solve(132, 0.3, 1.0, True, 0.5)
    assert (info == 0).all()
    views = tr.wout_views(w)
    for i, n in enumerate(naugs):
        Go = np.zeros((n, n))
        Bo = np.zeros((n, nout))
        oracle.train_accumulate(S[i], T[i], Go, Bo)
        wo, oinfo = oracle.train_solve(Go, Bo, 132, 0.3, 1.0, True, 0.5)
        assert oinfo == 0
        got = views[i].cpu().numpy()
        assert np.abs(got - wo).max() <= W_TOL * np.abs(wo).max(), (i, np.abs(got - wo).max())
    tr.close()


def test_solve_reports_the_first_non_positive_pivot(cuda):
    """potrf's info: 1-based index of the first leading minor that is not positive
    definite (a negative beta_res makes the regularised Gram indefinite)."""
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [300, 260], 136, 200
    S, T = _data(naugs, nout, m, seed=21)
    tr = Trainer(naugs, nout)
    _accumulate(tr, S, T, 1, cuda)
    _, info = tr.solve(132, -30.0, 1.0, False, 0.0)
    for i, n in enumerate(naugs):
        G = S[i].T @ S[i] + np.diag(np.where(np.arange(n) < 132, 1.0, -30.0))
        first = next(j for j in range(1, n + 1) if np.linalg.eigvalsh(G[:j, :j]).min() <= 0.0)
        assert info[i] == first, (i, info[i], first)
    tr.close()


def test_cholesky_panel_widths_agree(cuda):
    """The factor with panels of three block columns (sml_train_set_panel) against the
    default eight, over npad = 896: the narrow panels run every kind of launch --
    left-looking in-panel steps (the diagonal tile's quadrant update, the fused update +
    L_ik), the panel's first column, and right-looking trailing updates between panels
    -- whose sums group differently, so W_out agrees within W_TOL."""
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [777, 401, 640], 136, 1000
    S, T = _data(naugs, nout, m, seed=13)
    ws = []
    for panel in (None, 3):
        tr = Trainer(naugs, nout)
        if panel is not None:
            tr.set_panel(panel)
        _accumulate(tr, S, T, 2, cuda)
        w, info = tr.solve(132, 0.3, 1.0, True, 0.5)
        assert (info == 0).all()
        ws.append(w.cpu().numpy().copy())
        tr.close()
    assert np.abs(ws[1] - ws[0]).max() <= W_TOL * np.abs(ws[0]).max()


def test_forked_forward_substitution_is_deterministic(cuda):
    """Panels of two block columns over npad = 896 (four panels): each panel's forward
    substitution runs on the context's second stream beside the later panels'
    factorisation (sml_train_solve's fork / join).  It reads only finished block columns
    and writes only B, so three solves of the same sums are bitwise equal, and W_out
    agrees with the oracle."""
    from speedy_ml_amd.training import Trainer

    naugs, nout, m = [777, 401, 640], 136, 1000
    S, T = _data(naugs, nout, m, seed=17)
    tr = Trainer(naugs, nout)
    tr.set_panel(2)
    ws = []
    for _ in range(3):
        tr.reset()
        _accumulate(tr, S, T, 2, cuda)
        w, info = tr.solve(132, 0.3, 1.0, True, 0.5)
        assert (info == 0).all()
        ws.append(w.cpu().numpy().copy())
    assert all(np.array_equal(ws[0], w) for w in ws[1:])
    views = tr.wout_views(w)
    for i, n in enumerate(naugs):
        Go = np.zeros((n, n))
        Bo = np.zeros((n, nout))
        oracle.train_accumulate(S[i], T[i], Go, Bo)
        wo, _ = oracle.train_solve(Go, Bo, 132, 0.3, 1.0, True, 0.5)
        got = views[i].cpu().numpy()
        assert np.abs(got - wo).max() <= W_TOL * np.abs(wo).max(), (i, np.abs(got - wo).max())
    tr.close()

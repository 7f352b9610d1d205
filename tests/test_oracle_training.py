"""Oracle W_out training (chunking_matmul + fit_chunk_hybrid + mldivide).

mldivide calls LAPACK dgesv, which the reference does not vendor; the oracle
restates dgesv's published algorithm (LU with partial pivoting) and is checked
here against numpy.linalg.solve (LAPACK gesv).  No reference test or fixture
covers training: parity unpinned beyond the cited call sites."""
import numpy as np
import pytest

import oracle


def _data(naug, nout, m, seed=0):
    rng = np.random.default_rng(seed)
    S = np.tanh(rng.standard_normal((m, naug)))  # C (m, naug) == Fortran augmented_states(naug, m)
    S[:, :32] = rng.standard_normal((m, 32))      # "imperfect model" rows
    T = rng.standard_normal((m, nout))
    return S, T


def test_accumulate_matches_numpy_and_batches_add():
    S, T = _data(90, 20, 70)
    G = np.zeros((90, 90))
    B = np.zeros((90, 20))
    oracle.train_accumulate(S[:40], T[:40], G, B)
    oracle.train_accumulate(S[40:], T[40:], G, B)
    np.testing.assert_allclose(G, S.T @ S, rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(B, S.T @ T, rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("using_prior,prior_val", [(False, 0.0), (True, 0.0), (True, 0.3)])
def test_solve_matches_lapack(using_prior, prior_val):
    naug, nout, ncs = 120, 24, 32
    S, T = _data(naug, nout, 400, seed=1)
    G = S.T @ S
    B = S.T @ T
    bm, br = 1.0, 0.05
    w, info = oracle.train_solve(G, B, ncs, br, bm, using_prior, prior_val)
    assert info == 0
    add = np.where(np.arange(naug) < ncs, bm ** 2 if using_prior else bm, br ** 2 if using_prior else br)
    Greg = G + np.diag(add)
    rhs = B.copy()
    if using_prior:
        for i in range(min(ncs, nout)):
            rhs[i, i] += prior_val * bm ** 2
    ref = np.linalg.solve(Greg.T, rhs)
    np.testing.assert_allclose(w, ref, rtol=0, atol=1e-10 * np.abs(ref).max())

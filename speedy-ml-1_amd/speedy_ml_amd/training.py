"""W_out ridge training on the GPU (libspeedyml sml_train_*).

Mirrors the reference's training tail for a batch of regions:
chunking_matmul (src/mod_reservoir.f90:1643-1699) accumulates G = S S^T and
B = T S^T over batches of time steps, fit_chunk_hybrid / fit_chunk_ml
(:1233-1332 / :1175-1231) regularise and solve through mldivide
(src/mod_linalg.f90:109-151).

Layouts (C order of the reference's Fortran arrays): per region S is
augmented_states(naug, m) == C (m, naug), T is targetdata(nout, m) == C (m, nout),
W_out is wout(nout, naug) == C (naug, nout).  Device buffers are float64 CUDA
tensors packing the regions back to back.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr, stream_ptr

NOUT = 136


class Trainer:
    def __init__(self, naug, nout: int = NOUT):
        self.naug = [int(x) for x in naug]
        self.nout = nout
        arr = np.asarray(self.naug, dtype=np.int32)
        h = ctypes.c_void_p()
        check(lib().sml_train_create(len(self.naug), ptr(arr), nout, ctypes.byref(h)))
        self._h = h
        n = ctypes.c_int()
        check(lib().sml_train_npad(h, ctypes.byref(n)))
        self.npad = n.value

    def close(self):
        if self._h:
            lib().sml_train_destroy(self._h)
            self._h = None

    __del__ = close

    def set_panel(self, panel: int):
        """Block columns per Cholesky panel (sml_train_set_panel; default 8)."""
        check(lib().sml_train_set_panel(self._h, int(panel)))

    def reset(self, stream=None):
        check(lib().sml_train_reset(self._h, stream_ptr(stream)))

    def accumulate(self, states, targets, m: int, stream=None):
        """states: packed device tensor, sum(naug) * m doubles (region i's
        (m, naug_i) block after region i-1's); targets: len(naug) * m * nout."""
        if states.numel() != sum(self.naug) * m or targets.numel() != len(self.naug) * m * self.nout:
            raise ValueError("states / targets sizes do not match the regions and m")
        check(lib().sml_train_accumulate(self._h, ptr(states), ptr(targets), m, stream_ptr(stream)))

    def solve(self, ncs: int = 132, beta_res: float = 0.001, beta_model: float = 1.0, using_prior: bool = True,
              prior_val: float = 0.0, out=None, stream=None):
        """Regularise + solve (consumes the accumulators).  Returns (wout packed
        device tensor, per-region potrf info after synchronisation)."""
        import torch

        total = sum(self.naug) * self.nout
        if out is None:
            out = torch.empty(total, dtype=torch.float64, device="cuda")
        info = np.zeros(len(self.naug), dtype=np.int32)
        check(lib().sml_train_solve(self._h, ncs, beta_res, beta_model, int(using_prior), prior_val, ptr(out),
                                    ptr(info), stream_ptr(stream)))
        torch.cuda.synchronize()
        return out, info

    def wout_views(self, packed):
        """Per-region (naug_i, nout) views (C order == Fortran wout(nout, naug_i))."""
        views, off = [], 0
        for n in self.naug:
            views.append(packed[off:off + n * self.nout].view(n, self.nout))
            off += n * self.nout
        return views

    def gram(self, i: int):
        """Host copies: G (npad, npad) lower triangle valid (C order = transposed
        Fortran), B as (nout, npad) C order = B(j, o) at j + npad*o."""
        G = np.zeros((self.npad, self.npad))
        B = np.zeros((self.nout, self.npad))
        check(lib().sml_train_get_gram(self._h, i, ptr(G), ptr(B)))
        return G, B

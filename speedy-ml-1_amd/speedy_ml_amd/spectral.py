"""Batched T30 spectral transforms on the GPU (libspeedyml sml_*_batched).

Mirrors the reference's spe_spectral interface (grid, spec, vdspec, uvspec,
gridx/gridy/specx/specy; src/spe_spectral.f90:351-538,
src/spe_subfft_fftpack.f90:15-87), one call per batch of fields.  Tensors are torch
float64 CUDA tensors used as device memory (plumbing); all arithmetic happens in
the HIP kernels.  Shapes (C order == the reference's Fortran column-major arrays):
spectral (nf, 32, 62), Fourier (nf, 48, 62), grid (nf, 48, 96).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr, stream_ptr

EARTH_RADIUS = 6.371e6  # mod_dyncon1.f90 rearth


def _need_cuda(*ts):
    for t in ts:
        if not (t.is_cuda and t.dtype.is_floating_point and t.element_size() == 8 and t.is_contiguous()):
            raise ValueError("expected contiguous float64 CUDA tensors")


class Spectral:
    def __init__(self, radius: float = EARTH_RADIUS):
        h = ctypes.c_void_p()
        check(lib().sml_spectral_create(radius, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            lib().sml_spectral_destroy(self._h)
            self._h = None

    __del__ = close

    def tables(self):
        sia = np.zeros(24)
        wt = np.zeros(24)
        cpol = np.zeros((24, 32, 62))
        nsh2 = np.zeros(32, dtype=np.int32)
        check(lib().sml_spectral_tables(self._h, ptr(sia), ptr(wt), ptr(cpol), ptr(nsh2)))
        return {"sia": sia, "wt": wt, "cpol": cpol, "nsh2": nsh2}

    # --- composite transforms
    def grid(self, spec, out=None, kcos: int = 1, stream=None):
        import torch

        nf = spec.shape[0]
        out = out if out is not None else torch.empty((nf, 48, 96), dtype=torch.float64, device=spec.device)
        _need_cuda(spec, out)
        check(lib().sml_grid_batched(self._h, ptr(spec), ptr(out), nf, kcos, stream_ptr(stream)))
        return out

    def spec(self, grid, out=None, stream=None):
        import torch

        nf = grid.shape[0]
        out = out if out is not None else torch.empty((nf, 32, 62), dtype=torch.float64, device=grid.device)
        _need_cuda(grid, out)
        check(lib().sml_spec_batched(self._h, ptr(grid), ptr(out), nf, stream_ptr(stream)))
        return out

    def vdspec(self, ug, vg, kcos: int = 2, stream=None):
        import torch

        nf = ug.shape[0]
        vor = torch.empty((nf, 32, 62), dtype=torch.float64, device=ug.device)
        div = torch.empty_like(vor)
        _need_cuda(ug, vg, vor, div)
        check(lib().sml_vdspec_batched(self._h, ptr(ug), ptr(vg), ptr(vor), ptr(div), nf, kcos, stream_ptr(stream)))
        return vor, div

    def uvspec(self, vor, div, stream=None):
        import torch

        nf = vor.shape[0]
        u = torch.empty_like(vor)
        v = torch.empty_like(vor)
        _need_cuda(vor, div, u, v)
        check(lib().sml_uvspec_batched(self._h, ptr(vor), ptr(div), ptr(u), ptr(v), nf, stream_ptr(stream)))
        return u, v

    # --- stages
    def gridy(self, spec, stream=None):
        import torch

        nf = spec.shape[0]
        out = torch.empty((nf, 48, 62), dtype=torch.float64, device=spec.device)
        _need_cuda(spec, out)
        check(lib().sml_gridy_batched(self._h, ptr(spec), ptr(out), nf, stream_ptr(stream)))
        return out

    def gridx(self, varm, kcos: int = 1, stream=None):
        import torch

        nf = varm.shape[0]
        out = torch.empty((nf, 48, 96), dtype=torch.float64, device=varm.device)
        _need_cuda(varm, out)
        check(lib().sml_gridx_batched(self._h, ptr(varm), ptr(out), nf, kcos, stream_ptr(stream)))
        return out

    def specx(self, grid, stream=None):
        import torch

        nf = grid.shape[0]
        out = torch.empty((nf, 48, 62), dtype=torch.float64, device=grid.device)
        _need_cuda(grid, out)
        check(lib().sml_specx_batched(self._h, ptr(grid), ptr(out), nf, stream_ptr(stream)))
        return out

    def specy(self, varm, stream=None):
        import torch

        nf = varm.shape[0]
        out = torch.empty((nf, 32, 62), dtype=torch.float64, device=varm.device)
        _need_cuda(varm, out)
        check(lib().sml_specy_batched(self._h, ptr(varm), ptr(out), nf, stream_ptr(stream)))
        return out

    # --- host convenience (synchronous)
    def grid_host(self, spec: np.ndarray, kcos: int = 1) -> np.ndarray:
        spec = np.ascontiguousarray(spec, dtype=np.float64).reshape(-1, 32, 62)
        out = np.zeros((spec.shape[0], 48, 96))
        check(lib().sml_grid_host(self._h, ptr(spec), ptr(out), spec.shape[0], kcos))
        return out

    def spec_host(self, grid: np.ndarray) -> np.ndarray:
        grid = np.ascontiguousarray(grid, dtype=np.float64).reshape(-1, 48, 96)
        out = np.zeros((grid.shape[0], 32, 62))
        check(lib().sml_spec_host(self._h, ptr(grid), ptr(out), grid.shape[0]))
        return out

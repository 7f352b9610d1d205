"""Batched reservoir forward + exchange tiling on the GPU (libspeedyml sml_res_*).

Host-side mirror of the reference's reservoir interface for one rank:
  Reservoirs(...)            <- initialize_model_parameters + processor_decomposition +
                                per-region trained_reservoir_prediction
                                (src/parallelmain.f90:30-199, src/mod_reservoir.f90:1781)
  .load_region(...)          <- read_trained_res + allocate_res_new + mklsparse
  .predict(fb, lm, out)      <- predict for every region of the rank (mod_reservoir.f90:1416)
  .assemble / .tile_inputs   <- sendrecievegrid's gather and scatter (mpires.f90:218-780)
Device buffers are torch CUDA tensors (plumbing only).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import SML_F32, SML_F64, check, lib, ptr, stream_ptr
from .domain import CHUNK_PRED, CHUNK_SPEEDY, NUM_REGIONS


class Reservoirs:
    """One rank's reservoirs on the GPU (sml_res_*).  With `ninp` and `out_index` given,
    a generic context (sml_res_create_generic: the slab-ocean reservoir's shape,
    ninp per region, outputs unstandardized with mean/std slot out_index[o])."""

    def __init__(self, region_ids, sst_flags, n, k, numregions: int = NUM_REGIONS,
                 chunk_speedy: int = CHUNK_SPEEDY, nout: int = CHUNK_PRED, weight_dtype: str = "f32",
                 leakage: float = 1.0, ninp=None, out_index=None):
        self.region_ids = np.ascontiguousarray(region_ids, dtype=np.int32)
        self.sst = np.ascontiguousarray(sst_flags, dtype=np.uint8)
        self.n = np.ascontiguousarray(n, dtype=np.int32)
        self.k = np.ascontiguousarray(k, dtype=np.int32)
        self.nlocal = len(self.region_ids)
        self.numregions = numregions
        self.ncs = chunk_speedy
        self.nout = nout
        self.weight_dtype = weight_dtype
        dt = {"f32": SML_F32, "f64": SML_F64}[weight_dtype]
        h = ctypes.c_void_p()
        if ninp is None:
            check(lib().sml_res_create(numregions, self.nlocal, ptr(self.region_ids), ptr(self.sst), ptr(self.n),
                                       ptr(self.k), chunk_speedy, nout, dt, leakage, ctypes.byref(h)))
        else:
            self._ninp = np.ascontiguousarray(ninp, dtype=np.int32)
            self._oidx = np.ascontiguousarray(out_index, dtype=np.int8)
            check(lib().sml_res_create_generic(numregions, self.nlocal, ptr(self.region_ids), ptr(self._ninp),
                                               ptr(self.n), ptr(self.k), chunk_speedy, nout, ptr(self._oidx), dt,
                                               leakage, ctypes.byref(h)))
        self._h = h
        off = np.zeros(self.nlocal + 1, dtype=np.int64)
        check(lib().sml_res_feedback_offsets(self._h, ptr(off)))
        self.fb_offsets = off

    def close(self):
        if getattr(self, "_h", None):
            lib().sml_res_destroy(self._h)
            self._h = None

    __del__ = close

    @property
    def handle(self):
        return self._h

    def ninp(self, i: int) -> int:
        v = ctypes.c_int()
        check(lib().sml_res_ninp(self._h, i, ctypes.byref(v)))
        return v.value

    def load_region(self, i: int, rows, cols, vals, win, wout, mean, std):
        """Reference layouts: rows/cols 1-based (k,), vals (k,), win (ninp, n) C-order,
        wout (ncs+n, nout) C-order, mean/std (36,)."""
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.int32)
        mean = np.ascontiguousarray(mean, dtype=np.float64)
        std = np.ascontiguousarray(std, dtype=np.float64)
        if vals.dtype == np.float32 and win.dtype == np.float32 and wout.dtype == np.float32:
            f = lib().sml_res_load_region_f32
            vals, win, wout = (np.ascontiguousarray(a, dtype=np.float32) for a in (vals, win, wout))
        else:
            f = lib().sml_res_load_region_f64
            vals, win, wout = (np.ascontiguousarray(a, dtype=np.float64) for a in (vals, win, wout))
        check(f(self._h, i, ptr(rows), ptr(cols), ptr(vals), ptr(win), ptr(wout), ptr(mean), ptr(std)))

    def load_region_weights(self, i: int, w):
        self.load_region(i, w.rows, w.cols, w.vals, w.win, w.wout, w.mean, w.std)

    def load_netcdf(self, i: int, path: str):
        """Load region i from a reference weight file (read_trained_res)."""
        d = read_region_netcdf(path)
        self.load_region(i, d["rows"], d["cols"], d["vals"], d["win"], d["wout"],
                         d["mean"].astype(np.float64), d["std"].astype(np.float64))

    def set_state(self, i: int, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        check(lib().sml_res_set_state(self._h, i, ptr(x)))

    def get_state(self, i: int) -> np.ndarray:
        x = np.zeros(int(self.n[i]))
        check(lib().sml_res_get_state(self._h, i, ptr(x)))
        return x

    # --- device buffers
    def alloc_io(self, device="cuda"):
        import torch

        fb = torch.zeros(int(self.fb_offsets[-1]), dtype=torch.float64, device=device)
        lm = torch.zeros((self.nlocal, max(self.ncs, 1)), dtype=torch.float64, device=device)
        ov = torch.zeros((self.nlocal, self.nout), dtype=torch.float64, device=device)
        return fb, lm, ov

    def predict(self, d_feedback, d_local_model, d_outvec, stream=None):
        check(lib().sml_res_step(self._h, ptr(d_feedback), ptr(d_local_model if self.ncs else None),
                                 ptr(d_outvec), stream_ptr(stream)))

    def predict_begin(self, d_feedback, stream=None):
        """First half of predict: the state update and W_out(:, ncs+1:) x~ (v_ml of
        outvec_component_contribs, mod_reservoir.f90:1456-1459) -- no local_model needed."""
        check(lib().sml_res_step_begin(self._h, ptr(d_feedback), stream_ptr(stream)))

    def predict_finish_grid(self, d_fc4d, d_fc2d, d_local_model, d_outvec, stream=None):
        """tile_local_model + predict_finish in one launch (same results); d_local_model
        (or None) also receives the tiled local-model vectors."""
        check(lib().sml_res_step_finish_grid(self._h, ptr(d_fc4d), ptr(d_fc2d), ptr(d_local_model), ptr(d_outvec),
                                             stream_ptr(stream)))

    def predict_finish_assemble(self, d_fc4d, d_fc2d, d_local_model, d_outvec, g4, g2, pr, stream=None):
        """predict_finish_grid + assemble(d_outvec, g4, g2, pr) in one launch (one rank
        holding every region in order; same results)."""
        check(lib().sml_res_step_finish_assemble(self._h, ptr(d_fc4d), ptr(d_fc2d), ptr(d_local_model),
                                                 ptr(d_outvec), ptr(g4), ptr(g2), ptr(pr), stream_ptr(stream)))

    def set_read_waves(self, waves: int):
        """Cap on the v_ml readout's waves in predict_begin (0 = uncapped)."""
        check(lib().sml_res_set_read_waves(self._h, int(waves)))

    def set_update_cus(self, cus: int):
        """The CUs this context's launches get (sml_res_set_update_cus; 0 = the device)."""
        check(lib().sml_res_set_update_cus(self._h, int(cus)))

    def update_balanced(self) -> bool:
        """Whether the state update runs as k_res_update_bal (sml_res_update_balanced)."""
        b = ctypes.c_int()
        check(lib().sml_res_update_balanced(self._h, ctypes.byref(b)))
        return bool(b.value)

    def ell_layout(self, i: int) -> dict:
        """Local region i's compressed A / W_in form (sml_res_ell_layout)."""
        v = [ctypes.c_int() for _ in range(4)]
        check(lib().sml_res_ell_layout(self._h, int(i), *[ctypes.byref(x) for x in v]))
        return dict(a_width=v[0].value, a_overflow=bool(v[1].value), win_q=v[2].value, win_ell=bool(v[3].value))

    def set_reference_paths(self, csr: bool = False, per_region: bool = False, ungrouped_finish: bool = False):
        """Force the fallback paths for every region (sml_res_set_reference_paths): A /
        W_in from their CSR copies (before any region is loaded), the per-region state
        update, the v_p finish one thread per output -- bitwise the defaults."""
        flags = (1 if csr else 0) | (2 if per_region else 0) | (4 if ungrouped_finish else 0)
        check(lib().sml_res_set_reference_paths(self._h, flags))

    def set_begin_mode(self, mode: int):
        """predict_begin's form: 0 update grid + readout grid, 1 / 2 one fused launch
        (sml_res_set_begin_mode); bit-identical results."""
        check(lib().sml_res_set_begin_mode(self._h, int(mode)))

    @property
    def begin_fused(self) -> bool:
        """Whether predict_begin runs as the fused launch (the mode and this context's shapes)."""
        f = ctypes.c_int()
        check(lib().sml_res_begin_fused(self._h, ctypes.byref(f)))
        return bool(f.value)

    def predict_finish(self, d_local_model, d_outvec, stream=None):
        """Second half: outvec = W_out(:, 1:ncs) local_model + v_ml, unstandardized."""
        check(lib().sml_res_step_finish(self._h, ptr(d_local_model if self.ncs else None), ptr(d_outvec),
                                        stream_ptr(stream)))

    def synchronize(self, d_inputs, length: int, stride: int | None = None, stream=None):
        """synchronize (mod_reservoir.f90:1352-1378): `length` state updates, no
        readout.  d_inputs: device tensor of `length` packed feedback blocks
        (row t = block t, stride = total feedback doubles unless given)."""
        stride = int(self.fb_offsets[-1]) if stride is None else int(stride)
        if d_inputs.numel() < length * stride:
            raise ValueError("d_inputs holds fewer than length * stride doubles")
        check(lib().sml_res_synchronize(self._h, ptr(d_inputs), length, stride, stream_ptr(stream)))

    def start_prediction(self, d_inputs, length: int, d_feedback, stride: int | None = None, stream=None):
        """start_prediction (mod_reservoir.f90:938-959): synchronize_print over the first
        `length` input blocks, block `length` into d_feedback."""
        stride = int(self.fb_offsets[-1]) if stride is None else stride
        check(lib().sml_res_start_prediction(self._h, ptr(d_inputs), length, stride, ptr(d_feedback),
                                             stream_ptr(stream)))

    def predict_slab(self, d_feedback, d_local_model, d_local_model_next, d_outvec, stream=None):
        """predict_slab (mod_slab_ocean_reservoir.f90:1201-1249) on a generic context:
        outvec unstandardized, the raw outvec into d_local_model_next."""
        check(lib().sml_res_step_slab(self._h, ptr(d_feedback), ptr(d_local_model), ptr(d_local_model_next),
                                      ptr(d_outvec), stream_ptr(stream)))

    def predict_host(self, feedback: np.ndarray, local_model: np.ndarray | None) -> np.ndarray:
        fb = np.ascontiguousarray(feedback, dtype=np.float64)
        lm = np.ascontiguousarray(local_model, dtype=np.float64) if local_model is not None else None
        out = np.zeros((self.nlocal, self.nout))
        check(lib().sml_res_step_host(self._h, ptr(fb), ptr(lm), ptr(out)))
        return out

    def assemble(self, d_outvec_all, d_g4, d_g2, d_pr, stream=None):
        check(lib().sml_exchange_assemble(self._h, ptr(d_outvec_all), ptr(d_g4), ptr(d_g2), ptr(d_pr),
                                          stream_ptr(stream)))

    def tile_inputs(self, d_g4, d_g2, d_pr, d_fc4, d_fc2, d_tisr, d_feedback, d_local_model, stream=None):
        check(lib().sml_res_tile_inputs(self._h, ptr(d_g4), ptr(d_g2), ptr(d_pr), ptr(d_fc4), ptr(d_fc2),
                                        ptr(d_tisr), ptr(d_feedback), ptr(d_local_model), stream_ptr(stream)))

    def tile_feedback(self, d_g4, d_g2, d_pr, d_tisr, d_feedback, stream=None):
        check(lib().sml_res_tile_feedback(self._h, ptr(d_g4), ptr(d_g2), ptr(d_pr), ptr(d_tisr), ptr(d_feedback),
                                          stream_ptr(stream)))

    def tile_local_model(self, d_fc4, d_fc2, d_local_model, stream=None):
        check(lib().sml_res_tile_local_model(self._h, ptr(d_fc4), ptr(d_fc2), ptr(d_local_model),
                                             stream_ptr(stream)))

    # --- measurement
    def footprint(self):
        w = ctypes.c_int64()
        a = ctypes.c_int64()
        check(lib().sml_res_footprint(self._h, ctypes.byref(w), ctypes.byref(a)))
        return w.value, a.value

    def enable_timing(self, capacity: int):
        check(lib().sml_res_enable_timing(self._h, capacity))

    def kernel_times(self, max_steps: int = 100000):
        upd = np.zeros(max_steps, dtype=np.float32)
        rd = np.zeros(max_steps, dtype=np.float32)
        cnt = ctypes.c_int()
        check(lib().sml_res_kernel_times(self._h, ptr(upd), ptr(rd), max_steps, ctypes.byref(cnt)))
        return upd[:cnt.value].astype(np.float64), rd[:cnt.value].astype(np.float64)


def read_region_netcdf(path: str) -> dict:
    """Read a worker_XXXX_level_1_<trial>.nc weight file (read_trained_res layout)."""
    dims = np.zeros(6, dtype=np.int64)
    p = os.fsencode(path)
    check(lib().sml_nc_read_region(p, ptr(dims), None, None, None, None, None, None, None))
    n, ninp, nout, ncsn, k, nms = (int(v) for v in dims)
    out = {
        "win": np.zeros((ninp, n), dtype=np.float32),
        "wout": np.zeros((ncsn, nout), dtype=np.float32),
        "rows": np.zeros(k, dtype=np.int32),
        "cols": np.zeros(k, dtype=np.int32),
        "vals": np.zeros(k, dtype=np.float32),
        "mean": np.zeros(nms, dtype=np.float32),
        "std": np.zeros(nms, dtype=np.float32),
    }
    check(lib().sml_nc_read_region(p, ptr(dims), ptr(out["win"]), ptr(out["wout"]), ptr(out["rows"]),
                                   ptr(out["cols"]), ptr(out["vals"]), ptr(out["mean"]), ptr(out["std"])))
    return out


def write_region_netcdf(path: str, win, wout, rows, cols, vals, mean, std) -> None:
    """Write the reference's per-region weight layout (write_trained_res), CDF-1."""
    win = np.ascontiguousarray(win, dtype=np.float32)
    wout = np.ascontiguousarray(wout, dtype=np.float32)
    ninp, n = win.shape
    ncsn, nout = wout.shape
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    mean = np.ascontiguousarray(mean, dtype=np.float32)
    std = np.ascontiguousarray(std, dtype=np.float32)
    check(lib().sml_nc_write_region(os.fsencode(path), n, ninp, nout, ncsn, len(rows), ptr(win), ptr(wout),
                                    ptr(rows), ptr(cols), ptr(vals), ptr(mean), ptr(std)))

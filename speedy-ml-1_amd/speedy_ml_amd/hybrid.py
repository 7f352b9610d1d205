"""The hybrid prediction loop on one rank: reservoir predict for the rank's regions,
the outvec exchange, SPEEDY's run_model on the assembled grid, and the re-tiling of
the next step's inputs.

Reference: the time loop of src/parallelmain.f90:204-270 -- `predict` per region
(:225-234), then `sendrecievegrid` (src/mpires.f90:218-780), which gathers every
outvec at the root, assembles the global grid (:300-478), runs SPEEDY on it
(`run_model`, :1516-1628: iogrid(30) + safety check, stepone + 24 leapfrog steps,
iogrid(31), q floor), scatters the next feedback tiles and SPEEDY local vectors
(:558-751) and broadcasts `run_speedy` (:721); the loop ends when it is false
(:268-270).

The loop itself is native (csrc/sml_hybrid.hip, `sml_hybrid_*` in
include/speedy_ml.h): the Fortran host drives the same entry points.  This class
owns the device buffers (torch tensors: plumbing only) and supplies the exchange
between the two halves of a step: `predict` leaves the local outvecs on the loop's
main stream, `exchange` (speedy_ml_amd.exchange: torch.distributed all-gather, RCCL
over xGMI when world > 1) runs on that stream, `advance` takes every region's
outvecs.  With a NativeComm (speedy_ml_amd.comm) the exchange is the library's own
ncclAllGather on the main stream instead (sml_hybrid_step).

Schedule (overlap=True): the reservoir's update and ~98 % of
its readout bytes run on the main stream while SPEEDY integrates the previous
step's window on the side stream, on disjoint CUs (`speedy_cus`, default 64:
SPEEDY on CUs [0, 64), the reservoir on the rest); results are identical to the
one-stream schedule (overlap=False, one-pass readout).
"""
from __future__ import annotations

import ctypes
import os

import torch

from ._lib import check, lib, ptr
from .dynamics import ALPH, DELT, ROB, WIL


class HybridLoop:
    """res: Reservoirs (this rank's regions), dyn: Dynamics with state, forcing and
    physics set, exchange: OutvecExchange (or any callable [nlocal, nout] ->
    [numregions, nout] run on the current stream), tisr: [nlocal, 16] standardized
    tisr inputs (device) or None (feedback tisr entries left as they are)."""

    def __init__(self, res, dyn, exchange, device, tisr=None, overlap: bool = True, nleap: int = 24,
                 speedy_cus: int | None = None, delt: float = DELT, comm=None, slab=None):
        """slab: None, or a SlabOcean (the slab-ocean reservoirs of this rank's sst
        regions and the sst grids; sml_hybrid_set_slab) -- the exchange rows then carry
        each region's slab sst beside its outvec (`ov` is [nlocal, exchange_width])."""
        self.res, self.dyn, self.exchange, self.tisr, self.comm = res, dyn, exchange, tisr, comm
        self.overlap, self.nleap, self.slab = overlap, nleap, slab
        self.dev = torch.device(device)
        self.fb, self.lm, self.ov = res.alloc_io(self.dev)
        z = lambda *s: torch.zeros(s, dtype=torch.float64, device=self.dev)  # noqa: E731
        # variables3d(4, 96, 48, 8) / logp(96, 48) / precip(96, 48) in Fortran order
        self.g4, self.g2, self.pr = z(8, 48, 96, 4), z(48, 96), z(48, 96)
        self.f4, self.f2 = z(8, 48, 96, 4), z(48, 96)
        if speedy_cus is None:
            speedy_cus = int(os.environ.get("SML_SPEEDY_CUS", "64"))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.dev):
            check(lib().sml_hybrid_create(res.handle, dyn._h, comm.handle if comm is not None else None, nleap, delt,
                                          ALPH, ROB, WIL, int(overlap),
                                          int(speedy_cus if overlap else 0), ctypes.byref(h)))
        self._h = h
        if slab is not None:
            check(lib().sml_hybrid_set_slab(h, slab.res.handle, ptr(slab.base_sst), ptr(slab.sea_mask),
                                            int(slab.timestep), int(slab.timestep_slab), float(slab.sst_bias)))
            w = ctypes.c_int()
            check(lib().sml_hybrid_exchange_width(h, ctypes.byref(w)))
            self.ov = torch.zeros((res.nlocal, w.value), dtype=torch.float64, device=self.dev)
        self.exchange_width = int(self.ov.shape[1])
        check(lib().sml_hybrid_set_buffers(h, ptr(self.fb), ptr(self.lm if res.ncs else None), ptr(self.ov),
                                           ptr(self.g4), ptr(self.g2), ptr(self.pr), ptr(self.f4), ptr(self.f2),
                                           ptr(tisr)))
        m, s = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().sml_hybrid_streams(h, ctypes.byref(m), ctypes.byref(s)))
        self.main = torch.cuda.ExternalStream(m.value, device=self.dev)
        self.side = torch.cuda.ExternalStream(s.value, device=self.dev) if s.value != m.value else self.main
        sc, rc = ctypes.c_int(), ctypes.c_int()
        check(lib().sml_hybrid_cus(h, ctypes.byref(sc), ctypes.byref(rc)))
        self.speedy_cus, self.res_cus = sc.value, rc.value  # the CU split (0, 0: none)
        self._set_xstream()

    def _set_xstream(self):
        """The stream the local outvecs are ready on after predict (sml_hybrid_exchange_stream)."""
        x = ctypes.c_void_p()
        check(lib().sml_hybrid_exchange_stream(self._h, ctypes.byref(x)))
        self.xstream = self.side if x.value == self.side.cuda_stream else self.main

    def set_chain(self, mode: int):
        """SML_CHAIN_AUTO / SML_CHAIN_TWO_STREAMS / SML_CHAIN_SPEEDY (include/speedy_ml.h):
        where the finish -> exchange -> assembly -> tiling chain runs."""
        check(lib().sml_hybrid_set_chain(self._h, int(mode)))
        self._set_xstream()

    def chain(self):
        """(requested, effective) chain mode."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(lib().sml_hybrid_chain(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def close(self):
        """Wait for the loop's work and release its streams."""
        if getattr(self, "_h", None):
            check(lib().sml_hybrid_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tisr(self, tisr):
        """tisr inputs of the next steps (get_tisr_by_date, mpires.f90:1644-1676)."""
        self.tisr = tisr
        check(lib().sml_hybrid_set_tisr(self._h, ptr(tisr)))

    def set_tisr_table(self, table, startyear: int, hours_base: int, step_hours: int = 6):
        """get_tisr_by_date (mpires.f90:1644-1676): hourly global tisr fields
        `table` [nhours, 48, 96] (device), the calendar's start year and the hours
        before the first prediction step (traininglength + prediction marker +
        synclength in the reference); None switches back to the fixed tisr."""
        self._tisr_table = table
        n = 0 if table is None else int(table.shape[0])
        check(lib().sml_hybrid_set_tisr_table(self._h, ptr(table), n, int(startyear), int(hours_base),
                                              int(step_hours)))

    def set_hop_timeout(self, microseconds: int):
        """Give-up time of the loop's in-kernel waits (sml_hybrid_set_hop_timeout)."""
        check(lib().sml_hybrid_set_hop_timeout(self._h, int(microseconds)))

    def set_calendar(self, startyear: int, hours_base: int, step_hours: int = 6):
        """run_model's calendar (mpires.f90:1545): every advance t hands the window the
        date of hour hours_base + t * step_hours and refreshes its forcing at that date
        (Dynamics.fordate; the Dynamics needs set_surface).  Shared with the tisr table's."""
        check(lib().sml_hybrid_set_calendar(self._h, int(startyear), int(hours_base), int(step_hours)))

    def window_date(self):
        """(year, month, day, hour) of the next advance's window."""
        d = (ctypes.c_int * 4)()
        check(lib().sml_hybrid_window_date(self._h, d))
        return tuple(d)

    def start(self, g4, g2, pr, f4, f2):
        """start_prediction analogue: inputs of the first step from an analysis grid
        (g4, g2, pr) and a SPEEDY forecast from it (f4, f2)."""
        check(lib().sml_hybrid_start(self._h, ptr(g4), ptr(g2), ptr(pr), ptr(f4), ptr(f2)))

    def step(self):
        """One hybrid time step (asynchronous; `sync()` waits for it).  With a
        NativeComm (speedy_ml_amd.comm) the whole step is native, its all-gather on
        the main stream (sml_hybrid_step); else `exchange` runs between predict and
        advance."""
        # one rank whose exchange is the identity (OutvecExchange of world 1): the native
        # step too, whose finish then assembles the grids in the same launch
        identity = self.comm is None and getattr(self.exchange, "world", None) == 1
        if self.comm is not None or identity:  # a LocalRank at world > 1 is refused: no transport
            check(lib().sml_hybrid_step(self._h))
            return
        check(lib().sml_hybrid_predict(self._h))
        with torch.cuda.stream(self.xstream):
            glob = self.exchange(self.ov)  # RCCL all-gather over xGMI when world > 1
        check(lib().sml_hybrid_advance(self._h, ptr(glob)))

    def start_slab(self, slab_outvec):
        """start_prediction_slab's hand-over: the slab reservoirs' sst [nslab, 4]
        (device) until their first prediction (sml_hybrid_start_slab)."""
        check(lib().sml_hybrid_start_slab(self._h, ptr(slab_outvec)))

    def slab_state(self):
        """Host copies of the loop's slab state (after its work completes):
        wholegrid_sst [48, 96], the ring [ratio - 1, tot], the last slab feedback [tot]
        and slab outvecs [nslab, 4]."""
        import numpy as np

        sst, ring, fb, ov = (ctypes.c_void_p() for _ in range(4))
        n = ctypes.c_int()
        check(lib().sml_hybrid_slab_buffers(self._h, ctypes.byref(sst), ctypes.byref(ring), ctypes.byref(n),
                                            ctypes.byref(fb), ctypes.byref(ov)))
        sl = self.slab
        ratio = sl.timestep_slab // sl.timestep
        out = {"sst": np.zeros((48, 96)), "ring": np.zeros((ratio - 1, n.value)), "feedback": np.zeros(n.value),
               "outvec": np.zeros((sl.res.nlocal, 4))}
        for key, src in (("sst", sst), ("ring", ring), ("feedback", fb), ("outvec", ov)):
            a = out[key]
            if a.size:
                check(lib().sml_copy_to_host(ptr(a), src, a.nbytes))
        return out

    def predict(self):
        """First half of a step: this rank's outvecs into `ov` (on `xstream`)."""
        check(lib().sml_hybrid_predict(self._h))

    def advance_slabs(self, recv):
        """Second half from an all-gather's output recv [world * maxc, nout] (device;
        every rank's `ov` zero-padded to maxc, comm.exchange_plan), permuted into
        region order when the shares are uneven (sml_hybrid_advance_slabs)."""
        check(lib().sml_hybrid_advance_slabs(self._h, ptr(recv)))

    def set_pipelined(self, on: bool = True):
        """Each step also issues the next step's reservoir begin (sml_hybrid_set_pipelined):
        the same outvecs, grids and forecasts; the reservoir states run one update ahead."""
        check(lib().sml_hybrid_set_pipelined(self._h, 1 if on else 0))

    def set_force_exchange(self, on: bool = True):
        """With a NativeComm at world 1: run the world > 1 exchange path anyway (send
        slab -> ncclAllGather -> advance from the receive slab; sml_hybrid_set_force_exchange)."""
        check(lib().sml_hybrid_set_force_exchange(self._h, 1 if on else 0))

    def exchanges(self) -> int:
        """ncclAllGather calls the native step has issued (sml_hybrid_exchanges)."""
        n = ctypes.c_int64()
        check(lib().sml_hybrid_exchanges(self._h, ctypes.byref(n)))
        return n.value

    def set_hop_mode(self, mode: int):
        """SML_HOP_AUTO / SML_HOP_WAIT_VALUE / SML_HOP_EVENTS / SML_HOP_KERNEL (include/speedy_ml.h)."""
        check(lib().sml_hybrid_set_hop_mode(self._h, int(mode)))

    def hop_mode(self):
        """(requested, effective) hop mode."""
        a, b = ctypes.c_int(), ctypes.c_int()
        check(lib().sml_hybrid_hop_mode(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def run_speedy(self) -> bool:
        """run_speedy of the last step: False when its window entry failed iogrid(30)'s
        safety check -- the reference ends the prediction there."""
        r = ctypes.c_int()
        check(lib().sml_hybrid_run_speedy(self._h, ctypes.byref(r)))
        return bool(r.value)

    def sync(self):
        check(lib().sml_hybrid_sync(self._h))


class SlabOcean:
    """The slab-ocean side of the loop (parallelmain.f90:216-249): `res`, a generic
    ML-only Reservoirs over this rank's sst regions (7 * in2d inputs each, 4 sst
    outputs, out_index 35); base_sst / sea_mask [48, 96] device tensors
    (model_parameters%base_sst_grid / sea_mask, mod_reservoir.f90:845-883); the
    timesteps in hours (mod_reservoir.f90:36-37: 6 and 168) and current_sst_bias."""

    def __init__(self, res, base_sst, sea_mask, timestep: int = 6, timestep_slab: int = 168, sst_bias: float = 0.0):
        self.res, self.base_sst, self.sea_mask = res, base_sst, sea_mask
        self.timestep, self.timestep_slab, self.sst_bias = timestep, timestep_slab, sst_bias

